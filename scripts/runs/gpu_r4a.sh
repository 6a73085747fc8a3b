#!/bin/bash
# round 4 first GPU pass: the new tests (groups with filters, async sets, compact
# records, consumer scenarios), then the whole -m gpu suite and smoke().
# A timeout / crash ends the script (no further GPU work after it).
cd "${GRAFT_REPO_ROOT:-.}"
out=gpurun_out/r4a
mkdir -p $out
timeout -k 10 600 python -u -m pytest -v --maxfail=20 --timeout 120 --timeout-method thread -m gpu \
    tests/test_bpf_groups.py tests/test_mos_consumer.py > $out/pytest_new.log 2>&1
rc=$?; echo "pytest(new) rc=$rc"; tail -3 $out/pytest_new.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 900 python -u -m pytest -v --maxfail=20 --timeout 120 --timeout-method thread -m gpu tests \
    > $out/pytest_full.log 2>&1
rc=$?; echo "pytest(full) rc=$rc"; tail -3 $out/pytest_full.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 $out/smoke.log
exit $rc
