#!/bin/bash
# round 4: the real-clock consumer scenario, async vs synchronous filter install
# (the cause of round 3's seed-7 soak failure), and the async set's timings.
cd "${GRAFT_REPO_ROOT:-.}"
out=gpurun_out/r4b
mkdir -p $out
timeout -k 10 300 python -u scripts/repro_real_clock.py gpu 3 > $out/real_clock.log 2>&1
rc=$?; echo "repro rc=$rc"; cat $out/real_clock.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u -m pytest -s -v --timeout 120 --timeout-method thread -m gpu \
    tests/test_bpf_groups.py -k "async or back_to_back" > $out/async.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "set_async|passed|failed" $out/async.log
exit $rc
