#!/bin/bash
# round 3 validation: the whole -m gpu suite, smoke(), the driver's bench command.
# A timeout / crash ends the script (no further GPU work after it).
cd "${GRAFT_REPO_ROOT:-.}"
out=gpurun_out/r3full
mkdir -p $out
timeout -k 10 900 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests > $out/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $out/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 $out/smoke.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 --detail $out/bench_detail.json > $out/bench.out 2> $out/bench.err
rc=$?; echo "bench rc=$rc"; wc -c $out/bench.out
