# session-2 re-check: full GPU parity, batch-size scaling T(n)=a+bn, default bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout=120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_g.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_g.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_g.log 2>&1; rc=$?
echo "smoke rc=$rc"; tail -2 gpurun_out/smoke_g.log
[ $rc -ne 0 ] && exit $rc
TUNE_VARIANTS=2 TUNE_ROUNDS=3 TUNE_BW=1 TUNE_SCALE=1 timeout -k 10 300 python -u scripts/tune.py > gpurun_out/tune_scale.log 2>&1; rc=$?
echo "tune rc=$rc"; cat gpurun_out/tune_scale.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u bench.py > gpurun_out/bench_g.log 2>&1; rc=$?
echo "bench rc=$rc"; grep "^\[bench\]" gpurun_out/bench_g.log; tail -c 600 gpurun_out/bench_g.log
exit $rc
