# full GPU parity suite, smoke, then 1-stream bench lines of the main rows; logs under gpurun_out/
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -4 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?
cat gpurun_out/smoke.log | tail -3; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --workloads ${W:-M1500,IMIX,S64,M1500_1,IMIX_1,S64_1} --no-cpu --no-e2e > gpurun_out/bench_quick.log 2>&1; rc=$?
grep "^\[bench\]" gpurun_out/bench_quick.log
exit $rc
