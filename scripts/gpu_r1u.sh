# 1500 B batch queue (4 batches per launch): parity, bench lines
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout=120 --timeout-method thread -p no:cacheprovider -k "queue" > gpurun_out/pytest_u.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_u.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --workloads M1500,M1500_queue,S64_queue --no-cpu --no-e2e > gpurun_out/bench_u.log 2>&1; rc=$?
echo "bench rc=$rc"; grep "^\[bench\]" gpurun_out/bench_u.log
exit $rc
