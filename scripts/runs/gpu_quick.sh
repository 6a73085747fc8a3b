# quick iteration: GPU parity tests, then 1-stream bench lines of the main workloads (no CPU/e2e legs)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --workloads ${W:-M1500,IMIX,S64,S64_queue,M1500_queue,IMIX_cls_bpf} --no-cpu --no-e2e > gpurun_out/bench_quick.log 2>&1; rc=$?
grep "^\[bench\]" gpurun_out/bench_quick.log
exit $rc
