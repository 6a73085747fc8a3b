# BPF kernel: programs split across the waves of a 64-frame tile
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_bpf.py -m gpu -x -q --timeout=120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_t.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_t.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --workloads IMIX_bpf --no-cpu --no-e2e > gpurun_out/bench_t.log 2>&1; rc=$?
echo "bench rc=$rc"; grep "^\[bench\]" gpurun_out/bench_t.log
exit $rc
