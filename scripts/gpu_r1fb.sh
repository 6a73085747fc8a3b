# fused classify + BPF: parity (all BPF tests), then bench of the BPF rows
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout=120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_fb.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_fb.log; grep -E "FAILED|Error" gpurun_out/pytest_fb.log | head -5
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --workloads IMIX,IMIX_bpf,IMIX_cls_bpf --no-cpu --no-e2e > gpurun_out/bench_fb.log 2>&1; rc=$?
echo "bench rc=$rc"; grep "^\[bench\]" gpurun_out/bench_fb.log
exit $rc
