# BPF engines: parity (golden + random programs) and the JIT kernel's trace
set -o pipefail
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_bpf.py -m gpu -x -q --timeout=120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_y.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_y.log
[ $rc -ne 0 ] && exit $rc
W=IMIX_bpf
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/kt_$W -o kt --output-format csv -- python3 bench.py --workloads $W --streams 1 --no-cpu --no-e2e > gpurun_out/prof/kt_$W.log 2>&1; rc=$?
echo "kt $W rc=$rc"; grep "^\[bench\]" gpurun_out/prof/kt_$W.log; head -3 gpurun_out/prof/kt_$W/kt_kernel_stats.csv
exit $rc
