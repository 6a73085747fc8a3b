# header-parse change: full parity, then device-leg bench of the header-heavy workloads
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout=120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_s.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_s.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --workloads M1500,IMIX,S64,S64_queue --no-cpu --no-e2e > gpurun_out/bench_s.log 2>&1; rc=$?
echo "bench rc=$rc"; grep "^\[bench\]" gpurun_out/bench_s.log
exit $rc
