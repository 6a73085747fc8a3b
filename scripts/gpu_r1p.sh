# register-lean SMALL tile + whole-window datagrams: full parity, then bench (device legs)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout=120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_p.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_p.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --no-cpu --no-e2e > gpurun_out/bench_p.log 2>&1; rc=$?
echo "bench rc=$rc"; grep "^\[bench\]" gpurun_out/bench_p.log
exit $rc
