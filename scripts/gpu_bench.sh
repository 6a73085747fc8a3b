# The driver's bench command and the default one, logs under gpurun_out/
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_driver.log 2>&1; rc=$?
echo "driver-style bench rc=$rc"; grep "^\[bench\]" gpurun_out/bench_driver.log; [ $rc -ne 0 ] && { tail -20 gpurun_out/bench_driver.log; exit $rc; }
timeout -k 10 500 python -u bench.py ${ARGS:-} > gpurun_out/bench_default.log 2>&1; rc=$?
echo "default bench rc=$rc"; grep "^\[bench\]" gpurun_out/bench_default.log
exit $rc
