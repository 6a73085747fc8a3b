# parity tests, variant A/B (unrolled LARGE vs MID vs forced kinds), stream sweep
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests -m gpu -q -x --timeout=120 -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
TUNE_VARIANTS=2,10,14 TUNE_ROUNDS=3 TUNE_BW=1 TUNE_SCALE=0 timeout -k 10 300 python scripts/tune.py > gpurun_out/tune.log 2>&1; rc=$?
echo "tune rc=$rc"; tail -30 gpurun_out/tune.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python scripts/tune_streams.py > gpurun_out/streams.log 2>&1; rc=$?
echo "streams rc=$rc"; cat gpurun_out/streams.log
exit $rc
