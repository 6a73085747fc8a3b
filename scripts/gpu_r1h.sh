# stream shapes: parity first, then timing against LARGE
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout=120 --timeout-method thread -p no:cacheprovider -k "stream or forced or flow_hash_device" > gpurun_out/pytest_h.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_h.log
[ $rc -ne 0 ] && exit $rc
TUNE_VARIANTS=2,30,34,38,42,46,50 TUNE_ROUNDS=3 TUNE_BW=0 TUNE_SCALE=0 timeout -k 10 300 python -u scripts/tune.py > gpurun_out/tune_stream.log 2>&1; rc=$?
echo "tune rc=$rc"; cat gpurun_out/tune_stream.log
exit $rc
