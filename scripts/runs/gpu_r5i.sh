# round 5: the whole -m gpu suite after the compact / hint / stream changes
set -o pipefail
mkdir -p gpurun_out/r5i
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/r5i/pytest.log 2>&1; rc=$?
tail -5 gpurun_out/r5i/pytest.log
exit $rc
