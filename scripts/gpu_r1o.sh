# 54-VGPR stream tiles (lean unsorted path): parity, then timing incl. unsorted descriptors
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout=120 --timeout-method thread -p no:cacheprovider -k "stream or config or forced" > gpurun_out/pytest_o.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_o.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 100 ./scripts/probe_classify 2 65536 > gpurun_out/probe_sb.log 2>&1 && timeout -k 10 100 ./scripts/probe_classify 3 262144 >> gpurun_out/probe_sb.log 2>&1; rc=$?
cat gpurun_out/probe_sb.log
exit $rc
