# stream_scan (H=1 prefix-scan streamer): parity, then time shares
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout=120 --timeout-method thread -p no:cacheprovider -k "stream or forced or flow_hash_device or tx_forced" > gpurun_out/pytest_j.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_j.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 100 ./scripts/probe_classify 2 65536 > gpurun_out/probe_classify5.log 2>&1 && timeout -k 10 100 ./scripts/probe_classify 3 262144 >> gpurun_out/probe_classify5.log 2>&1 && timeout -k 10 100 ./scripts/probe_classify 1 32768 >> gpurun_out/probe_classify5.log 2>&1; rc=$?
cat gpurun_out/probe_classify5.log
exit $rc
