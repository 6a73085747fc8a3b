# SMALL tile size for one 32K-frame 64 B batch per launch
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 100 ./scripts/probe_classify 1 32768 > gpurun_out/probe_small.log 2>&1; rc=$?
cat gpurun_out/probe_small.log
exit $rc
