# stream-tile time shares (scripts/probe_classify.hip), 1500 B and IMIX
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 100 ./scripts/probe_classify 2 65536 > gpurun_out/probe.log 2>&1 && timeout -k 10 100 ./scripts/probe_classify 3 262144 >> gpurun_out/probe.log 2>&1; rc=$?
cat gpurun_out/probe.log
exit $rc
