# two header waves per stream tile (scripts/probe_h2.h) at ring size and batch size, IMIX
set -o pipefail
mkdir -p gpurun_out/probe
timeout -k 10 150 scripts/probe_timeline 3 2097152 2 2 > gpurun_out/probe/h2_ring_imix.log 2>&1; rc=$?
echo "ring rc=$rc"; sed -n 2,20p gpurun_out/probe/h2_ring_imix.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 150 scripts/probe_timeline 3 262144 6 2 > gpurun_out/probe/h2_imix.log 2>&1; rc=$?
echo "single rc=$rc"; sed -n 2,20p gpurun_out/probe/h2_imix.log
exit $rc
