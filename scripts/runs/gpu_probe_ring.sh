# stream-tile variants on ring-sized single launches (2M IMIX frames, 512K 1500 B frames), scripts/probe_timeline
set -o pipefail
mkdir -p gpurun_out/probe
timeout -k 10 150 scripts/probe_timeline 3 2097152 2 > gpurun_out/probe/ring_imix.log 2>&1; rc=$?
echo "imix rc=$rc"; head -14 gpurun_out/probe/ring_imix.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 150 scripts/probe_timeline 2 524288 2 > gpurun_out/probe/ring_m1500.log 2>&1; rc=$?
echo "m1500 rc=$rc"; head -14 gpurun_out/probe/ring_m1500.log
exit $rc
