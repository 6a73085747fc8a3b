# timeline + bound probes on the current kernels (scripts/probe_timeline, built here); logs under gpurun_out/probe
set -o pipefail
mkdir -p gpurun_out/probe
timeout -k 10 120 scripts/probe_timeline 3 262144 6 > gpurun_out/probe/timeline_imix.log 2>&1; rc=$?
echo "imix rc=$rc"; head -20 gpurun_out/probe/timeline_imix.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 scripts/probe_timeline 1 8388608 2 4 > gpurun_out/probe/small_bound_8M.log 2>&1; rc=$?
echo "s64 8M rc=$rc"; cat gpurun_out/probe/small_bound_8M.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 scripts/probe_timeline 1 32768 40 4 > gpurun_out/probe/small_bound_32K.log 2>&1; rc=$?
echo "s64 32K rc=$rc"; cat gpurun_out/probe/small_bound_32K.log
exit $rc
