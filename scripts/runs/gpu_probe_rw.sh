# read+write streaming rate at the classify rows' read:write mixes (scripts/probe_rw)
set -o pipefail
mkdir -p gpurun_out/probe
timeout -k 10 120 scripts/probe_rw 648 2 > gpurun_out/probe/rw_648.log 2>&1 || exit $?
timeout -k 10 120 scripts/probe_rw 128 8 > gpurun_out/probe/rw_128.log 2>&1 || exit $?
cat gpurun_out/probe/rw_648.log gpurun_out/probe/rw_128.log
