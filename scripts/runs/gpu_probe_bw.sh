mkdir -p gpurun_out
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -o /tmp/probe_bw scripts/probe_bw.hip 2>/dev/null && timeout -k 10 120 /tmp/probe_bw > gpurun_out/probe_bw.log 2>&1; rc=$?; echo "probe_bw rc=$rc"; cat gpurun_out/probe_bw.log
exit $rc
