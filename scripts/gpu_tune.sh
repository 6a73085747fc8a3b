mkdir -p gpurun_out
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O2 -o /tmp/probe_rangecheck scripts/probe_rangecheck.hip 2>/dev/null && timeout -k 10 60 /tmp/probe_rangecheck > gpurun_out/probe.log 2>&1; echo "probe rc=$?"; cat gpurun_out/probe.log
timeout -k 10 300 python scripts/tune.py > gpurun_out/tune.log 2>&1; rc=$?; echo "tune rc=$rc"; cat gpurun_out/tune.log
exit $rc
