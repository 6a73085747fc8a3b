mkdir -p gpurun_out
timeout -k 10 60 ./scripts/probe_rangecheck > gpurun_out/probe.log 2>&1; echo "probe rc=$?"; cat gpurun_out/probe.log
bash scripts/gpu_iter.sh
