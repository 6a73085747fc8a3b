# round 5: the 64 B ring's table fill (probe_tabfill), then the backend legs (r5f)
set -o pipefail
mkdir -p gpurun_out/r5g
timeout -k 10 120 scripts/probe_tabfill > gpurun_out/r5g/tabfill.log 2>&1; rc=$?
cat gpurun_out/r5g/tabfill.log; [ $rc -ne 0 ] && exit $rc
bash scripts/runs/gpu_r5f.sh
