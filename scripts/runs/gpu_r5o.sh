# round 5: backend soak with 8-byte records and random auto-group byte budgets; BPF soak
set -o pipefail
mkdir -p gpurun_out/r5o
timeout -k 10 330 python3 -u scripts/soak_backend.py 300 31 > gpurun_out/r5o/soak_backend_seed31.log 2>&1; rc=$?
tail -2 gpurun_out/r5o/soak_backend_seed31.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 270 python3 -u scripts/soak_bpf.py 240 32 > gpurun_out/r5o/soak_bpf_seed32.log 2>&1; rc=$?
tail -2 gpurun_out/r5o/soak_bpf_seed32.log
exit $rc
