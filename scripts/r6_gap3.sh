# VERDICT r5 next #1, third pass: host- or device-side pages behind the post-DMA slowdown
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/gap3
cat /sys/kernel/mm/transparent_hugepage/enabled /sys/kernel/mm/transparent_hugepage/defrag > gpurun_out/gap3/thp.txt 2>&1
run() {  # name, key, phase
  timeout -k 10 150 rocprofv3 --kernel-trace --stats -d gpurun_out/gap3/kt_$1 -o kt -- \
    python3 -u scripts/diag_backend_gap.py $2 $3 >> gpurun_out/gap3/diag.log 2>gpurun_out/gap3/err_$1.log || exit $?
}
run c8_b2b M1500c8 res_b2b
run c8_hostpages M1500c8 res_dma_hostpages
run c8_devpages M1500c8 res_dma_devpages
run c8_fresh_other M1500c8 res_fresh_other
