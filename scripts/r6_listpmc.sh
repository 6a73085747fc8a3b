cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6list
timeout -k 10 120 rocprofv3 -L > gpurun_out/r6list/avail.txt 2>&1
grep -i -E "mall|umc|dram|hbm|df_|TCC_EA0_(RD|WR)" gpurun_out/r6list/avail.txt | head -60
wc -l gpurun_out/r6list/avail.txt
