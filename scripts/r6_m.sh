cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6m
timeout -k 10 300 python3 -u scripts/r6_cycle_direct.py > gpurun_out/r6m/cycle_block.jsonl 2> gpurun_out/r6m/cycle.err || { tail -20 gpurun_out/r6m/cycle.err; exit 1; }
MOSRX_WAIT_SPIN=1 timeout -k 10 300 python3 -u scripts/r6_cycle_direct.py > gpurun_out/r6m/cycle_spin.jsonl 2>> gpurun_out/r6m/cycle.err || { tail -20 gpurun_out/r6m/cycle.err; exit 1; }
paste -d'\n' gpurun_out/r6m/cycle_block.jsonl gpurun_out/r6m/cycle_spin.jsonl | cut -c1-220
