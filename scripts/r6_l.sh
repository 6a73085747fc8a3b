cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6l
timeout -k 10 300 python3 -u scripts/r6_cycle_direct.py > gpurun_out/r6l/cycle.jsonl 2> gpurun_out/r6l/cycle.err || { tail -20 gpurun_out/r6l/cycle.err; exit 1; }
cat gpurun_out/r6l/cycle.jsonl
