cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6d
timeout -k 10 500 python -u scripts/r6_gb.py > gpurun_out/r6d/gb.jsonl 2> gpurun_out/r6d/gb.err || { tail -20 gpurun_out/r6d/gb.err; exit 1; }
cat gpurun_out/r6d/gb.jsonl
