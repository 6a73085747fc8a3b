cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6f
timeout -k 10 600 python -u scripts/r6_gb2.py > gpurun_out/r6f/gb2.jsonl 2> gpurun_out/r6f/gb2.err || { tail -20 gpurun_out/r6f/gb2.err; exit 1; }
cat gpurun_out/r6f/gb2.jsonl
