cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6c
timeout -k 10 500 python -u scripts/r6_cap.py > gpurun_out/r6c/cap.jsonl 2> gpurun_out/r6c/cap.err || { tail -20 gpurun_out/r6c/cap.err; exit 1; }
cat gpurun_out/r6c/cap.jsonl
