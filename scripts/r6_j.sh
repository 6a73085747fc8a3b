cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6j
timeout -k 10 600 python -u scripts/r6_direct2.py > gpurun_out/r6j/direct2.jsonl 2> gpurun_out/r6j/direct2.err || { tail -20 gpurun_out/r6j/direct2.err; exit 1; }
grep -v "^\[" gpurun_out/r6j/direct2.err | tail -40
