cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6i
timeout -k 10 300 python -u -m pytest tests/test_direct_gpu.py -m gpu -x -q \
  --timeout 120 --timeout-method thread > gpurun_out/r6i/direct.log 2>&1 || { tail -40 gpurun_out/r6i/direct.log; exit 1; }
tail -2 gpurun_out/r6i/direct.log
timeout -k 10 500 python -u -m pytest tests/test_backend_gpu.py tests/test_bpf_groups.py tests/test_mos_consumer.py tests/test_simple_firewall.py -m gpu -x -q \
  --timeout 120 --timeout-method thread > gpurun_out/r6i/backend.log 2>&1 || { tail -40 gpurun_out/r6i/backend.log; exit 1; }
tail -2 gpurun_out/r6i/backend.log
timeout -k 10 400 python -u scripts/r6_direct.py > gpurun_out/r6i/direct_sweep.jsonl 2> gpurun_out/r6i/direct_sweep.err || { tail -20 gpurun_out/r6i/direct_sweep.err; exit 1; }
cat gpurun_out/r6i/direct_sweep.err | grep -v "^\[" | tail -40
