cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6k
timeout -k 10 500 python -u -m pytest tests/test_direct_gpu.py tests/test_backend_gpu.py tests/test_latency.py tests/test_parity_gpu.py -m gpu -x -q \
  --timeout 120 --timeout-method thread > gpurun_out/r6k/pytest.log 2>&1 || { tail -40 gpurun_out/r6k/pytest.log; exit 1; }
tail -2 gpurun_out/r6k/pytest.log
