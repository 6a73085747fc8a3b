# round 6: parity of the touched paths (counters, backend), then the latency table
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6a
timeout -k 10 400 python -u -m pytest tests/test_parity_gpu.py tests/test_backend_gpu.py tests/test_simple_firewall.py -m gpu -x -q \
  --timeout 120 --timeout-method thread > gpurun_out/r6a/pytest.log 2>&1 || { tail -30 gpurun_out/r6a/pytest.log; exit 1; }
tail -3 gpurun_out/r6a/pytest.log
timeout -k 10 400 python -u scripts/r6_latency.py S64,M1500 0,2000 > gpurun_out/r6a/latency.jsonl 2> gpurun_out/r6a/latency.err || { tail -20 gpurun_out/r6a/latency.err; exit 1; }
cat gpurun_out/r6a/latency.jsonl
