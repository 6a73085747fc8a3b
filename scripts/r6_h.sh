cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6h
timeout -k 10 500 python -u -m pytest tests/test_backend_gpu.py tests/test_mos_consumer.py tests/test_simple_firewall.py tests/test_parity_gpu.py -m gpu -x -q \
  --timeout 120 --timeout-method thread > gpurun_out/r6h/pytest.log 2>&1 || { tail -30 gpurun_out/r6h/pytest.log; exit 1; }
tail -2 gpurun_out/r6h/pytest.log
rm -rf gpurun_out/latprof
bash scripts/r6_g.sh
