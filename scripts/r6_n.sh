cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6n
timeout -k 10 600 python -u -m pytest tests/test_direct_gpu.py tests/test_backend_gpu.py tests/test_simple_firewall.py tests/test_mos_consumer.py -m gpu -x -q \
  --timeout 120 --timeout-method thread > gpurun_out/r6n/pytest.log 2>&1 || { tail -40 gpurun_out/r6n/pytest.log; exit 1; }
tail -2 gpurun_out/r6n/pytest.log
timeout -k 10 300 python3 -u scripts/r6_lat90.py > gpurun_out/r6n/lat90.jsonl 2> gpurun_out/r6n/lat90.err || { tail -20 gpurun_out/r6n/lat90.err; exit 1; }
grep -v "^\[" gpurun_out/r6n/lat90.err
