# round 5: backend legs with dispatch-stamped device time and packed compact records
set -o pipefail
mkdir -p gpurun_out/r5f
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_backend_gpu.py tests/test_layout_hint.py tests/test_rx_loop.py -m gpu -x -q \
  --timeout 120 --timeout-method thread > gpurun_out/r5f/pytest.log 2>&1; rc=$?
tail -1 gpurun_out/r5f/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 --workloads M1500,S64,IMIX,S64_c8 --no-cpu \
  --detail gpurun_out/r5f/bench_detail.json > gpurun_out/r5f/bench.out 2> gpurun_out/r5f/bench.err; rc=$?
echo "bench rc=$rc"; grep "^\[bench\]" gpurun_out/r5f/bench.err
python3 - <<'PY'
import json
d = json.load(open("gpurun_out/r5f/bench_detail.json"))
for k, v in d["e2e"]["backend"].items():
    print(k, {kk: v[kk] for kk in ("mpkts", "batches_per_launch", "device_us_per_batch", "device_roofline_frac", "records")})
PY
exit $rc
