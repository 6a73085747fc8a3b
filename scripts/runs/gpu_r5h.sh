# round 5: the 64 B backend legs (compact census fast path, 512 MiB auto groups)
set -o pipefail
mkdir -p gpurun_out/r5h
timeout -k 10 300 python -u -m pytest tests/test_rx_loop.py tests/test_backend_gpu.py -m gpu -x -q --timeout 120 \
  --timeout-method thread > gpurun_out/r5h/pytest.log 2>&1; rc=$?
tail -1 gpurun_out/r5h/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 --workloads S64 --no-cpu \
  --detail gpurun_out/r5h/bench_detail.json > gpurun_out/r5h/bench.out 2> gpurun_out/r5h/bench.err; rc=$?
echo "bench rc=$rc"
python3 - <<'PY'
import json
d = json.load(open("gpurun_out/r5h/bench_detail.json"))
for k, v in d["e2e"]["backend"].items():
    print(k, {kk: v[kk] for kk in ("mpkts", "batches_per_launch", "device_us_per_batch", "device_roofline_frac", "records")})
PY
exit $rc
