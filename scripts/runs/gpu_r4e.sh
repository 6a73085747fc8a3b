#!/bin/bash
# round 4: BPF parity after sizing the fused window to the set, then the fused rows
# and the backend legs with filters.  A failure ends the script.
cd "${GRAFT_REPO_ROOT:-.}"
out=gpurun_out/r4e
mkdir -p $out
timeout -k 10 400 python -u -m pytest -v --maxfail=5 --timeout 120 --timeout-method thread -m gpu \
    tests/test_bpf.py tests/test_bpf_groups.py > $out/pytest_bpf.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $out/pytest_bpf.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python -u bench.py --workloads S64,IMIX,IMIX_cls_bpf,IMIX_cls_bpf_ring,S64_cls_bpf_ring \
    --no-cpu --steps 20 --warmup 5 --detail $out/bench_detail.json > $out/bench.out 2> $out/bench.err
rc=$?; echo "bench rc=$rc"; grep "^\[bench\]" $out/bench.err
python3 - <<'PY'
import json
d = json.load(open("gpurun_out/r4e/bench_detail.json"))
for k, v in (d.get("e2e") or {}).get("backend", {}).items():
    print("backend", k, round(v["mpkts"], 1), "Mpkt/s", v["group"], "bpl", v["batches_per_launch"], "dev_us", v["device_us_per_batch"], "frac", v["device_roofline_frac"])
PY
exit $rc
