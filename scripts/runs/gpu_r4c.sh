#!/bin/bash
# round 4: the new bench rows (compact S64_hdr, fused classify + BPF rings, the
# backend with filters) next to their round-3 forms.
cd "${GRAFT_REPO_ROOT:-.}"
out=gpurun_out/r4c
mkdir -p $out
timeout -k 10 600 python -u bench.py --workloads S64,S64_hdr,S64_hdr16,S64_hdr_packed,IMIX,IMIX_cls_bpf,IMIX_cls_bpf_ring,S64_cls_bpf_ring \
    --no-cpu --steps 20 --warmup 5 --detail $out/bench_detail.json > $out/bench.out 2> $out/bench.err
rc=$?; echo "bench rc=$rc"; grep "^\[bench\]" $out/bench.err
python3 - <<'PY'
import json
d = json.load(open("gpurun_out/r4c/bench_detail.json"))
for k, v in (d.get("e2e") or {}).get("backend", {}).items():
    print("backend", k, round(v["mpkts"], 1), "Mpkt/s", v["group"], "bpl", v["batches_per_launch"], "dev_us", v["device_us_per_batch"], "frac", v["device_roofline_frac"])
print("numa", d.get("numa"))
PY
exit $rc
