"""Round 6: where direct groups stop paying -- saturated backend legs (64 B one
batch / 8 batches per launch, 1500 B one batch, IMIX one batch) with
cfg.direct_kb 0 / 4 MiB / 1 GiB, and the 90 % latency legs at 4 / 16 / 64 MiB."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "mos-networking-stack_amd"))
import bench  # noqa: E402

for key, g, target in (("S64", 1, 32_768 * 3000), ("S64", 8, 32_768 * 4000), ("M1500", 1, 65_536 * 120),
                       ("IMIX", 1, 262_144 * 40)):
    tr = bench.backend_trace(key, {"S64": 32_768, "M1500": 65_536, "IMIX": 262_144}[key] * (64 if key == "S64" else 4))
    for kb in (0, 4096, 1 << 20):
        t = time.time()
        r = bench.measure_backend(tr, key, target, cpu=0, group=g, direct_kb=kb)
        out = {"leg": f"{key}_group{g}", "direct_kb": kb, "mpkts": round(r["mpkts"], 2),
               "device_us_per_batch": r["device_us_per_batch"], "direct_launches": r["direct_launches"],
               "kernel_launches": r["kernel_launches"]}
        print(json.dumps(out), flush=True)
        print(f"{out} ({time.time() - t:.1f}s)", file=sys.stderr, flush=True)
for key, g, rate in (("S64", 0, 301), ("S64", 8, 284), ("M1500", 0, 35), ("M1500", 1, 31.3), ("M1500", 8, 32.3)):
    for kb in (4096, 16384, 65536):
        r = bench.measure_backend_latency(key, g, rate, cpu=0, seconds=0.4, direct_kb=kb)
        r.update(key=key, direct_kb=kb)
        print(json.dumps(r), flush=True)
        print(f"{key} g{g} {rate} kb{kb}: p50 {r['avail_us']['p50_us']} p99 {r['avail_us']['p99_us']} "
              f"delivered {r['delivered_mpkts']} direct {r['direct_groups']}/{r['groups']}", file=sys.stderr, flush=True)
