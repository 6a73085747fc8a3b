"""Round 6: saturated backend throughput and device fraction under latency caps
(cfg.group_max_us 0 / 2000 / 5000 / 20000), and the 25 % latency leg again."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "mos-networking-stack_amd"))
import bench  # noqa: E402
import mosrx  # noqa: E402

for key, tgt in (("S64", 48_000_000), ("M1500", 3_000_000)):
    tr = mosrx.Trace({"S64": mosrx.TRACE_S64, "M1500": mosrx.TRACE_M1500}[key], {"S64": 32768, "M1500": 65536}[key])
    for rep in range(2):
        for cap in (0, 2000, 5000, 20000):
            r = bench.measure_backend(tr, key, tgt, cpu=0, group=0, group_max_us=cap)
            print(json.dumps({"key": key, "cap": cap, "rep": rep, "mpkts": round(r["mpkts"], 1),
                              "dev_frac": r["device_roofline_frac"], "dev_us": r["device_us_per_batch"],
                              "bpl": r["batches_per_launch"]}), flush=True)
for cap in (0, 2000):
    r = bench.measure_backend_latency("S64", 0, 87.0, cpu=0, group_max_us=cap)
    print(json.dumps({"lat": "S64 auto 87", "cap": cap, "avail": r["avail_us"], "max_grp": r["max_group_frames"]}),
          flush=True)
