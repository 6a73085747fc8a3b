"""Round 6: the drop-in path's residency table (bench.measure_backend_latency)
at 25 / 50 / 90 % of each configuration's saturated rate, with and without a
latency cap.  Prints one JSON line per leg."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "mos-networking-stack_amd"))
import bench  # noqa: E402
import mosrx  # noqa: E402

keys = sys.argv[1].split(",") if len(sys.argv) > 1 else ["S64", "M1500"]
caps = [int(x) for x in sys.argv[2].split(",")] if len(sys.argv) > 2 else [0]
for key in keys:
    tr = mosrx.Trace({"S64": mosrx.TRACE_S64, "M1500": mosrx.TRACE_M1500}[key], {"S64": 32768, "M1500": 65536}[key])
    for group in (0, 1, 8):
        sat = bench.measure_backend(tr, key, {"S64": 24_000_000, "M1500": 2_000_000}[key], cpu=0, group=group)
        print(json.dumps({"key": key, "group": group, "saturated_mpkts": round(sat["mpkts"], 1),
                          "dev_frac": sat["device_roofline_frac"]}), flush=True)
        for load in (0.25, 0.5, 0.9):
            for cap in caps:
                r = bench.measure_backend_latency(key, group, load * sat["mpkts"], cpu=0, group_max_us=cap)
                r.update(key=key, load=load)
                print(json.dumps(r), flush=True)
