"""Round 6: direct (copy-free) small groups -- the latency legs of the bench's
table with cfg.direct_kb off and at two limits, and the saturated 64 B
one-batch-per-launch leg (2.2 MB groups) copied vs direct.  One JSON line per
leg, progress on stderr."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "mos-networking-stack_amd"))
import bench  # noqa: E402
import mosrx  # noqa: E402

legs = [("S64", 0, r) for r in (84, 167, 301)] + [("S64", 1, r) for r in (60, 120)] + \
       [("M1500", 0, r) for r in (9.7, 19.4)] + [("M1500", 1, r) for r in (8.7, 17.4)]
limits = [int(x) for x in (sys.argv[1].split(",") if len(sys.argv) > 1 else ["0", "1024", "4096"])]
for key, g, rate in legs:
    for kb in limits:
        t = time.time()
        r = bench.measure_backend_latency(key, g, rate, cpu=0, seconds=0.4, direct_kb=kb)
        r.update(key=key, direct_kb=kb)
        print(json.dumps(r), flush=True)
        print(f"{key} g{g} {rate} kb{kb}: p50 {r['avail_us']['p50_us']} p99 {r['avail_us']['p99_us']} "
              f"direct {r['direct_groups']}/{r['groups']} ({time.time() - t:.1f}s)", file=sys.stderr, flush=True)
tr = mosrx.Trace(mosrx.TRACE_S64, 32_768 * 64)
for kb in (0, 4096):
    r = bench.measure_backend(tr, "S64", 32_768 * 3000, cpu=0, group=1, direct_kb=kb)
    print(json.dumps({"leg": "S64_group1_saturated", "direct_kb": kb, "mpkts": round(r["mpkts"], 1),
                      "device_us_per_batch": r["device_us_per_batch"]}), flush=True)
    print(f"S64 g1 saturated kb{kb}: {r['mpkts']:.1f} Mpkt/s", file=sys.stderr, flush=True)
