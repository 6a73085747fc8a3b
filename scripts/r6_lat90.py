"""Round 6: the latency legs most sensitive to the direct-group limits, repeated
(64 B auto groups at 90 % load three times), with the defaults in effect."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "mos-networking-stack_amd"))
import bench  # noqa: E402

for key, g, rate in (("S64", 0, 301.7), ("S64", 0, 301.7), ("S64", 0, 301.7), ("S64", 0, 84), ("S64", 0, 168),
                     ("S64", 1, 258), ("S64", 8, 290), ("M1500", 1, 31.4), ("M1500", 0, 9.8), ("M1500", 0, 19.7)):
    r = bench.measure_backend_latency(key, g, rate, cpu=0)
    r.update(key=key)
    print(json.dumps(r), flush=True)
    print(f"{key} g{g} {rate}: p50 {r['avail_us']['p50_us']} p99 {r['avail_us']['p99_us']} delivered "
          f"{r['delivered_mpkts']} direct {r['direct_groups']}/{r['groups']} mean {r['mean_group_frames']}",
          file=sys.stderr, flush=True)
