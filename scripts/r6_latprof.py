"""Round 6: one latency leg (64 B, one batch per launch, 25 % load) alone, for a
rocprofv3 kernel + memory-copy trace of the drop-in path's group cycle."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "mos-networking-stack_amd"))
import bench  # noqa: E402

key = sys.argv[1] if len(sys.argv) > 1 else "S64"
group = int(sys.argv[2]) if len(sys.argv) > 2 else 1
rate = float(sys.argv[3]) if len(sys.argv) > 3 else 60.0
r = bench.measure_backend_latency(key, group, rate, cpu=0, seconds=0.3)
print(json.dumps(r), flush=True)
