"""Round 6: the backend's 64 B device time against the launch's size, interleaved on one box:
auto groups of 256 MiB / 512 MiB / 1 GiB of frames and explicit groups of 128 batches."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "mos-networking-stack_amd"))
import bench  # noqa: E402
import mosrx  # noqa: E402

tr = mosrx.Trace(mosrx.TRACE_S64, 32768)
legs = [("auto256", dict(group=0, group_bytes=256 << 20)), ("auto512", dict(group=0, group_bytes=512 << 20)),
        ("auto1024", dict(group=0, group_bytes=1 << 30)), ("g128", dict(group=128)), ("g64", dict(group=64))]
for rep in range(3):
    for name, kw in legs:
        r = bench.measure_backend(tr, "S64", 96_000_000, cpu=0, **kw)
        print(json.dumps({"leg": name, "rep": rep, "mpkts": round(r["mpkts"], 1), "dev_frac": r["device_roofline_frac"],
                          "dev_us": r["device_us_per_batch"], "bpl": r["batches_per_launch"]}), flush=True)
