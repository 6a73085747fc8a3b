"""Throughput of back-to-back independent batches on 1/2/4 streams (diagnostic)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mos-networking-stack_amd"))
import mosrx  # noqa: E402

ctx = mosrx.Context(0)
L3 = 256 << 20
ITERS = 200
for name, kind, n in [("M1500", mosrx.TRACE_M1500, 65536), ("IMIX", mosrx.TRACE_IMIX, 262144),
                      ("S64", mosrx.TRACE_S64, 32768)]:
    t = mosrx.Trace(kind, n)
    ncopy = min(256, max(4, -(-2 * L3 // t.frames_bytes)))
    dbs = [ctx.upload(t.frames, t.off, t.len, frames_bytes=t.frames_bytes, max_len=t.max_len) for _ in range(ncopy)]
    ab = t.caplen_sum + 22 * t.n
    ctx.time_dev(dbs, 20)
    for ns in (1, 2, 4):
        best = min(ctx.time_dev_streams(dbs, ITERS, ns) for _ in range(3))
        per = best / ITERS
        print(f"{name} streams={ns}: {per*1e3:7.2f} us/batch  {ab/(per*1e-3)/1e9:7.0f} GB/s  "
              f"{n/(per*1e-3)/1e6:9.0f} Mpkt/s", flush=True)
    for d in dbs:
        d.free()
