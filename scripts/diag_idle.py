"""Does a kernel that runs after idle gaps (a PCIe-bound pipeline's duty cycle)
run slower than back-to-back?  Device-resident queue launches, events around
each, with 0 / 0.5 / 2 ms of host sleep between them."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mos-networking-stack_amd"))
import numpy as np  # noqa: E402
import mosrx  # noqa: E402

ctx = mosrx.Context(0)
for kind, n, nb in [(mosrx.TRACE_S64, 32768, 64), (mosrx.TRACE_M1500, 65536, 8)]:
    tr = mosrx.Trace(kind, n)
    dbs = [ctx.upload(tr.frames, tr.off, tr.len, frames_bytes=tr.frames_bytes, max_len=tr.max_len) for _ in range(nb)]
    q = ctx.queue(dbs)
    tot, _ = q.time(200, kernels=False)
    print(f"kind {kind} x{nb}: back-to-back {1e3 * tot / 200:.1f} us/launch", flush=True)
    for gap in (0.0, 0.0005, 0.002, 0.01):
        ks = []
        for i in range(30):
            if gap:
                time.sleep(gap)
            _, k = q.time(1)
            ks.append(k)
        print(f"  gap {gap * 1e3:.1f} ms: isolated median {1e3 * np.median(ks):.1f} us, min {1e3 * min(ks):.1f}", flush=True)
    q.destroy()
    for d in dbs:
        d.free()
ctx.close()
