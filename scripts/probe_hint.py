#!/usr/bin/env python3
"""A/B of the layout hint on config #2's single launch (one 32K x 64 B batch per
launch), for rocprofv3 --kernel-trace: hinted and plain launches alternate in one
process, each launch isolated (the host waits for it), over 256 resident copies
of each (1 GB, past the Infinity Cache).  The kernels tell the forms apart by
name (mosrx_classify_kernel<0, 256> hinted, <0, 0> plain); the trace's
per-kernel durations are the comparison.  Records are checked equal first."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mos-networking-stack_amd"))
import numpy as np  # noqa: E402

import mosrx  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 4000
COPIES = 256
ctx = mosrx.Context(0)
ctx.set_params(mosrx.default_params())
t = mosrx.Trace(mosrx.TRACE_S64, 32_768)
hinted = [ctx.upload(t.frames, t.off, t.len, frames_bytes=t.frames_bytes, max_len=t.max_len, hint="auto")
          for _ in range(COPIES)]
plain = [ctx.upload(t.frames, t.off, t.len, frames_bytes=t.frames_bytes, max_len=t.max_len, hint=None)
         for _ in range(COPIES)]
assert hinted[0].hint is not None and plain[0].hint is None
ctx.classify_dev(hinted[0])
ctx.classify_dev(plain[0])
assert np.array_equal(hinted[0].results().view(np.uint8), plain[0].results().view(np.uint8))
for i in range(N):
    ctx.classify_dev(hinted[i % COPIES], sync=True)
    ctx.classify_dev(plain[(i * 7) % COPIES], sync=True)
print(f"probe_hint: {N} isolated launches of each form", flush=True)
ctx.close()
