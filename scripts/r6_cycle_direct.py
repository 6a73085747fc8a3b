"""Round 6: the group cycle's fixed cost, direct vs copied -- one 64 B group of n
frames submitted and waited in a loop (mosrx_classify_host_group_submit_c8 on
pinned staging), mean microseconds per cycle; then two slots alternating."""
import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "mos-networking-stack_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np  # noqa: E402
import mosrx  # noqa: E402
from test_direct_gpu import _stage  # noqa: E402

ctx = mosrx.Context(0)
ctx.set_params(mosrx.default_params())
for kind, name in ((mosrx.TRACE_S64, "S64"), (mosrx.TRACE_M1500, "M1500")):
    for n in (256, 1024, 4096, 32768):
        t = mosrx.Trace(kind, n, nflows=500)
        base, arr = ctx.host_alloc(t.frames_bytes + 8 * n + 4096)
        rp, rec = ctx.host_alloc(16 * n)
        batches, _ = _stage(arr, base, t, 1)
        for direct in (0, 1 << 30):
            ctx.set_direct(direct)
            for _ in range(50):
                ctx.group_submit_c8(0, batches, [rp])
                ctx.group_wait(0)
            iters = 2000 if n <= 4096 else 500
            t0 = time.perf_counter()
            for _ in range(iters):
                ctx.group_submit_c8(0, batches, [rp])
                ctx.group_wait(0)
            one = (time.perf_counter() - t0) / iters * 1e6
            t0 = time.perf_counter()
            ctx.group_submit_c8(0, batches, [rp])
            for i in range(iters):
                ctx.group_submit_c8((i + 1) & 1, batches, [rp])
                ctx.group_wait(i & 1)
            ctx.group_wait(iters & 1)
            two = (time.perf_counter() - t0) / iters * 1e6
            # the kernel's own duration (dispatch-stamped, mosrx_set_timing), median of 200 timed cycles
            L = mosrx.lib()
            L.mosrx_set_timing(ctx.handle, 1)
            ks = []
            for _ in range(200):
                ctx.group_submit_c8(0, batches, [rp])
                ctx.group_wait(0)
                ms = C.c_float()
                if L.mosrx_last_kernel_ms(ctx.handle, C.byref(ms)) == 0:
                    ks.append(ms.value * 1e3)
            L.mosrx_set_timing(ctx.handle, 0)
            print(json.dumps({"frames": name, "n": n, "direct": bool(direct), "slot_direct": ctx.slot_direct(0),
                              "us_per_cycle_1slot": round(one, 2), "us_per_group_2slots": round(two, 2),
                              "kernel_us": round(float(np.median(ks)), 2) if ks else None}), flush=True)
        ctx.host_free(rp)
        ctx.host_free(base)
ctx.set_direct(0)
