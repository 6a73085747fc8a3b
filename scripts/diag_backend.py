"""Backend device-time diagnosis: kernel time per batch (HIP events) through
gpu_module_func with and without a group in flight behind the consumed one."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "mos-networking-stack_amd"))
import bench  # noqa: E402
import mosrx  # noqa: E402

for key, kind, n in [("S64", mosrx.TRACE_S64, 32768), ("M1500", mosrx.TRACE_M1500, 65536)]:
    tr = mosrx.Trace(kind, n)
    for group in (1, 8, 64):
        if key == "M1500" and group == 64:
            continue
        for pipe in (False, True):
            ctx_batch = n
            src = mosrx.mem_source(tr.frames, tr.off, tr.len, loops=max(2, 4 * group))
            be = mosrx.GpuBackend([src], batch=ctx_batch, pipeline=pipe, cpu=0, group=group, timing=True)
            try:
                be.run_loop(max_pkts=ctx_batch * group)
                s0 = be.stats()
                st = be.run_loop()
                s1 = be.stats()
            finally:
                be.close()
            b = s1.rx_batches - s0.rx_batches
            us = 1e3 * (s1.kernel_ms - s0.kernel_ms) / max(b, 1)
            frac = bench.algo_bytes(tr) / (us * 1e-6) / 1e9 / 8000 if us > 0 else 0
            print(f"{key} group {group:2d} pipeline {int(pipe)}: {b} batches, {s1.kernel_launches - s0.kernel_launches} "
                  f"launches, device {us:.2f} us/batch, frac {frac:.3f}", flush=True)
