"""Quick GPU measurements for kernel tuning (not part of the bench contract).

Interleaves kernel variants in one process (rounds x variants) and reports the
median kernel time per workload, so variant deltas are not cross-process noise."""
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mos-networking-stack_amd"))
import mosrx  # noqa: E402

VARIANTS = [int(v) for v in os.environ.get("TUNE_VARIANTS", "0,1,2,3").split(",")]
ROUNDS = int(os.environ.get("TUNE_ROUNDS", "5"))
ctx = mosrx.Context(0)
if os.environ.get("TUNE_BW", "1") == "1":
    print(f"read_bw 96 MiB x6: {ctx.probe_read_bw(96 << 20, 6, 60):.1f} GB/s", flush=True)
L3 = 256 << 20
for name, kind, n in [("M1500", mosrx.TRACE_M1500, 65536), ("IMIX", mosrx.TRACE_IMIX, 262144),
                      ("S64", mosrx.TRACE_S64, 32768)]:
    t = mosrx.Trace(kind, n)
    ncopy = min(256, max(2, -(-2 * L3 // t.frames_bytes)))
    dbs = [ctx.upload(t.frames, t.off, t.len, frames_bytes=t.frames_bytes, max_len=t.max_len) for _ in range(ncopy)]
    ab = t.caplen_sum + 22 * t.n
    res = {v: [] for v in VARIANTS}
    for r in range(ROUNDS):
        for v in VARIANTS:
            ctx.set_variant(v)
            ctx.time_dev(dbs, 10)
            res[v].append(ctx.time_dev_kernels(dbs, 60))
    for v in VARIANTS:
        k = statistics.median(res[v])
        print(f"{name} var{v}: kernel {k*1e3:6.1f} us  {ab/(k*1e-3)/1e9:6.0f} GB/s  "
              f"min {min(res[v])*1e3:.1f}", flush=True)
    for d in dbs:
        d.free()

if os.environ.get("TUNE_SCALE", "1") == "1":
    # kernel time vs batch size: T(n) = a + b n separates launch/startup cost from streaming rate
    ctx.set_variant(int(os.environ.get("TUNE_SCALE_VAR", "2")))
    for n in (8192, 16384, 32768, 65536, 131072, 262144):
        t = mosrx.Trace(mosrx.TRACE_M1500, n)
        ncopy = min(64, max(2, -(-2 * L3 // t.frames_bytes)))
        dbs = [ctx.upload(t.frames, t.off, t.len, frames_bytes=t.frames_bytes, max_len=t.max_len) for _ in range(ncopy)]
        ab = t.caplen_sum + 22 * t.n
        ctx.time_dev(dbs, 10)
        k = min(ctx.time_dev_kernels(dbs, 40) for _ in range(3))
        q = [ctx.queue(dbs[i:i + 2]) for i in range(0, len(dbs) - 1, 2)]
        _, kq = q[0].time(40, q[1:])
        print(f"M1500 n={n:6d}: kernel {k*1e3:7.1f} us {ab/(k*1e-3)/1e9:6.0f} GB/s | queue-of-2 "
              f"{kq*1e3:7.1f} us {2*ab/(kq*1e-3)/1e9:6.0f} GB/s", flush=True)
        for x in q:
            x.destroy()
        for d in dbs:
            d.free()
