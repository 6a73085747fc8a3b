"""Where the fused classify + BPF 64 B ring's extra time goes (diagnostic): the
ring of 256 x 32K 64 B frames as plain classification, fused with 8 trivial
programs (`ret #1`: the fused tile's fixed cost, masks stored), and fused with
the bench's 8 mOS filters; dispatch-stamped medians.  Records and masks are
checked against the oracle first.

    python3 scripts/probe_fused_cost.py [S64|IMIX] [set indices, comma separated: 0 plain, 1 8 x ret, 2 the 8 filters, 3+j 8 x filter j, 11 / 12 one trivial program]

PROBE_SHORT=1: no prewarm and a handful of launches (for rocprofv3 --pmc passes).
"""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for d in ("", "tests", "mos-networking-stack_amd"):
    sys.path.insert(0, os.path.join(ROOT, d))
import bench, mosrx, oracle_py as O

key = sys.argv[1] if len(sys.argv) > 1 else "S64"
kind, batch, ring = {"S64": (mosrx.TRACE_S64, 32768, 256), "IMIX": (mosrx.TRACE_IMIX, 262144, 8)}[key]
ctx = mosrx.Context(0)
trs = [mosrx.Trace(kind, batch, seed=bench.job_seed(kind, b)) for b in range(4)]
nres = 2 * ring
dbs = [ctx.upload(t.frames, t.off, t.len, frames_bytes=t.frames_bytes, max_len=t.max_len)
       for t in (trs[i % 4] for i in range(nres))]
trivial = [(np.array([(0x06, 0, 0, 1)], mosrx.BPF_INSN), m % 2) for m in range(8)]
sets = {"plain": None, "fused, 8 x ret #1": trivial, "fused, 8 mOS filters": bench.bpf_bench_programs()}
for j, (p, m) in enumerate(bench.bpf_bench_programs()):   # one filter's cost: 8 copies of it
    sets[f"fused, 8 x filter {j}"] = [(p, m)] * 8
sets["fused, 1 x ret #1 (frame length)"] = trivial[:1]    # 11: the fixed cost of the fused tile
sets["fused, 1 x ret #1 (datagram length)"] = trivial[1:2]  # 12
if len(sys.argv) > 2:
    sets = dict([list(sets.items())[int(a)] for a in sys.argv[2].split(",")])
short = os.environ.get("PROBE_SHORT") == "1"
for name, ps in sets.items():
    if ps is not None:
        ctx.bpf_set(ps)
        assert ctx.bpf_fused(), ctx.bpf_jit_log()
    qs = [ctx.queue_ex(dbs[i:i + ring], match=ps is not None) for i in range(0, nres, ring)]
    qs[0].run()
    t, d = trs[0], dbs[0]
    assert np.array_equal(d.results().view(np.uint8), O.classify(t.frames, t.off, t.len, O.params()).view(np.uint8))
    if ps is not None:
        np.testing.assert_array_equal(d.matches(), O.bpf_eval(ps, t.frames[:t.frames_bytes], t.off, t.len))
    if not short:
        bench.prewarm(lambda: qs[0].time(8, qs[1:], kernels=False))
    us = [1e3 * qs[0].time_dispatch(4 if short else 64, qs[1:]) for _ in range(1 if short else 5)]
    print(f"{key} ring {ring} x {batch}: {name:24s} {np.median(us):8.2f} us per launch "
          f"(min {min(us):.2f}, max {max(us):.2f})", flush=True)
    for q in qs:
        q.destroy()
