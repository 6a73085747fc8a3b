"""Isolated launches of one bench workload's kernel, for rocprofv3 --pmc passes.

Same traces, resident batches (>= 1.2 GB, past the 256 MiB Infinity Cache) and
kernel as bench.py: for a ring workload N queue launches (one per step), else
N single classify launches, all on one stream.
Usage: python3 scripts/pmc_run.py M1500 [N]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "mos-networking-stack_amd"))
import bench  # noqa: E402
import mosrx  # noqa: E402

key = sys.argv[1] if len(sys.argv) > 1 else "M1500"
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 40
kind, batch, ring, _ = bench.WORKLOADS[key]
ctx = mosrx.Context(0)
ctx.set_params(mosrx.default_params(skip_tcp_csum=1 if key.startswith("S64_hdr") else 0))
probe = mosrx.Trace(kind, batch)
if ring:
    nres = max(2 * ring, -(-bench.RESIDENT_BYTES // probe.frames_bytes))
    nres = -(-nres // ring) * ring
else:
    nres = min(256, max(2, -(-bench.RESIDENT_BYTES // probe.frames_bytes)))
dbs, trs, _ = bench.resident_batches(ctx, key, 1, 0, nres)
tr = trs[0]
ab = bench.algo_bytes(tr, key) * (ring or 1)
if ring:   # the queues bench.measure builds for the row
    if "_cls_bpf" in key:
        ctx.bpf_set(bench.bpf_bench_programs())
    qs = [ctx.queue_ex(dbs[i:i + ring], match="_cls_bpf" in key, compact=key in bench.COMPACT)
          for i in range(0, len(dbs), ring)]
    _, avg = qs[0].time(iters, qs[1:])
    for q in qs:
        q.destroy()
else:
    op = bench.OPS.get(key, mosrx.OP_CLASSIFY)
    if op in (mosrx.OP_BPF, mosrx.OP_CLASSIFY_BPF):
        ctx.bpf_set(bench.bpf_bench_programs())
    arg = mosrx.TX_IP_CSUM | mosrx.TX_TCP_CSUM if op in (mosrx.OP_TX_CSUM, mosrx.OP_TX_CHECKS) else 0
    _, avg = ctx.time_op(op, dbs, iters, 1, arg, total=False)
print(f"{key}: {iters} isolated launches, avg {avg * 1e3:.2f} us (HIP events), "
      f"algo bytes/launch {ab}", flush=True)
for d in dbs:
    d.free()
ctx.close()
