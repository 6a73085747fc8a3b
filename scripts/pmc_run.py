"""Isolated launches of one bench workload's kernel, for rocprofv3 --pmc passes.

Same trace, resident copies (> 256 MiB Infinity Cache) and kernel as bench.py;
N single launches on one stream.  Usage: python3 scripts/pmc_run.py M1500 [N]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "mos-networking-stack_amd"))
import bench  # noqa: E402
import mosrx  # noqa: E402

key = sys.argv[1] if len(sys.argv) > 1 else "M1500"
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 40
kind, batch, _ = bench.WORKLOADS[key]
ctx = mosrx.Context(0)
ctx.set_params(mosrx.default_params(skip_tcp_csum=1 if key == "S64_hdr" else 0))
tr = mosrx.Trace(kind, batch)
ncopy = min(256, max(2, -(-2 * bench.L3_BYTES // tr.frames_bytes)))
dbs = [ctx.upload(tr.frames, tr.off, tr.len, frames_bytes=tr.frames_bytes, max_len=tr.max_len) for _ in range(ncopy)]
op = bench.OPS.get(key, mosrx.OP_CLASSIFY)
if op == mosrx.OP_BPF:
    ctx.bpf_set(bench.bpf_bench_programs())
arg = mosrx.TX_IP_CSUM | mosrx.TX_TCP_CSUM if op == mosrx.OP_TX_CSUM else 0
_, avg = ctx.time_op(op, dbs, iters, 1, arg, total=False)
print(f"{key}: {iters} isolated launches, avg {avg * 1e3:.2f} us (HIP events), "
      f"algo bytes/launch {bench.algo_bytes(tr, key)}", flush=True)
for d in dbs:
    d.free()
ctx.close()
