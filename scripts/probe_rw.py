"""Mixed read/write rate of the box (mosrx_probe_rw_bw) for several write ratios.

Diagnostic for the roofline report: the 64 B rows write one 16-byte record per
~70 B read, IMIX one per ~364 B, 1500 B one per ~1520 B."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mos-networking-stack_amd"))
import mosrx  # noqa: E402

ctx = mosrx.Context(0)
for rep in range(2):
    print(f"read only 512 MiB x3 240 passes: {ctx.probe_read_bw(512 << 20, 3, 240):.1f} GB/s", flush=True)
    for k in (4, 8, 16, 32, 64):
        print(f"rw 1 in {k:<3d} 512 MiB x3 240 passes: {ctx.probe_rw_bw(k, 512 << 20, 3, 240):.1f} GB/s", flush=True)
ctx.close()
