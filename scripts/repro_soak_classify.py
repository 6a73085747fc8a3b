"""Replay one batch of scripts/soak_classify.py by its seed and show where the
GPU and the oracle differ (diagnostic).  Usage: repro_soak_classify.py SEED"""
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mos-networking-stack_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "scripts"))
import numpy as np  # noqa: E402

import mosrx  # noqa: E402
import oracle_py as O  # noqa: E402
import soak_classify as S  # noqa: E402
from pktlib import pack_frames  # noqa: E402

s = int(sys.argv[1])
rng = random.Random(s)
fr = [S.rand_frame(rng) for _ in range(rng.choice([1, 2, 63, 64, 65, 255, 256, 257, rng.randint(1, 3000)]))]
assert rng.random() < 0.8   # the packed branch (the only one with the TX rewrite)
buf, off, ln = pack_frames(fr, align=rng.choice([1, 2, 4, 16]), phase=rng.randint(0, 15), gap=rng.choice([0, 0, 3, 64]))
ln = ln.copy()
for i in rng.sample(range(len(ln)), k=min(len(ln), rng.randint(0, 5))):
    ln[i] = rng.randint(0, int(ln[i]))
p = S.rand_params(rng)
variant = rng.choice(S.ALL_VARIANTS)
ctx = mosrx.Context(0)
ctx.set_variant(variant)
S.run_both(ctx, buf, off, ln, p, side=True)
assert rng.random() < 0.3
fl = rng.choice([mosrx.TX_IP_CSUM, mosrx.TX_TCP_CSUM, mosrx.TX_IP_CSUM | mosrx.TX_TCP_CSUM])
print("variant", variant, "flags", fl, "n", len(fr), "offsets", off[:4], "bytes", len(buf))
want = O.tx_csum(buf, off, ln, fl)
for v in S.ALL_VARIANTS:
    ctx.set_variant(v)
    got = ctx.tx_csum_host(buf, off, ln, fl)
    d = np.nonzero(got != want)[0]
    print("variant", v, "bytes differing", len(d))
    if len(d) and v == variant:
        for b in d[:8]:
            i = int(np.searchsorted(off.astype(np.int64), b, side="right") - 1)
            o = int(off[i])
            print(f"  byte {b}: frame {i} (off {o}, caplen {ln[i]}, len {len(fr[i])}) at +{b - o}: gpu {got[b]:#x} ora {want[b]:#x} orig {buf[b]:#x}")
            f = buf[o:o + 60]
            print("   hdr", bytes(f[12:54]).hex())
