"""Debug: stream shapes vs oracle on the layouts of test_stream_shapes_layouts (diagnostic)."""
import os, random, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mos-networking-stack_amd")); sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np
import mosrx
import oracle_py as O
from pktlib import pack_frames
from golden.make_golden import random_frames
ctx = mosrx.Context(0)
p = mosrx.default_params(forward=0)
ctx.set_params(p)
rng = random.Random(30)
frames = random_frames(rng, 300, 0) + random_frames(rng, 150, 2) + random_frames(rng, 150, 1)
rng.shuffle(frames)
buf, off, ln = pack_frames(frames, align=rng.choice([1, 2, 16]), phase=0, gap=rng.randint(0, 3))
ora = O.classify(buf, off, ln, O.params(forward=0))
for var in (2, 6, 30, 34, 38, 46):
    ctx.set_variant(var)
    out = ctx.classify_host(buf, off, ln)
    bad = np.nonzero(np.any(out.view(np.uint8).reshape(-1, 16) != ora.view(np.uint8).reshape(-1, 16), 1))[0]
    print("variant", var, "bad", bad.tolist())
    for i in bad[:8]:
        o = int(off[i])
        print("   ", i, "off", o, "len", int(ln[i]), "gpu", out[i], "ora", ora[i], "prev hi", int(off[i-1]) + int(ln[i-1]) if i else -1)
