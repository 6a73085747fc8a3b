"""Soak of the batched BPF engines (diagnostic, not a test).

    python3 scripts/soak_bpf.py [seconds=240] [seed=1]

Random admitted program sets (tests/test_bpf.py's generator: every opcode,
jump shape and bound, 32 programs per set at both call-site lengths) on the
hipRTC-compiled engine, the interpreter and the fused classify + BPF pass,
over the reference's golden BPF frames and a random IMIX trace per set, until
the time is up.  Every match mask must equal the oracle's (itself pinned to
mOS's sfbpf_filter), and the fused pass's records the oracle's records.  A
mismatch prints the seed and exits 1.
"""
import os
import random
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mos-networking-stack_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np  # noqa: E402

import mosrx  # noqa: E402
import oracle_py as O  # noqa: E402
import test_bpf as TB  # noqa: E402


def main():
    budget = float(sys.argv[1]) if len(sys.argv) > 1 else 240.0
    seed = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    rnd = random.Random(seed)
    z, _ = TB.load()
    ctx = mosrx.Context(0)
    ctx.set_params(mosrx.default_params())
    t0 = last = time.time()
    sets = frames = 0
    while time.time() - t0 < budget:
        s = rnd.getrandbits(31)
        ps = TB.random_sets(s, nsets=1)[0]
        t = mosrx.Trace(mosrx.TRACE_IMIX, rnd.choice([1, 63, 64, 65, 1000, 4096]), nflows=300, seed=s | 1)
        for buf, off, ln in ((z["frames"], z["off"], z["len"]), (t.frames[:t.frames_bytes], t.off, t.len)):
            want = O.bpf_eval(ps, buf, off, ln)
            for eng in (mosrx.BPF_ENGINE_JIT, mosrx.BPF_ENGINE_INTERP):
                ctx.bpf_set_engine(eng)
                ctx.bpf_set(ps)
                if ctx.bpf_engine() != eng:
                    print(f"FAIL set seed {s}: engine {ctx.bpf_engine()} != {eng}: {ctx.bpf_jit_log()}", flush=True)
                    sys.exit(1)
                got = ctx.bpf_host(buf, off, ln)
                if not np.array_equal(got, want):
                    i = int(np.nonzero(got != want)[0][0])
                    print(f"FAIL set seed {s} engine {eng}: frame {i} mask {got[i]:#x} vs {want[i]:#x}", flush=True)
                    sys.exit(1)
            # one pass: records and masks (the fused kernel, JIT engine)
            ctx.bpf_set_engine(mosrx.BPF_ENGINE_JIT)
            ctx.bpf_set(ps)
            db = ctx.upload(buf, off, ln, frames_bytes=len(buf))
            ctx.classify_bpf_dev(db)
            rec, got = db.results(), db.matches()
            db.free()
            if not np.array_equal(got, want) or \
                    rec.tobytes() != O.classify(buf, off, ln, O.params()).tobytes():
                print(f"FAIL set seed {s}: fused classify + BPF differs", flush=True)
                sys.exit(1)
            frames += len(off)
        sets += 1
        if time.time() - last > 10:
            last = time.time()
            print(f"[soak] {sets} sets, {frames} frames, {last - t0:.0f} s", flush=True)
    print(f"[soak] OK: {sets} random 32-program sets x (JIT, interpreter, fused), {frames} frames in "
          f"{time.time() - t0:.0f} s (seed {seed})", flush=True)


if __name__ == "__main__":
    main()
