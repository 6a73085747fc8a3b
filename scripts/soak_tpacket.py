"""Soak of the TPACKET_V3 ring source lent zero-copy to gpu_module_func
(diagnostic, not a test).

    python3 scripts/soak_tpacket.py [seconds=180] [seed=1]

Random scenarios until the time is up, each over a fresh ring in a memfd
mapping (tests/pktlib.py TpacketRing, the kernel's block layout): 2-12 blocks
of 64 KiB - 1 MiB, a random trace (1 to 4000 frames of random sizes, some
ICMP), a producer that hands over a random number of frames per block as
blocks come back, and a backend with random frames per batch, batches per
launch and pipelining.  Every frame must come out once and in order with the
oracle's record, every pointer must lie in a block that is still lent, and
blocks given back are scribbled over at once (a block recycled while its
frames are exposed would show as a changed frame).  A mismatch prints the
scenario and exits 1.
"""
import ctypes as C
import os
import random
import struct
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mos-networking-stack_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np  # noqa: E402

import mosrx  # noqa: E402
import oracle_py as O  # noqa: E402
from pktlib import TpacketRing, icmp_frame, pack_frames, tcp_frame  # noqa: E402

JUNK = [tcp_frame("1.1.1.1", "2.2.2.2", 1, 1, b"\xEE" * 900)] * 1200


def frames_of(rng, n):
    out = []
    for i in range(n):
        if rng.random() < 0.05:
            out.append(icmp_frame("10.0.0.1", "192.168.0.9", payload=rng.randbytes(rng.randint(0, 100))))
        else:
            out.append(tcp_frame(f"10.0.{i % 200}.{1 + i % 250}", "192.168.0.9", 1000 + i % 5000, 80,
                                 rng.randbytes(rng.choice([0, 6, 100, 536, 1460, rng.randint(0, 1460)])),
                                 seq=i, flags=0x18, tcp_csum=0x1111 if rng.random() < 0.01 else None))
    return out


def scenario(rng):
    nb = rng.randint(2, 12)
    bsz = rng.choice([1 << 16, 1 << 17, 1 << 18, 1 << 20])
    frames = frames_of(rng, rng.choice([1, 2, 50, rng.randint(1, 4000)]))
    ring = TpacketRing(nb, bsz)
    src = mosrx.lib().mosrx_source_tpacket_v3(C.c_void_p(ring.addr), nb, bsz)
    if not src:
        return "source refused the ring"
    if mosrx.afpacket_info(src).zero_copy != 1:
        return "ring not registered (no zero-copy)"
    be = mosrx.GpuBackend([src], batch=rng.choice([1, 16, 100, 256, 2048]), pipeline=rng.random() < 0.7,
                          group=rng.choice([0, 1, 3]))
    try:
        pending, nxt, got, recs, idle = list(frames), 0, [], [], 0
        for _ in range(200000):
            for _k in range(rng.randint(0, 3)):          # the producer: next block in ring order once it is back
                b = nxt % nb
                if not pending or ring.status(b) != 0:
                    break
                take = rng.choice([len(pending), rng.randint(1, len(pending))])
                pending = pending[ring.fill(b, pending[:take]):]
                nxt += 1
            n = be.recv_pkts(0)
            if n < 0:
                return f"recv_pkts {n}"
            if n == 0:
                idle += 1
                if not pending and idle > 30:
                    break
                continue
            idle = 0
            ln = C.c_uint16()
            for i in range(n):
                p = be._rptr(be.ctx, 0, i, C.byref(ln))
                if not ring.addr <= p < ring.addr + nb * bsz:
                    return "a frame pointer outside the ring"
                if ring.status((p - ring.addr) // bsz) != 1:
                    return "a frame exposed from a block already given back"
            got += [be.get_rptr(0, i) for i in range(n)]
            recs.append(be.results(0, n))
            for b2 in range(nb):                         # scribble over every block already given back
                if ring.status(b2) == 0 and b2 != nxt % nb:
                    ring.fill(b2, JUNK)
                    struct.pack_into("<I", ring.m, b2 * bsz + 8, 0)
        if got != frames:
            return f"{len(got)} frames out, {len(frames)} in, or out of order / changed"
        buf, off, ln_ = pack_frames(frames)
        want = O.classify(buf, off, ln_, O.params())
        if np.concatenate(recs).tobytes() != want.tobytes():
            return "records differ from the oracle"
    finally:
        be.close()
        ring.close()
    return None


def main():
    budget = float(sys.argv[1]) if len(sys.argv) > 1 else 180.0
    seed = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    rnd = random.Random(seed)
    t0 = last = time.time()
    count = frames = 0
    while time.time() - t0 < budget:
        s = rnd.getrandbits(31)
        rng = random.Random(s)
        err = scenario(rng)
        if err:
            print(f"FAIL scenario seed {s}: {err}", flush=True)
            sys.exit(1)
        count += 1
        if time.time() - last > 10:
            last = time.time()
            print(f"[soak] {count} ring scenarios, {last - t0:.0f} s", flush=True)
    print(f"[soak] OK: {count} ring scenarios in {time.time() - t0:.0f} s (seed {seed})", flush=True)


if __name__ == "__main__":
    main()
