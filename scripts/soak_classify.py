"""Soak of the classify kernels against the oracle (diagnostic, not a test).

    python3 scripts/soak_classify.py [seconds=240] [seed=1] [queue]

Random batches until the time is up: TCP frames with IP / TCP options of every
length, payloads from 0 to ~1500 B, corrupted bytes, bad checksums, wrong
lengths, ICMP to and past local addresses, other ethertypes and protocols,
random garbage with an IPv4 ethertype, captures cut short; packed at random
alignments and gaps or at random (unsorted, overlapping) offsets.  Random
stack state (monitor / end-host sockets, forward, 1-16 queues and both queue
maps, skip_tcp_csum, random or MSDN RSS keys, netdev addresses) and a random
kernel shape (library choice, or SMALL / stream tile forced with either tail
cache policy).  Records, flow hashes and pkt_info fields through the host and
the device paths, and the TX rewrite, must equal the oracle's.  Some batches
are small frames at a fixed stride handed over with a layout hint (right,
right but for moved lanes, wrong, unpackable), in 16- and 8-byte records; the
queue mode mixes them in and runs some queues with 8-byte records.  A mismatch
prints the seed and exits 1.
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
from pktlib import icmp_frame, pack_frames, tcp_frame  # noqa: E402
from test_parity_gpu import ALL_VARIANTS, oparams, run_both  # noqa: E402

LOCAL = ["10.0.0.2", "192.168.1.1", "172.16.0.9"]


def rand_frame(rng):
    r = rng.random()
    ip = lambda: f"{rng.choice([10, 172, 192])}.{rng.randint(0, 255)}.{rng.randint(0, 255)}.{rng.randint(1, 254)}"
    if r < 0.65:
        ihl = 5 if rng.random() < 0.7 else rng.randint(0, 15)
        doff = 5 if rng.random() < 0.6 else rng.randint(0, 15)
        plen = rng.choice([0, 1, 6, 7, 33, 100, 535, 1000, 1448, rng.randint(0, 1460)])
        if rng.random() < 0.01:
            plen = rng.randint(1460, 9000)                          # jumbo
        pl = rng.randbytes(plen)
        kw = {}
        if rng.random() < 0.05:
            kw["tot_len"] = rng.randint(0, 1600)
        if rng.random() < 0.03:
            kw["ip_csum"] = rng.getrandbits(16)
        if rng.random() < 0.03:
            kw["tcp_csum"] = rng.getrandbits(16)
        f = bytearray(tcp_frame(ip(), ip(), rng.getrandbits(16), rng.getrandbits(16), pl,
                                ihl=max(ihl, 5) if rng.random() < 0.9 else ihl, doff=doff,
                                flags=rng.getrandbits(8), seq=rng.getrandbits(32), ack=rng.getrandbits(32),
                                window=rng.getrandbits(16), pad_to=rng.choice([0, 0, 60, 64]), **kw))
        if rng.random() < 0.1:
            f[14] = (f[14] & 0x0F) | (rng.randint(0, 15) << 4)      # version
        if rng.random() < 0.15:                                     # a flipped bit anywhere past the MACs
            f[rng.randint(12, len(f) - 1)] ^= 1 << rng.randint(0, 7)
        return bytes(f)
    if r < 0.75:
        dst = rng.choice(LOCAL) if rng.random() < 0.5 else ip()
        return icmp_frame(ip(), dst, icmp_type=rng.randint(0, 20), payload=bytes(rng.randint(0, 200)),
                          ihl=rng.choice([5, 5, 6, 15]))
    if r < 0.85:
        f = bytearray(tcp_frame(ip(), ip(), 1, 2, b"x" * rng.randint(0, 100), proto=rng.choice([17, 47, 89])))
        return bytes(f)
    if r < 0.92:
        f = bytearray(rng.getrandbits(8) for _ in range(rng.randint(14, 200)))
        f[12:14] = bytes(rng.choice([(0x08, 0x06), (0x86, 0xDD), (0x81, 0x00), (0x88, 0xCC)]))
        return bytes(f)
    f = bytearray(rng.getrandbits(8) for _ in range(rng.randint(0, 300)))
    if len(f) >= 24:
        f[12:14] = b"\x08\x00"
        f[14] = 0x40 | rng.randint(0, 15)
        f[23] = 6
    return bytes(f)


def rand_params(rng):
    key = rng.choice([None, mosrx.MS_KEY, bytes(rng.getrandbits(8) for _ in range(40)),
                      bytes(rng.getrandbits(8) for _ in range(52))])
    kw = dict(num_msp=rng.randint(0, 1), num_esp=rng.randint(0, 1), forward=rng.randint(0, 1),
              num_queues=rng.choice([1, 2, 3, 4, 8, 16]), queue_mode=rng.randint(0, 1),
              skip_tcp_csum=int(rng.random() < 0.1), local=rng.sample(LOCAL, rng.randint(0, 3)))
    if key is not None:
        kw["key"] = key
    return mosrx.default_params(**kw)


def rand_batch(rng):
    """(buf, off, len, packed) of one random batch."""
    fr = [rand_frame(rng) for _ in range(rng.choice([1, 2, 63, 64, 65, 255, 256, 257, rng.randint(1, 3000)]))]
    packed = rng.random() < 0.8
    if packed:
        buf, off, ln = pack_frames(fr, align=rng.choice([1, 2, 4, 16]), phase=rng.randint(0, 15),
                                   gap=rng.choice([0, 0, 3, 64]))
        ln = ln.copy()
        for i in rng.sample(range(len(ln)), k=min(len(ln), rng.randint(0, 5))):
            ln[i] = rng.randint(0, int(ln[i]))                      # captures cut short
    else:                                                           # unsorted / overlapping offsets
        buf, off, ln = pack_frames(fr)
        perm = list(range(len(fr)))
        rng.shuffle(perm)
        off, ln = off[perm].copy(), ln[perm].copy()
        for i in rng.sample(range(len(off)), k=min(len(off), rng.randint(0, 8))):
            off[i] = rng.randint(0, max(0, len(buf) - 1))
    return buf, off, ln, packed


def uniform_batch(rng):
    """(buf, off, len, hint) of a batch of small frames (the SMALL tile's) at a fixed
    stride, some lanes moved elsewhere, with a hint that is right, right for the
    unmoved lanes, wholly wrong, or unpackable."""
    n = rng.choice([1, 2, 255, 256, 257, rng.randint(1, 40_000)])
    ln_ = rng.choice([14, 34, 54, 58, 60, 64, 74, 78])
    stride = rng.choice([ln_, ln_ + 2, 64, 80, 128, 2048]) if ln_ <= 64 else rng.choice([ln_, 80, 128, 2048])
    stride = max(stride, ln_)
    off0 = rng.choice([0, 2, 18, rng.randint(0, 200)])
    moved = rng.sample(range(n), k=min(n, rng.choice([0, 0, 1, 5, 300])))
    buf = np.zeros(off0 + stride * n + 128 * (len(moved) + 1), np.uint8)
    off = (off0 + stride * np.arange(n, dtype=np.int64)).astype(np.uint32)
    lens = np.full(n, ln_, np.uint16)
    for i in range(n):
        f = rand_frame(rng)[:ln_]
        f = f + bytes(ln_ - len(f))
        buf[off[i]:off[i] + ln_] = np.frombuffer(f, np.uint8)
    at = off0 + stride * n + 2
    for i in moved:                          # moved: the hinted address now holds other bytes
        buf[at:at + ln_] = buf[off[i]:off[i] + ln_]
        buf[off[i]:off[i] + ln_] = rng.getrandbits(8)
        off[i] = at
        at += 128
    for i in rng.sample(range(n), k=min(n, rng.randint(0, 3))):
        lens[i] = rng.randint(0, ln_)       # captures cut short
    hint = rng.choice([(off0, stride), (off0, stride), (rng.randint(0, 300), rng.randint(1, 300)),
                       (off0, 0x10000), "auto", None])
    return buf, off, lens, hint


def hint_check(ctx, rng, p):
    """A fixed-stride batch handed over with a layout hint (mosrx_batch.layout):
    16- and 8-byte records through the single launch equal the oracle's."""
    buf, off, ln, hint = uniform_batch(rng)
    ctx.set_params(p)
    want = O.classify(buf, off, ln, oparams(p))
    db = ctx.upload(buf, off, ln, frames_bytes=len(buf), hint=hint)
    try:
        ctx.classify_dev(db)
        if db.results().tobytes() != want.tobytes():
            raise AssertionError(f"hinted batch ({hint}, {len(off)} frames) differs")
        ctx.classify_dev_compact(db)
        r8 = db.results8()
        for f in ("rss", "reason", "queue", "verdict", "tcp_flags"):
            if not np.array_equal(r8[f], want[f]):
                raise AssertionError(f"hinted batch ({hint}): compact {f} differs")
    finally:
        db.free()
    return len(off)


def queue_soak(ctx, rnd, budget):
    """`queue` mode: random batch queues (mosrx_queue_*: one launch over 1-40
    resident batches of different sizes, layouts and frame mixes) against the
    oracle, batch by batch."""
    t0 = last = time.time()
    queues = frames = 0
    while time.time() - t0 < budget:
        s = rnd.getrandbits(31)
        rng = random.Random(s)
        p = rand_params(rng)
        variant = rng.choice(ALL_VARIANTS)
        ctx.set_variant(variant)
        ctx.set_params(p)
        batches = [rand_batch(rng) if rng.random() < 0.7 else uniform_batch(rng)
                   for _ in range(rng.choice([1, 2, 3, 8, rng.randint(1, 40)]))]
        dbs = [ctx.upload(b, o, l, frames_bytes=len(b), hint=x if not isinstance(x, bool) else None)
               for b, o, l, x in batches]
        compact = rng.random() < 0.3                 # 8-byte records (the drop-in path's form)
        q = ctx.queue_ex(dbs, compact=compact)
        q.run()
        for k, ((b, o, l, _), db) in enumerate(zip(batches, dbs)):
            want = O.classify(b, o, l, oparams(p))
            if compact:
                r8 = db.results8()
                ok = all(np.array_equal(r8[f], want[f]) for f in ("rss", "reason", "queue", "verdict", "tcp_flags"))
            else:
                ok = db.results().tobytes() == want.tobytes()
            if not ok:
                print(f"FAIL queue seed {s} variant {variant}: batch {k} of {len(dbs)} differs "
                      f"(compact {compact})", flush=True)
                sys.exit(1)
            frames += len(o)
        q.destroy()
        for db in dbs:
            db.free()
        queues += 1
        if time.time() - last > 10:
            last = time.time()
            print(f"[soak] {queues} queues, {frames} frames, {last - t0:.0f} s", flush=True)
    ctx.set_variant(2)
    print(f"[soak] OK: {queues} random batch queues, {frames} frames in {time.time() - t0:.0f} s", flush=True)


def main():
    budget = float(sys.argv[1]) if len(sys.argv) > 1 else 240.0
    seed = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    if len(sys.argv) > 3 and sys.argv[3] == "queue":
        return queue_soak(mosrx.Context(0), random.Random(seed), budget)
    rnd = random.Random(seed)
    ctx = mosrx.Context(0)
    t0 = last = time.time()
    batches = frames = 0
    while time.time() - t0 < budget:
        s = rnd.getrandbits(31)
        rng = random.Random(s)
        fr = [rand_frame(rng) for _ in range(rng.choice([1, 2, 63, 64, 65, 255, 256, 257, rng.randint(1, 3000)]))]
        packed = rng.random() < 0.8
        if packed:
            buf, off, ln = pack_frames(fr, align=rng.choice([1, 2, 4, 16]), phase=rng.randint(0, 15),
                                       gap=rng.choice([0, 0, 3, 64]))
            ln = ln.copy()
            for i in rng.sample(range(len(ln)), k=min(len(ln), rng.randint(0, 5))):
                ln[i] = rng.randint(0, int(ln[i]))                  # captures cut short
        else:                                                       # unsorted / overlapping offsets
            buf, off, ln = pack_frames(fr)
            perm = list(range(len(fr)))
            rng.shuffle(perm)
            off, ln = off[perm].copy(), ln[perm].copy()
            for i in rng.sample(range(len(off)), k=min(len(off), rng.randint(0, 8))):
                off[i] = rng.randint(0, max(0, len(buf) - 1))
        p = rand_params(rng)
        variant = rng.choice(ALL_VARIANTS)
        try:
            ctx.set_variant(variant)
            run_both(ctx, buf, off, ln, p, side=True)
            if rng.random() < 0.3:          # a fixed-stride batch of small frames with a layout hint
                frames += hint_check(ctx, rng, p)
            # the TX rewrite of frames that overlap depends on the order they are written in
            if rng.random() < 0.3 and packed:
                fl = rng.choice([mosrx.TX_IP_CSUM, mosrx.TX_TCP_CSUM, mosrx.TX_IP_CSUM | mosrx.TX_TCP_CSUM])
                got = ctx.tx_csum_host(buf, off, ln, fl)
                if not np.array_equal(got, O.tx_csum(buf, off, ln, fl)):
                    raise AssertionError("TX rewrite differs")
        except AssertionError as e:
            print(f"FAIL batch seed {s} variant {variant}: {str(e)[:1500]}", flush=True)
            sys.exit(1)
        batches += 1
        frames += len(fr)
        if time.time() - last > 10:
            last = time.time()
            print(f"[soak] {batches} batches, {frames} frames, {last - t0:.0f} s", flush=True)
    ctx.set_variant(2)
    print(f"[soak] OK: {batches} random batches, {frames} frames in {time.time() - t0:.0f} s (seed {seed})",
          flush=True)


if __name__ == "__main__":
    main()
