"""Soak of gpu_module_func against the oracle (diagnostic, not a test).

    python3 scripts/soak_backend.py [seconds=90] [seed=1]

Random scenarios until the time is up, each a fresh backend over an in-memory
source: trace kind and size, frames per batch, batches per launch (auto or
1..8; auto groups of random byte budgets), pipelining, how the source hands
frames over (lent / runs / frame by frame), replays, 16- or 8-byte records
(cfg.compact), pkt_info and flow-hash side arrays, and stack-state changes
(num_msp / num_esp / forward through dev_ioctl(MOSRX_PKT_SET_PARAMS)) at
random points between recv_pkts calls.  Every batch handed out must equal the
oracle's records (and side arrays) for its frames under the state in effect
at the recv_pkts that handed it out -- batches classified earlier under
another state are classified again by the backend.  A mismatch prints the
scenario and exits 1.  Prints a progress line every ~10 s.
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

KINDS = [mosrx.TRACE_IMIX, mosrx.TRACE_M1500, mosrx.TRACE_S64, mosrx.TRACE_FW64]


def oparams(p):
    q = O.Params()
    for f, _ in mosrx.Params._fields_:
        setattr(q, f, getattr(p, f))
    return q


def scenario(rnd):
    kind = rnd.choice(KINDS)
    n = rnd.choice([1, 2, 63, 64, 65, 255, 256, 257, rnd.randint(1, 3000), rnd.randint(1000, 20000)])
    return dict(kind=kind, n=n, nflows=rnd.choice([1, 17, 300, 5000]), seed=rnd.randint(1, 1 << 30),
                batch=rnd.choice([1, 7, 64, 255, 256, 1024, rnd.randint(1, 4096)]),
                group=rnd.choice([0, 0, 1, 2, 3, 8]), pipeline=rnd.random() < 0.7,
                mode=rnd.choice([mosrx.SRC_BEST, mosrx.SRC_FILL, mosrx.SRC_PER_FRAME]),
                loops=rnd.choice([1, 1, 2, 3]), tcpinfo=rnd.random() < 0.3, flowhash=rnd.random() < 0.3,
                toggle=rnd.choice([0.0, 0.0, 0.1, 0.5]), fwd=rnd.randint(0, 1),
                compact=rnd.random() < 0.4,
                group_bytes=rnd.choice([0, 0, 1 << 16, 1 << 20, 16 << 20]))


def run(sc, rnd):
    t = mosrx.Trace(sc["kind"], sc["n"], nflows=sc["nflows"], seed=sc["seed"])
    p = mosrx.default_params(forward=sc["fwd"])
    src = mosrx.mem_source(t.frames, t.off, t.len, loops=sc["loops"], mode=sc["mode"])
    compact = sc["compact"] and not sc["tcpinfo"]     # (the module refuses compact records with pkt_info)
    be = mosrx.GpuBackend([src], params=p, batch=sc["batch"], pipeline=sc["pipeline"], cpu=rnd.randint(0, 7),
                          group=sc["group"], tcpinfo=sc["tcpinfo"], flowhash=sc["flowhash"], compact=compact,
                          group_bytes=sc["group_bytes"])
    cache = {}

    def ora(state):
        if state not in cache:
            q = mosrx.default_params(num_msp=state[0], num_esp=state[1], forward=state[2])
            cache[state] = O.classify_ex(t.frames[:t.frames_bytes], t.off, t.len, oparams(q))
        return cache[state]

    state = (1, 0, sc["fwd"])
    seen = batches = 0
    try:
        while True:
            if sc["toggle"] and rnd.random() < sc["toggle"]:
                state = (rnd.randint(0, 1), rnd.randint(0, 1), state[2])
                q = mosrx.default_params(num_msp=state[0], num_esp=state[1], forward=state[2])
                if be.set_params(0, q):
                    return f"SET_PARAMS failed at batch {batches}"
            n = be.recv_pkts(0)
            if n < 0:
                return f"recv_pkts {n} at batch {batches}"
            if n == 0:
                break
            idx = (seen + np.arange(n)) % t.n
            rec, fh, ti = ora(state)
            if compact:
                got8 = be.results8(0, n)
                for f in ("rss", "reason", "queue", "verdict", "tcp_flags"):
                    if not np.array_equal(got8[f], rec[idx][f]):
                        return f"8-byte records' {f} differ at batch {batches} (frames {seen}..), state {state}"
                got = None
            else:
                got = be.results(0, n)
            if got is not None and got.tobytes() != rec[idx].tobytes():
                i = int(np.nonzero(np.any(got.view(np.uint8).reshape(-1, 16) !=
                                          rec[idx].view(np.uint8).reshape(-1, 16), axis=1))[0][0])
                return f"records differ at batch {batches} (frames {seen}..), first {i}: {got[i]} vs {rec[idx][i]}, state {state}"
            if sc["tcpinfo"] and be.tcpinfo(0, n).tobytes() != ti[idx].tobytes():
                return f"pkt_info differs at batch {batches}"
            if sc["flowhash"] and not np.array_equal(be.fhashes(0, n), fh[idx]):
                return f"flow hashes differ at batch {batches}"
            j = int(idx[-1])
            if be.get_rptr(0, n - 1) != bytes(t.frames[t.off[j]:t.off[j] + t.len[j]]):
                return f"get_rptr frame differs at batch {batches}"
            seen += n
            batches += 1
        if seen != sc["loops"] * t.n:
            return f"{seen} frames handed out, {sc['loops'] * t.n} expected"
        st = be.stats()
        if st.rx_frames != seen or st.rx_drops:
            return f"stats rx_frames {st.rx_frames} rx_drops {st.rx_drops}"
    finally:
        be.close()
    return None


def main():
    budget = float(sys.argv[1]) if len(sys.argv) > 1 else 90.0
    seed = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    rnd = random.Random(seed)
    t0 = last = time.time()
    count = frames = 0
    while time.time() - t0 < budget:
        sc = scenario(rnd)
        err = run(sc, rnd)
        if err:
            print(f"FAIL scenario {count}: {sc}: {err}", flush=True)
            sys.exit(1)
        count += 1
        frames += sc["n"] * sc["loops"]
        if time.time() - last > 10:
            last = time.time()
            print(f"[soak] {count} scenarios, {frames} frames, {last - t0:.0f} s", flush=True)
    print(f"[soak] OK: {count} scenarios, {frames} frames in {time.time() - t0:.0f} s (seed {seed})", flush=True)


if __name__ == "__main__":
    main()
