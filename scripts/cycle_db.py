"""The drop-in path's group cycle from a rocprofv3 kernel + memory-copy trace
(rocpd SQLite): every GPU operation in start order, grouped into cycles at each
classify launch, and the median duration of each step and of the gaps between
them.  Usage: python3 scripts/cycle_db.py <results.db> [skip_first_n_cycles]"""
import sqlite3
import statistics as st
import sys


def ops(path):
    db = sqlite3.connect(path)
    out = [("K:" + n.split("(")[0].replace("void ", "")[:40], s, e, 0)
           for n, s, e in db.execute("select name, start, end from kernels")]
    out += [("C:" + n + f":{sz}", s, e, sz) for n, s, e, sz in db.execute("select name, start, end, size from memory_copies")]
    return sorted(out, key=lambda r: r[1])


def cycles(path, skip=20):
    o = ops(path)
    cyc, cur = [], []
    for r in o:
        if r[0].startswith("K:mosrx_classify") and cur:
            cyc.append(cur)
            cur = []
        cur.append(r)
    cyc.append(cur)
    return cyc[skip:]


if __name__ == "__main__":
    cs = cycles(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 20)
    steps = {}
    period = []
    for a, b in zip(cs, cs[1:]):
        period.append((b[0][1] - a[0][1]) / 1e3)
    for c in cs:
        t0 = c[0][1]
        for i, (n, s, e, sz) in enumerate(c):
            key = n if not n.startswith("C:") else n.split(":")[0] + ":" + n.split(":")[1] + (":big" if sz > 65536 else ":small")
            steps.setdefault(key, []).append(((s - t0) / 1e3, (e - s) / 1e3))
    print(f"{len(cs)} cycles, launch-to-launch median {st.median(period):.1f} us")
    for k, v in sorted(steps.items(), key=lambda kv: st.median([x[0] for x in kv[1]])):
        print(f"  {k:60s} n={len(v):5d} starts at +{st.median([x[0] for x in v]):8.1f} us, lasts {st.median([x[1] for x in v]):7.1f} us")
