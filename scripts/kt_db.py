"""Per-dispatch kernel durations from a rocprofv3 kernel-trace database
(rocpd SQLite, ROCm 7's default output): for each kernel name matching a
pattern, the count and the median / mean duration of its last N dispatches.
Usage: python3 scripts/kt_db.py <results.db> [pattern] [last_n]"""
import sqlite3
import statistics as st
import sys


def dispatches(path, pattern="classify"):
    db = sqlite3.connect(path)
    rows = db.execute("select name, start, end from kernels order by start").fetchall()
    return [(n, s, e) for n, s, e in rows if pattern in n]


def summary(path, pattern="classify", last=None):
    out = {}
    for n, s, e in dispatches(path, pattern):
        out.setdefault(n, []).append((e - s) / 1e3)
    res = {}
    for n, d in out.items():
        d = d[-last:] if last else d
        res[n] = {"n": len(d), "median_us": round(st.median(d), 3), "mean_us": round(st.mean(d), 3),
                  "min_us": round(min(d), 3), "max_us": round(max(d), 3)}
    return res


if __name__ == "__main__":
    p = sys.argv[2] if len(sys.argv) > 2 else "classify"
    last = int(sys.argv[3]) if len(sys.argv) > 3 else None
    for n, r in summary(sys.argv[1], p, last).items():
        print(f"{n[:70]:70s} {r}")
