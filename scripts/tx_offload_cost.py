"""Cost of the backend's TX checksum offload (cfg.tx_csum) per send_pkts
(diagnostic, not a test): a TX batch of `n` frames of `size` bytes written
through get_wptr, every one asking for the IP + TCP checks (mOS's
PKT_TX_*_CSUM ioctls), then send_pkts into a pcap dump on /dev/shm; the same
without the offload (frames sent as written).  Median of 50 batches each.
Usage: python3 scripts/tx_offload_cost.py [n=64] [size=60 1514]"""
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mos-networking-stack_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np  # noqa: E402

import mosrx  # noqa: E402
from pktlib import tcp_frame  # noqa: E402


def run(n, size, offload):
    t = mosrx.Trace(mosrx.TRACE_M1500, 64)
    src = mosrx.mem_source(t.frames, t.off, t.len, loops=1)
    d = tempfile.mkdtemp(dir="/dev/shm" if os.path.isdir("/dev/shm") else None)
    mosrx.source_tx_pcap(src, os.path.join(d, "tx.pcap"))
    be = mosrx.GpuBackend([src], batch=1024, tx_batch=n, tx_csum=offload)
    f = tcp_frame(payload=b"p" * max(0, size - 54))
    ts = []
    try:
        for it in range(60):
            t0 = time.perf_counter()
            for _ in range(n):
                be.send_offloaded(0, f, offload, offload)
            t1 = time.perf_counter()
            be.send_pkts(0)
            t2 = time.perf_counter()
            if it >= 10:
                ts.append((t1 - t0, t2 - t1))
        st = be.stats()
    finally:
        be.close()
    w = np.median([a for a, _ in ts]) * 1e6
    s = np.median([b for _, b in ts]) * 1e6
    return {"n": n, "size": size, "offload": offload, "write_us": round(float(w), 1),
            "send_pkts_us": round(float(s), 1), "offloaded": int(st.tx_csum_offloaded)}


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    sizes = [int(x) for x in sys.argv[2:]] or [60, 1514]
    for size in sizes:
        for off in (False, True):
            print(run(n, size, off), flush=True)


if __name__ == "__main__":
    main()
