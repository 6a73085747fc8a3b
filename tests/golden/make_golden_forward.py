"""Generate tests/golden/forward.npz: which frames mOS's OWN ProcessPacket
forwards with mos.conf `forward = 1`, per stack state, on the frames of the
edge / rand_* fixtures (loaded from their .npz, so the inputs are identical).

Run in the build container (needs /root/reference):
    make -C oracle ref && python tests/golden/make_golden_forward.py

oracle/_ref/mosref wraps ForwardIPPacket / ForwardEthernetFrame (-Wl,--wrap)
and records the call as the record's `fwd` instead of transmitting: the
forwarding decision of eth_in.c:60-77, ip_in.c:66-70 / :86-91,
tcp.c:438-442 and the stream engine (tcp.c:453-510, flow table empty at start).
Stored per (fixture, state): verdict (ProcessPacket's return with forward = 1),
fwd, and `have` (bit 3: frame skipped, as in the other fixtures).  Only data.
"""
from __future__ import annotations

import os
import struct
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))

import oracle_py as O  # noqa: E402

FIXTURES = ["edge", "rand_small", "rand_mid", "rand_large"]
LOCAL = ("10.0.0.2", "192.168.1.1", "172.16.9.77")
# (name, num_msp, num_esp, local addresses, end-host listener)
FSTATES = [
    ("msp1", 1, 0, (), False),            # simple_firewall: a monitor socket, forwarding
    ("noverify", 0, 0, (), False),        # no socket at all: ForwardIPPacket before TCP
    ("esp1", 0, 1, (), False),            # end-host client socket only
    ("msp1_esp1", 1, 1, (), False),       # monitor + end-host client socket, no listener
    ("msp1_esp1_listen", 1, 1, (), True),  # monitor + end-host listener: orphans get a RST
    ("msp1_local", 1, 0, LOCAL, False),   # ICMP to the netdevs' addresses is consumed
]


def dst_ports(z) -> set[int]:
    out = set()
    buf = z["frames"]
    for o, n in zip(z["off"].tolist(), z["len"].tolist()):
        f = bytes(buf[o:o + n])
        if n >= 38 and f[12:14] == b"\x08\x00" and f[23] == 6:
            ihl = (f[14] & 0xF) * 4
            if 14 + ihl + 4 <= n:
                out.add(struct.unpack("!H", f[14 + ihl + 2:14 + ihl + 4])[0])
    return out


def main():
    if not O.have_ref():
        sys.exit("oracle/_ref/mosref missing: run `make -C oracle ref` first (needs /root/reference)")
    zs = {fx: np.load(os.path.join(HERE, f"{fx}.npz")) for fx in FIXTURES}
    used = set().union(*(dst_ports(z) for z in zs.values()))
    port = next(p for p in range(1, 65536) if p not in used)   # a port no frame targets
    out = {"listen_port": np.array([port], np.uint16)}
    for fx, z in zs.items():
        for st, msp, esp, loc, listen in FSTATES:
            rec, _ = O.run_ref(z["frames"], z["off"], z["len"], num_msp=msp, num_esp=esp, local=loc, forward=1,
                               listen_port=port if listen else None)
            out[f"{fx}__{st}__verdict"] = np.ascontiguousarray(rec["verdict"])
            out[f"{fx}__{st}__fwd"] = np.ascontiguousarray(rec["fwd"].astype(np.uint8))
            out[f"{fx}__{st}__have"] = np.ascontiguousarray(rec["have"])
            print(f"{fx} {st}: {int(rec['fwd'].sum())} of {len(rec)} forwarded")
    np.savez_compressed(os.path.join(HERE, "forward.npz"), **out)
    print(f"forward.npz: listener port {port}")


if __name__ == "__main__":
    main()
