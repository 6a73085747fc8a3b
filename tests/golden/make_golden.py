"""Generate the golden vectors in tests/golden/ from mOS's OWN compiled rx path.

Run in the build container (needs /root/reference):
    make -C oracle ref && python tests/golden/make_golden.py

For every fixture trace it runs oracle/_ref/mosref (core/src objects compiled
from /root/reference by oracle/ref.mk + oracle/ref_harness.c) under several
stack states and stores inputs and the reference's outputs as .npz data:
  verdict  = ProcessPacket() return (eth_in.c:27)
  ip_csum  = ip_fast_csum(iph, ihl) (include/ip_in.h:10)
  tcp_csum = TCPCalcChecksum(...)   (tcp_util.c:157)
  rss      = GetRSSHash(ntohl(saddr), ntohl(daddr), ntohs(sp), ntohs(dp)) (util.c:61)
  queue    = GetRSSCPUCore(...)     (util.c:114, FetchEndianType wrapped for ixgbe)
  fbucket  = HashFlow(&FindStream's reversed tuple) (fhash.c:72, tcp.c:185-190)
  have     = which of those the harness computed (bit3: frame skipped, bit4: fbucket)
plus the NETSTAT rx counters.  The MSDN Toeplitz KAT (util/rss.c:177-193) is
stored as its own fixture.  Nothing here is reference source: only data.
"""
from __future__ import annotations

import os
import random
import struct
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))

from pktlib import ETH_ARP, REF_FIELDS, icmp_frame, pack_frames, tcp_frame  # noqa: E402
import oracle_py as O  # noqa: E402

# the netdevs' addresses of the "local" states (netdev_table entries: ICMP to them is "to me")
LOCAL = ("10.0.0.2", "192.168.1.1", "172.16.9.77")
STATES = [  # (name, num_msp, num_esp, num_queues, queue_mode, local addresses)
    ("msp1", 1, 0, 1, 1, ()),
    ("noverify", 0, 0, 1, 1, ()),
    ("esp1", 0, 1, 1, 1, ()),
    ("q2_i40e", 1, 0, 2, 1, ()),
    ("q4_i40e", 1, 0, 4, 1, ()),
    ("q8_i40e", 1, 0, 8, 1, ()),
    ("q3_ixgbe", 1, 0, 3, 0, ()),
    ("q8_ixgbe", 1, 0, 8, 0, ()),
    ("msp1_local", 1, 0, 1, 1, LOCAL),
    ("esp1_local", 0, 1, 4, 1, LOCAL),
    ("noverify_local", 0, 0, 1, 1, LOCAL),
]


def edge_frames() -> list[bytes]:
    """Hand-made frames for the edges listed in SURVEY.md §8a."""
    f = []
    f.append(tcp_frame(payload=b"abcdef"))                              # valid 64B-class
    f.append(tcp_frame(payload=b"abcde"))                               # odd length valid
    odd = bytearray(tcp_frame(payload=b"abcde")); odd[-1] ^= 0x40
    f.append(bytes(odd))                                                # odd payload corrupted
    f.append(tcp_frame(payload=b"abcde", pad_to=60))                    # odd, byte after end = 0
    odd2 = bytearray(tcp_frame(payload=b"abcde", pad_to=60)); odd2[14 + 45] = 0x77
    f.append(bytes(odd2))                                               # byte after odd end changed
    th = bytearray(tcp_frame(payload=b"xyz!")); th[14 + 20 + 4] ^= 1
    f.append(bytes(th))                                                 # TCP header corrupted
    for ihl in range(0, 5):
        f.append(tcp_frame(ihl=ihl, pad_to=60))                         # ihl 0..4 quirk
    f.append(tcp_frame(version=6))
    f.append(tcp_frame(tot_len=19, pad_to=60))
    f.append(tcp_frame(tot_len=0, pad_to=60))
    f.append(tcp_frame(tot_len=20, pad_to=60))
    f.append(tcp_frame(tot_len=39, pad_to=60))
    f.append(tcp_frame(proto=17, payload=b"udpudpudp"))
    f.append(tcp_frame(proto=17, payload=b"udp", ip_csum=0x1234))       # UDP bad IP csum
    f.append(tcp_frame(proto=1, payload=b"\x08\x00icmp"))               # ICMP, no local IP
    f.append(tcp_frame(ip_csum=0xBEEF))                                 # bad IP checksum
    f.append(tcp_frame(ethertype=ETH_ARP, pad_to=60))
    f.append(tcp_frame(ethertype=0x86DD, pad_to=60))
    f.append(tcp_frame(ethertype=0x8100, pad_to=60))
    f.append(tcp_frame(doff=4))
    f.append(tcp_frame(doff=0))
    f.append(tcp_frame(doff=15, tot_len=46, pad_to=100))
    f.append(tcp_frame(ihl=6, payload=b"opts"))
    f.append(tcp_frame(ihl=15, payload=b"maxopts"))
    f.append(tcp_frame(ihl=15, doff=15, payload=b"both max"))
    v = tcp_frame(payload=b"complement")
    vv = bytearray(v); c = struct.unpack("!H", vv[14 + 20 + 16:14 + 20 + 18])[0]
    vv[14 + 20 + 16:14 + 20 + 18] = struct.pack("!H", (~c) & 0xFFFF)
    f.append(bytes(vv))                                                 # TCP check complemented
    big = tcp_frame(payload=bytes(range(256)) * 5 + bytes(168), doff=8)
    f.append(big)                                                       # 1514 B valid
    bb = bytearray(big); bb[700] ^= 0x10
    f.append(bytes(bb))                                                 # one payload bit flipped
    sw = bytearray(big); sw[600:602], sw[602:604] = sw[602:604], sw[600:602]
    f.append(bytes(sw))                                                 # two aligned words swapped
    pad = bytearray(tcp_frame(payload=b"ab", pad_to=60)); pad[58] = 0xAA
    f.append(bytes(pad))                                                # Ethernet pad byte corrupted
    f.append(tcp_frame(payload=bytes(1), flags=0x02))                   # SYN, 1 byte
    f.append(tcp_frame(src="255.255.255.255", dst="255.255.255.255", sport=65535, dport=65535))
    f.append(tcp_frame(src="0.0.0.0", dst="0.0.0.0", sport=0, dport=0))
    # ip_fast_csum carry-chain corner: header words summing to 0 / 0xFFFF classes
    f.append(tcp_frame(src="255.255.255.255", dst="255.255.255.255", tos=0xFF, ip_id=0xFFFF, ttl=255))
    # ICMP (ip_in.c:83-85, icmp.c:187-227): to a local address in the *_local states, else not
    f.append(icmp_frame(dst="10.0.0.2", icmp_type=8, payload=b"echo request"))      # echo request
    f.append(icmp_frame(dst="192.168.1.1", icmp_type=0))                           # echo reply
    f.append(icmp_frame(dst="172.16.9.77", icmp_type=3, code=1))                   # dest unreachable
    f.append(icmp_frame(dst="172.16.9.77", icmp_type=11))                          # time exceeded
    f.append(icmp_frame(dst="10.0.0.2", icmp_type=42))                             # unsupported type
    f.append(icmp_frame(dst="10.0.0.2", icmp_type=8, icmp_csum=0xDEAD))            # echo, bad ICMP csum
    f.append(icmp_frame(dst="10.0.0.2", icmp_type=8, ip_csum=0x1111))              # bad IP csum first
    f.append(icmp_frame(dst="10.0.0.2", icmp_type=8, ihl=7, payload=b"opts"))      # IP options
    f.append(icmp_frame(dst="10.0.0.3", icmp_type=8))                              # not local
    f.append(icmp_frame(src="10.0.0.2", dst="10.9.9.9", icmp_type=8))              # local source only
    f.append(icmp_frame(dst="192.168.1.1", icmp_type=8, payload=b"", pad_to=60))   # padded minimum
    f.append(tcp_frame(proto=17, dst="10.0.0.2", payload=b"udp to me"))            # UDP to a local address
    f.append(tcp_frame(dst="192.168.1.1", payload=b"tcp to me"))                   # TCP to a local address
    return f


def random_frames(rng: random.Random, n: int, size_class: int) -> list[bytes]:
    """Valid frames with random mutations of every header field the path reads."""
    out = []
    for _ in range(n):
        if size_class == 0:
            plen = rng.randint(0, 26)
        elif size_class == 1:
            plen = rng.randint(400, 560)
        else:
            plen = rng.randint(1300, 1460)
        ihl = 5 if rng.random() < 0.7 else rng.randint(5, 15)
        doff = 5 if rng.random() < 0.5 else rng.randint(5, 15)
        ip = lambda: ".".join(str(rng.randint(0, 255)) for _ in range(4))  # noqa: E731
        fr = bytearray(tcp_frame(ip(), ip(), rng.randint(0, 65535), rng.randint(0, 65535),
                                 bytes(rng.getrandbits(8) for _ in range(plen)), ihl=ihl, doff=doff,
                                 flags=rng.choice([0x02, 0x10, 0x18, 0x11, 0x04]),
                                 seq=rng.getrandbits(32), ack=rng.getrandbits(32),
                                 window=rng.getrandbits(16), ip_id=rng.getrandbits(16),
                                 tos=rng.getrandbits(8), ttl=rng.randint(1, 255)))
        m = rng.random()
        tot = len(fr) - 14
        if m < 0.25:
            pass                                                       # valid
        elif m < 0.35:
            fr[rng.randint(14 + ihl * 4, len(fr) - 1)] ^= 1 << rng.randint(0, 7)   # payload flip
        elif m < 0.42:
            fr[rng.randint(14, 14 + ihl * 4 - 1)] ^= 1 << rng.randint(0, 7)        # IP header flip
        elif m < 0.50:                                                 # shorter tot_len (Ethernet pad)
            nt = rng.randint(0, tot)
            fr[16:18] = struct.pack("!H", nt)
        elif m < 0.56:
            fr[14] = (fr[14] & 0xF0) | rng.randint(0, 15)              # ihl
        elif m < 0.62:
            fr[14] = (rng.randint(0, 15) << 4) | (fr[14] & 0xF)        # version
        elif m < 0.68:
            fr[14 + ihl * 4 + 12] = (rng.randint(0, 15) << 4) | (fr[14 + ihl * 4 + 12] & 0xF)  # doff
        elif m < 0.72:
            fr[23] = rng.choice([1, 17, 47, 0, 255])                   # protocol
        elif m < 0.76:
            fr[12:14] = struct.pack("!H", rng.choice([0x0806, 0x86DD, 0x8100, 0x0000, 0x0801]))
        elif m < 0.88:                                                 # fix up IP csum after a field change
            nt = rng.randint(20, tot)
            fr[16:18] = struct.pack("!H", nt)
            fr[24:26] = b"\0\0"
            from pktlib import csum16
            fr[24:26] = struct.pack("!H", csum16(bytes(fr[14:14 + ihl * 4])))
        else:
            fr[14 + ihl * 4 + 16] ^= rng.getrandbits(8)                # TCP check field
        if rng.random() < 0.1:
            fr += bytes(rng.getrandbits(8) for _ in range(rng.randint(1, 9)))  # trailing bytes in caplen
        out.append(bytes(fr))
    return out


def run_states(frames: list[bytes], name: str, phase: int = 2):
    buf, off, ln = pack_frames(frames, phase=phase)
    res = {}
    for st, msp, esp, nq, qm, loc in STATES:
        rec, stats = O.run_ref(buf, off, ln, num_msp=msp, num_esp=esp, num_queues=nq, queue_mode=qm, local=loc)
        res[st] = rec
        res[st + "_stats"] = np.array([stats["rx_packets"], stats["rx_bytes"], stats["rx_errors"]],
                                      np.uint64)
    out = {"frames": buf, "off": off, "len": ln}
    for st, *_ in STATES:
        r = res[st]
        for fld in REF_FIELDS:
            out[f"{st}__{fld}"] = np.ascontiguousarray(r[fld])
        out[f"{st}__stats"] = res[st + "_stats"]
    np.savez_compressed(os.path.join(HERE, f"{name}.npz"), **out)
    print(f"{name}: {len(frames)} frames, {len(buf)} bytes")


def tx_fixture(frames: list[bytes], name: str, phase: int):
    """TX checksum rewrite vectors (mos_api.c:1177-1193).  The check fields are
    zeroed first, as mtcp_setlastpkt does, and mOS's compiled path is run on
    those frames: its ip_fast_csum / TCPCalcChecksum outputs are exactly the
    values the rewrite stores.  Stored per frame: whether each check is
    rewritten and the reference's value; the inputs keep their old checks."""
    buf, off, ln = pack_frames(frames, phase=phase)
    z = buf.copy()
    for o, n in zip(off.tolist(), ln.tolist()):
        f = z[o:o + n]
        if n < 34 or f[12] != 0x08 or f[13] != 0x00 or (f[14] & 0xF) < 5:
            continue
        ihl = f[14] & 0xF
        f[24:26] = 0
        if f[23] == 6 and 14 + ihl * 4 + 18 <= n:
            f[14 + ihl * 4 + 16:14 + ihl * 4 + 18] = 0
    rec, _ = O.run_ref(z, off, ln, num_msp=1)
    ihl = np.array([z[o + 14] & 0xF if n > 14 else 0 for o, n in zip(off.tolist(), ln.tolist())])
    ipv4 = np.array([n >= 34 and z[o + 12] == 8 and z[o + 13] == 0 for o, n in zip(off.tolist(), ln.tolist())])
    live = (rec["have"] & 8) == 0
    ip_w = live & ipv4 & (ihl >= 5)
    tcp_w = ip_w & ((rec["have"] & 2) != 0)
    np.savez_compressed(os.path.join(HERE, f"{name}.npz"), frames=buf, off=off, len=ln,
                        ip_w=ip_w, ip_check=rec["ip_csum"], tcp_w=tcp_w, tcp_check=rec["tcp_csum"])
    print(f"{name}: {len(frames)} frames, {ip_w.sum()} IP / {tcp_w.sum()} TCP rewrites")


def short_segment_frames():
    """TCP frames whose tot_len leaves the segment shorter than a TCP header
    (doff < 5 passes mOS's length check, tcp.c:429-430): tcph->check then lies
    past the ip_len - ihl*4 bytes TCPCalcChecksum covers, wholly (segment <= 16
    bytes) or by its second byte (17).  Captures run past tot_len, so the check
    field itself is captured and written."""
    rng = random.Random(0x5E6)
    frames = []
    for seglen in range(12, 24):
        for doff in range(0, 6):
            if (5 + doff) * 4 > 20 + seglen:
                continue
            for odd in (0, 1):
                pl = bytes(rng.getrandbits(8) for _ in range(rng.choice([0, 7, 30])))
                frames.append(tcp_frame(payload=pl, doff=doff, tot_len=20 + seglen, seq=rng.getrandbits(32),
                                        flags=rng.getrandbits(8), pad_to=60 + 3 * odd))
    return frames


def main():
    if not O.have_ref():
        sys.exit("oracle/_ref/mosref missing: run `make -C oracle ref` first (needs /root/reference)")
    rng = random.Random(0x6D4F5321)
    run_states(edge_frames(), "edge")
    run_states(random_frames(rng, 256, 0), "rand_small")
    run_states(random_frames(rng, 256, 1), "rand_mid", phase=7)   # odd frame starts: byte-swap path
    run_states(random_frames(rng, 256, 2), "rand_large")
    txr = random.Random(0x7C5)
    tx_fixture(edge_frames() + random_frames(txr, 200, 0) + random_frames(txr, 100, 1), "tx_mixed", phase=2)
    tx_fixture(random_frames(txr, 120, 2) + random_frames(txr, 60, 0), "tx_odd", phase=7)
    tx_fixture(short_segment_frames(), "tx_short", phase=3)   # round 3: check field past the segment
    # MSDN Toeplitz vectors (util/rss.c:177-193), Microsoft key (util/rss.c:75-81)
    kat = np.array([
        (0x420995bb, 0xa18e6450, 2794, 1766, 0x51ccc178),
        (0xc75c6f02, 0x41458c53, 14230, 4739, 0xc626b0ea),
        (0x1813c65f, 0x0c16cfb8, 12898, 38024, 0x5c2b394a),
        (0x261bcd1e, 0xd18ea306, 48228, 2217, 0xafc7327f),
        (0x9927a3bf, 0xcabc7f02, 44251, 1303, 0x10e828a2),
    ], dtype=[("sip", "<u4"), ("dip", "<u4"), ("sp", "<u2"), ("dp", "<u2"), ("hash", "<u4")])
    np.savez_compressed(os.path.join(HERE, "rss_msdn_kat.npz"), kat=kat,
                        key=np.frombuffer(O.MS_KEY, np.uint8))
    print("rss_msdn_kat: 5 vectors")


if __name__ == "__main__":
    main()
