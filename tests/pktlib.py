"""Frame construction and trace (de)serialisation helpers for the tests.

Pure Python, standard RFC 1071 arithmetic written independently of both the
HIP kernels and the oracle, used only to BUILD input frames (valid or
deliberately broken).  Expected outputs always come from the oracle / the
reference harness, never from this file.
"""
from __future__ import annotations

import struct

import numpy as np

ETH_IP = 0x0800
ETH_ARP = 0x0806
RESULT_DTYPE = np.dtype([
    ("rss", "<u4"), ("ip_csum", "<u2"), ("tcp_csum", "<u2"), ("payloadlen", "<u2"),
    ("payload_off", "u1"), ("verdict", "i1"), ("reason", "u1"), ("queue", "u1"),
    ("tcp_flags", "u1"), ("ihl_doff", "u1"),
])
assert RESULT_DTYPE.itemsize == 16

R = dict(TCP_OK=0, ARP=1, NON_IPV4=2, IP_SHORT=3, IP_BADVER=4, NOVERIFY_PASS=5, IP_BADCSUM=6,
         NOT_TCP=7, TCP_SHORT=8, TCP_BADCSUM=9, TRUNCATED=10, TCP_LEN_OK=11, ICMP_LOCAL=12)
NREASON = len(R)


def csum16(data: bytes) -> int:
    """RFC 1071 one's-complement checksum of big-endian 16-bit words."""
    if len(data) % 2:
        data = data + b"\0"
    s = sum(struct.unpack("!%dH" % (len(data) // 2), data))
    while s >> 16:
        s = (s & 0xFFFF) + (s >> 16)
    return (~s) & 0xFFFF


def ip4(a: str) -> bytes:
    return bytes(int(x) for x in a.split("."))


def tcp_frame(src="10.0.0.1", dst="10.0.0.2", sport=1234, dport=80, payload=b"", *,
              ihl=5, doff=5, flags=0x10, seq=1, ack=1, window=65535, ttl=64, ip_id=0,
              proto=6, version=4, tot_len=None, ip_opts=None, tcp_opts=None,
              ip_csum=None, tcp_csum=None, pad_to=0, ethertype=ETH_IP, tos=0) -> bytes:
    """Build an Ethernet/IPv4/TCP frame.  Checksums are valid unless overridden."""
    ip_opts = ip_opts if ip_opts is not None else b"\x01" * (ihl * 4 - 20 if ihl > 5 else 0)
    tcp_opts = tcp_opts if tcp_opts is not None else b"\x01" * (doff * 4 - 20 if doff > 5 else 0)
    tcph_wo = struct.pack("!HHIIBBHHH", sport, dport, seq, ack, (doff & 0xF) << 4, flags, window, 0, 0)
    seg = tcph_wo + tcp_opts + payload
    hdr_len = 20 + len(ip_opts)
    if tot_len is None:
        tot_len = hdr_len + len(seg)
    s, d = ip4(src), ip4(dst)
    iph = struct.pack("!BBHHHBBH4s4s", ((version & 0xF) << 4) | (ihl & 0xF), tos, tot_len & 0xFFFF,
                      ip_id & 0xFFFF, 0x4000, ttl, proto, 0, s, d) + ip_opts
    if ip_csum is None:
        ip_csum = csum16(iph)
    iph = iph[:10] + struct.pack("!H", ip_csum) + iph[12:]
    if proto == 6 and tcp_csum is None:
        pseudo = s + d + struct.pack("!BBH", 0, 6, len(seg))
        tcp_csum = csum16(pseudo + seg)
    if proto == 6:
        seg = seg[:16] + struct.pack("!H", tcp_csum) + seg[18:]
    eth = b"\x02\x00\x00\x00\x00\x02" + b"\x02\x00\x00\x00\x00\x01" + struct.pack("!H", ethertype)
    frame = eth + iph + seg
    if len(frame) < pad_to:
        frame += b"\0" * (pad_to - len(frame))
    return frame


def icmp_frame(src="10.0.0.1", dst="10.0.0.2", icmp_type=8, code=0, payload=b"ping", *, ihl=5,
               ip_csum=None, icmp_csum=None, tot_len=None, pad_to=0) -> bytes:
    """Build an Ethernet/IPv4/ICMP frame (echo-style header: type, code, check, id, seq)."""
    ip_opts = b"\x01" * (ihl * 4 - 20 if ihl > 5 else 0)
    body = struct.pack("!BBHHH", icmp_type, code, 0, 0x1234, 7) + payload
    if icmp_csum is None:
        icmp_csum = csum16(body)
    body = body[:2] + struct.pack("!H", icmp_csum) + body[4:]
    if tot_len is None:
        tot_len = 20 + len(ip_opts) + len(body)
    iph = struct.pack("!BBHHHBBH4s4s", 0x40 | (ihl & 0xF), 0, tot_len & 0xFFFF, 0, 0x4000, 64, 1, 0,
                      ip4(src), ip4(dst)) + ip_opts
    if ip_csum is None:
        ip_csum = csum16(iph)
    iph = iph[:10] + struct.pack("!H", ip_csum) + iph[12:]
    eth = b"\x02\x00\x00\x00\x00\x02" + b"\x02\x00\x00\x00\x00\x01" + struct.pack("!H", ETH_IP)
    frame = eth + iph + body
    if len(frame) < pad_to:
        frame += b"\0" * (pad_to - len(frame))
    return frame


def pack_frames(frames: list[bytes], align: int = 16, phase: int = 2, gap: int = 0):
    """Pack frames into one buffer; frame i starts at a multiple of `align` plus `phase`.

    Returns (buf: uint8[], off: uint32[], len: uint16[]).  The buffer gets 64 zero
    bytes of tail padding (the reference's masked odd-tail read may touch one byte
    past a frame).
    """
    offs, pos = [], phase
    for f in frames:
        offs.append(pos)
        pos += len(f) + gap
        if align > 1:
            pos = ((pos - phase + align - 1) // align) * align + phase
    buf = np.zeros(pos + 64, np.uint8)
    for o, f in zip(offs, frames):
        buf[o:o + len(f)] = np.frombuffer(f, np.uint8)
    return buf, np.asarray(offs, np.uint32), np.asarray([len(f) for f in frames], np.uint16)


def write_ref_trace(path, buf, off, ln, *, num_msp=1, num_esp=0, forward=0, num_queues=1,
                    queue_mode=1, local=()):
    """Trace file consumed by oracle/_ref/mosref (format in oracle/ref_harness.c, version 2:
    `local` = raw u32 netdev addresses)."""
    loc = list(local) + [0] * (16 - len(local))
    with open(path, "wb") as fh:
        fh.write(b"MRXT" + struct.pack("<IIQIIiii", 2, len(off), len(buf), num_msp, num_esp,
                                       forward, num_queues, queue_mode))
        fh.write(struct.pack("<I16I", len(local), *loc))
        fh.write(np.asarray(off, "<u4").tobytes())
        fh.write(np.asarray(ln, "<u2").tobytes())
        fh.write(np.asarray(buf, np.uint8).tobytes())


REF_DTYPE = np.dtype([("verdict", "i1"), ("have", "u1"), ("ip_csum", "<u2"), ("tcp_csum", "<u2"),
                      ("fwd", "<u2"), ("rss", "<u4"), ("queue", "<i4"), ("fbucket", "<u4"),
                      ("payloadlen", "<u2"), ("payload_off", "<u2"), ("seq", "<u4"), ("ack_seq", "<u4"),
                      ("window", "<u2"), ("tcp_flags", "u1"), ("ihl_doff", "u1"), ("ip_len", "<u2"),
                      ("pad2", "<u2")])
assert REF_DTYPE.itemsize == 40
# fields stored per stack state in the golden fixtures (fbucket = HashFlow bucket, have bit 4;
# payloadlen .. ihl_doff = mOS's FillPacketContextTCPInfo output, have bit 5)
REF_FIELDS = ("verdict", "have", "ip_csum", "tcp_csum", "rss", "queue", "fbucket",
              "payloadlen", "payload_off", "seq", "ack_seq", "window", "tcp_flags", "ihl_doff", "ip_len")


def read_ref_results(path, n):
    raw = open(path, "rb").read()
    sz = REF_DTYPE.itemsize
    rec = np.frombuffer(raw[: n * sz], REF_DTYPE)
    stats = struct.unpack("<QQQ", raw[n * sz: n * sz + 24])
    return rec, dict(rx_packets=stats[0], rx_bytes=stats[1], rx_errors=stats[2])


def conversation_frames(nflows: int = 64, seed: int = 7, *, listen_port: int = 0, local_ip: str = "127.0.0.1"):
    """Frames of TCP conversations interleaved the way a monitored link carries
    them -- handshake, data both ways, FIN or RST teardown, retransmissions --
    plus the traffic around them a stack sees: orphan segments, bad IP / TCP
    checksums, ARP, IPv6, UDP, ICMP to and past the local address, IP options.
    Per-flow order is kept; flows interleave pseudo-randomly (seeded).  With
    listen_port, some flows go to local_ip:listen_port (an end host's listener)."""
    import random
    rnd = random.Random(seed)
    flows = []
    for f in range(nflows):
        cli = f"10.{1 + f % 7}.{(f * 37) % 250}.{1 + (f * 11) % 250}"
        srv = f"192.168.{f % 5}.{1 + (f * 13) % 250}"
        cp, sp = 20000 + f * 7 % 40000, (80, 443, 8080)[f % 3]
        if listen_port and f % 4 == 3:
            srv, sp = local_ip, listen_port
        ic, is_ = rnd.getrandbits(32), rnd.getrandbits(32)
        mss = struct.pack("!BBH", 2, 4, 1460)
        pk = []

        def c2s(flags, seq, ack, pl=b"", opts=b""):
            pk.append(tcp_frame(cli, srv, cp, sp, pl, flags=flags, seq=seq & 0xFFFFFFFF, ack=ack & 0xFFFFFFFF,
                                doff=5 + len(opts) // 4, tcp_opts=opts, ip_id=len(pk)))

        def s2c(flags, seq, ack, pl=b"", opts=b""):
            pk.append(tcp_frame(srv, cli, sp, cp, pl, flags=flags, seq=seq & 0xFFFFFFFF, ack=ack & 0xFFFFFFFF,
                                doff=5 + len(opts) // 4, tcp_opts=opts, ip_id=len(pk)))

        c2s(0x02, ic, 0, opts=mss)                       # SYN
        s2c(0x12, is_, ic + 1, opts=mss)                 # SYN-ACK
        c2s(0x10, ic + 1, is_ + 1)                       # ACK
        cs, ss = ic + 1, is_ + 1
        for r in range(rnd.randint(1, 4)):
            pl = bytes(rnd.getrandbits(8) for _ in range(rnd.choice((1, 100, 536, 1400))))
            c2s(0x18, cs, ss, pl)
            if rnd.random() < 0.2:
                c2s(0x18, cs, ss, pl)                    # retransmission
            cs += len(pl)
            pl = bytes(rnd.getrandbits(8) for _ in range(rnd.choice((0, 64, 1000))))
            s2c(0x18 if pl else 0x10, ss, cs, pl)
            ss += len(pl)
        if f % 5 == 4:
            c2s(0x14, cs, ss)                            # RST
        else:
            c2s(0x11, cs, ss)                            # FIN
            s2c(0x11, ss, cs + 1)
            c2s(0x10, cs + 1, ss + 1)
        flows.append(pk)
    extra = [
        tcp_frame("10.9.9.9", "192.168.9.9", 5555, 80, b"orphan", flags=0x18, seq=99),
        tcp_frame("10.9.9.8", "192.168.9.9", 5556, 80, b"orphan", flags=0x10, seq=7),
        tcp_frame("10.9.9.7", "192.168.9.9", 5557, 80, b"x" * 300, flags=0x18, ip_csum=0x1234),
        tcp_frame("10.9.9.6", "192.168.9.9", 5558, 80, b"y" * 301, flags=0x18, tcp_csum=0x4321),
        tcp_frame("10.9.9.6", "192.168.9.9", 5558, 80, b"syn", flags=0x02, tcp_csum=0x4322),
        tcp_frame("10.9.9.5", "192.168.9.9", 5559, 80, b"z" * 64, flags=0x18, ihl=7),
        tcp_frame("10.9.9.4", "192.168.9.9", 5560, 80, b"", flags=0x10, doff=4, tot_len=36),
        tcp_frame("10.9.9.3", "192.168.9.9", 5561, 80, b"", flags=0x10, tot_len=19, pad_to=60),
        tcp_frame("10.9.9.2", "192.168.9.9", 5562, 80, b"v6", flags=0x10, version=6),
        tcp_frame("10.9.9.2", "192.168.9.9", 5562, 80, b"arp", ethertype=ETH_ARP, pad_to=60),
        tcp_frame("10.9.9.2", "192.168.9.9", 5562, 80, b"ipv6", ethertype=0x86DD, pad_to=60),
        tcp_frame("10.9.9.1", "192.168.9.9", 5563, 53, b"udp" * 10, proto=17),
        icmp_frame("10.9.9.1", local_ip, 8),
        icmp_frame("10.9.9.1", "192.168.9.9", 8),
        icmp_frame("10.9.9.1", local_ip, 0, ip_csum=0x0101),
        tcp_frame("10.9.9.0", "192.168.9.8", 5564, 80, b"rst", flags=0x04, seq=5),
    ]
    out, cursors = [], [0] * len(flows)
    live = list(range(len(flows)))
    while live:
        i = rnd.choice(live)
        out.append(flows[i][cursors[i]])
        cursors[i] += 1
        if cursors[i] == len(flows[i]):
            live.remove(i)
        if extra and rnd.random() < 0.04:
            out.append(extra.pop(0))
    return out + extra


class TpacketRing:
    """A TPACKET_V3 receive ring in a shared memfd mapping, filled the way the
    kernel fills an AF_PACKET PACKET_RX_RING (linux/if_packet.h): each block a
    tpacket_block_desc (48 B) then frames, each frame a tpacket3_hdr (48 B) +
    sockaddr_ll, its Ethernet header at offset 82 (network header 16-byte
    aligned, TPACKET3_HDRLEN + 16 rounded), block_status TP_STATUS_USER (1) when
    handed to the reader, TP_STATUS_KERNEL (0) when given back."""

    def __init__(self, nblocks: int, block_size: int):
        import mmap
        import os
        self.nb, self.bsz = nblocks, block_size
        self.fd = os.memfd_create("mosrx-tpacket-ring")
        os.ftruncate(self.fd, nblocks * block_size)
        self.m = mmap.mmap(self.fd, nblocks * block_size, mmap.MAP_SHARED, mmap.PROT_READ | mmap.PROT_WRITE)
        import ctypes
        self._anchor = ctypes.c_char.from_buffer(self.m)
        self.addr = ctypes.addressof(self._anchor)
        self.seq = 0

    def status(self, b: int) -> int:
        return struct.unpack_from("<I", self.m, b * self.bsz + 8)[0]

    def fill(self, b: int, frames: list[bytes]) -> int:
        """Write as many of `frames` as fit into block b and hand it over; returns the count."""
        base, pos, k = b * self.bsz, 48, 0
        for f in frames:
            rec = (82 + len(f) + 15) & ~15
            if pos + rec > self.bsz:
                break
            hdr = struct.pack("<IIIIIIHH", rec, 0, 0, len(f), len(f), 1, 82, 96) + b"\0" * 20
            sll = struct.pack("<HHiHBB8s", 17, 0x0300, 1, 1, 0, 6, b"")          # sll_pkttype 0: PACKET_HOST
            self.m[base + pos:base + pos + 48] = hdr
            self.m[base + pos + 48:base + pos + 68] = sll
            self.m[base + pos + 82:base + pos + 82 + len(f)] = f
            pos += rec
            k += 1
        self.seq += 1
        struct.pack_into("<IIIIIIQ", self.m, base, 3, 0, 0, k, 48, pos, self.seq)
        struct.pack_into("<I", self.m, base + 8, 1)                              # TP_STATUS_USER, last
        return k

    def close(self):
        import os
        del self._anchor
        self.m.close()
        os.close(self.fd)
