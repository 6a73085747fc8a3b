"""Generate tests/golden/bpf.npz from mOS's OWN BPF compiler + interpreter.

Run in the build container (needs /root/reference):
    make -C oracle ref && python tests/golden/make_golden_bpf.py

oracle/_ref/mosbpf (core/src/bpf sources compiled where they lie, driven by
oracle/ref_bpf.c) compiles every expression below exactly as SET_BPFFILTER
does (sfbpf_compile(ETH_FRAME_LEN, DLT_EN10MB, .., optimize=1, 0),
include/bpf/sfbpf.h:83) and evaluates it with sfbpf_filter on every frame at
both call-site lengths (ip_in.c:56-63 whole frame; tcp.c:49-52 / 486-496
IP datagram + 14).  Hand-assembled programs ("raw") cover interpreter paths
no expression emits.  Stored: the programs (bytecode = compiler output, data),
the frames, and the reference's return values.  Nothing here is reference source.
"""
from __future__ import annotations

import os
import random
import struct
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))

from pktlib import ETH_ARP, pack_frames, tcp_frame  # noqa: E402
import oracle_py as O  # noqa: E402

EXPRS = [
    "tcp", "udp", "arp", "ip", "ip6", "icmp", "vlan", "ip and not tcp",
    "tcp port 80", "tcp dst port 443", "port 22 or port 80", "portrange 1000-2000",
    "tcp src portrange 0-1023", "udp and dst port 53",
    "src host 10.0.0.1", "dst net 10.0.0.0/8", "net 192.168.0.0/16 and tcp",
    "host 10.0.0.1 and port 80", "src net 172.16.0.0/12 or dst host 8.8.8.8",
    "tcp[tcpflags] & tcp-syn != 0", "tcp[tcpflags] & (tcp-syn|tcp-ack) == tcp-syn",
    "tcp[tcpflags] & (tcp-fin|tcp-rst) != 0", "tcp[13] & 7 != 0",
    "ip[8] < 64", "ip[1] & 0xfc == 0x28", "ip[6:2] & 0x1fff != 0", "ip[0] & 0xf > 5",
    "ip[2:2] > 576 and tcp", "len > 1000", "greater 500", "less 100",
    "ip proto 17 or ip proto 1", "tcp[0:2] > 1024 and tcp[2:2] < 1024",
    "tcp[((tcp[12:1] & 0xf0) >> 2):4] = 0x47455420",
    "ether host 02:00:00:00:00:01", "ether broadcast", "ether multicast",
    "ether dst 02:00:00:00:00:02 and not arp",
    "tcp and (tcp[4:4] & 0xff == 0x11)", "ip[12:4] - ip[16:4] > 0x1000000",
    "tcp[2:2] * 3 > 3000", "tcp[0:2] / 100 == 8", "udp[4:2] > 100",
]

# opcodes (include/bpf/sfbpf.h)
LD, LDX, ST, STX, ALU, JMP, RET, MISC = range(8)
W, H, B = 0, 8, 0x10
IMM, ABS, IND, MEM, LEN, MSH = 0, 0x20, 0x40, 0x60, 0x80, 0xa0
ADD, SUB, MUL, DIV, OR, AND, LSH, RSH, NEG = 0, 0x10, 0x20, 0x30, 0x40, 0x50, 0x60, 0x70, 0x80
JA, JEQ, JGT, JGE, JSET = 0, 0x10, 0x20, 0x30, 0x40
K, X, A = 0, 8, 0x10
TAX, TXA = 0, 0x80


def I(code, k=0, jt=0, jf=0):  # noqa: E743
    return struct.pack("<HBBI", code, jt, jf, k & 0xFFFFFFFF)


RAW = {
    "ret_len": [I(LD | W | LEN), I(RET | A)],
    "ldx_len_sub": [I(LDX | W | LEN), I(MISC | TXA), I(ALU | SUB | K, 60), I(RET | A)],
    "ind_wrap_ok": [I(LDX | IMM, 0xFFFFFFF0), I(LD | W | IND, 0x20), I(RET | A)],
    "ind_negative": [I(LDX | IMM, 0x80000000), I(LD | W | IND, 0), I(RET | K, 7)],
    "ind_negative_b": [I(LDX | IMM, 0xFFFFFFFF), I(LD | B | IND, 0), I(RET | K, 7)],
    "last_word": [I(LDX | W | LEN), I(LD | W | IND, 0xFFFFFFFC), I(RET | A)],
    "past_last_word": [I(LDX | W | LEN), I(LD | W | IND, 0xFFFFFFFD), I(RET | K, 9)],
    "last_half": [I(LDX | W | LEN), I(LD | H | IND, 0xFFFFFFFE), I(RET | A)],
    "past_last_half": [I(LDX | W | LEN), I(LD | H | IND, 0xFFFFFFFF), I(RET | K, 9)],
    "last_byte": [I(LDX | W | LEN), I(LD | B | IND, 0xFFFFFFFF), I(ALU | OR | K, 0x100), I(RET | A)],
    "past_last_byte": [I(LDX | W | LEN), I(LD | B | IND, 0), I(ALU | OR | K, 0x100), I(RET | A)],
    "abs_deep": [I(LD | W | ABS, 1200), I(RET | A)],
    "abs_huge": [I(LD | B | ABS, 0xFFFFFFFF), I(RET | K, 1)],
    "div_x_zero": [I(LDX | IMM, 0), I(LD | IMM, 5), I(ALU | DIV | X), I(RET | K, 3)],
    "div_x": [I(LD | H | ABS, 16), I(LDX | IMM, 7), I(ALU | DIV | X), I(RET | A)],
    "shifts_ge32": [I(LD | B | ABS, 23), I(LDX | IMM, 33), I(ALU | LSH | X), I(ALU | RSH | K, 40),
                    I(ALU | LSH | K, 35), I(RET | A)],
    "rsh_x": [I(LD | W | ABS, 26), I(LDX | IMM, 63), I(ALU | RSH | X), I(ALU | ADD | K, 1), I(RET | A)],
    "msh_ind": [I(LDX | MSH | B, 14), I(LD | H | IND, 14), I(RET | A)],
    "msh_oob": [I(LDX | MSH | B, 5000), I(RET | K, 1)],
    "mem": [I(LD | B | ABS, 23), I(ST, 3), I(LD | IMM, 7), I(LDX | MEM, 3), I(ALU | ADD | X), I(STX, 15),
            I(ST, 0), I(LD | MEM, 15), I(LDX | MEM, 0), I(ALU | MUL | X), I(RET | A)],
    "mul_neg": [I(LD | W | ABS, 26), I(ALU | MUL | K, 0x9E3779B9), I(ALU | NEG), I(ALU | AND | K, 0xFFFF7),
                I(RET | A)],
    "jx": [I(LD | H | ABS, 12), I(LDX | IMM, 0x0800), I(JMP | JEQ | X, 0, 0, 5), I(LD | B | ABS, 14),
           I(LDX | IMM, 0x45), I(JMP | JGT | X, 0, 1, 0), I(RET | K, 2), I(JMP | JGE | X, 0, 0, 1),
           I(RET | K, 0), I(JMP | JSET | X, 0, 0, 1), I(RET | K, 4), I(RET | K, 5)],
    "jk": [I(LD | B | ABS, 47), I(JMP | JSET | K, 0x12, 0, 3), I(LD | H | ABS, 36), I(JMP | JGE | K, 1024, 2, 0),
           I(RET | K, 11), I(RET | K, 0), I(JMP | JGT | K, 60000, 0, 1), I(RET | K, 12), I(RET | K, 13)],
    "ja": [I(JMP | JA, 2), I(RET | K, 0), I(RET | K, 1), I(LD | IMM, 0x55), I(JMP | JA, 0), I(RET | A)],
    "ret_zero": [I(LD | H | ABS, 12), I(RET | K, 0)],
    "ret_allones": [I(RET | K, 0xFFFFFFFF)],
    "tax_txa": [I(LD | B | ABS, 14), I(MISC | TAX), I(LD | IMM, 1), I(ALU | LSH | X), I(MISC | TXA),
                I(ALU | SUB | X), I(ALU | OR | X), I(ALU | AND | X), I(RET | A)],
    # rejected by sfbpf_validate (no ret at the end; jump out of range; mem index).  A
    # constant division by zero is NOT rejected there (it tests BPF_RVAL, sf_bpf_filter.c:628)
    # and SIGFPEs in sfbpf_filter, so it cannot be run here: tests/test_bpf.py covers it.
    "bad_noret": [I(LD | IMM, 1)],
    "bad_jump": [I(JMP | JEQ | K, 1, 5, 0), I(RET | K, 1)],
    "bad_mem": [I(LD | MEM, 16), I(RET | A)],
    "bad_ja": [I(JMP | JA, 1), I(RET | K, 1)],
}


def bpf_frames(rng: random.Random, n: int) -> list[bytes]:
    hosts = ["10.0.0.1", "10.0.0.2", "192.168.1.7", "172.20.3.4", "8.8.8.8", "1.2.3.4"]
    ports = [80, 443, 22, 53, 1500, 1999, 2000, 2001, 800, 801, 65535, 0, 1023, 1024]
    out = []
    for _ in range(n):
        rnd_ip = lambda: ".".join(str(rng.randint(0, 255)) for _ in range(4))  # noqa: E731
        src = rng.choice(hosts) if rng.random() < 0.7 else rnd_ip()
        dst = rng.choice(hosts) if rng.random() < 0.7 else rnd_ip()
        sp = rng.choice(ports) if rng.random() < 0.7 else rng.randint(0, 65535)
        dp = rng.choice(ports) if rng.random() < 0.7 else rng.randint(0, 65535)
        size = rng.choice([0, 5, 20, 200, 500, 900, 1200, 1460])
        payload = bytes(rng.getrandbits(8) for _ in range(size))
        if rng.random() < 0.15:
            payload = b"GET /index.html HTTP/1.1\r\n" + payload
        proto = rng.choice([6, 6, 6, 17, 1])
        fr = bytearray(tcp_frame(src, dst, sp, dp, payload, proto=proto,
                                 ihl=5 if rng.random() < 0.8 else rng.randint(6, 15),
                                 doff=5 if rng.random() < 0.6 else rng.randint(6, 15),
                                 flags=rng.choice([0x02, 0x12, 0x10, 0x18, 0x11, 0x04, 0x14, 0x01, 0x29]),
                                 ttl=rng.choice([1, 32, 63, 64, 128, 255]), tos=rng.getrandbits(8),
                                 ip_id=rng.getrandbits(16), seq=rng.getrandbits(32)))
        m = rng.random()
        if m < 0.06:
            fr[12:14] = struct.pack("!H", ETH_ARP)
        elif m < 0.10:
            fr[12:14] = struct.pack("!H", 0x86DD)
        elif m < 0.14:
            fr[12:14] = struct.pack("!H", 0x8100)
        elif m < 0.20:
            fr[20:22] = struct.pack("!H", rng.getrandbits(16))              # fragment field
        elif m < 0.25:
            fr[0:6] = b"\xff" * 6                                           # broadcast
        elif m < 0.30:
            fr[0] |= 1                                                      # multicast
        elif m < 0.36:
            fr = fr[:rng.randint(0, len(fr))]                               # short capture
        elif m < 0.42:
            fr[16:18] = struct.pack("!H", rng.randint(0, len(fr) + 40))     # odd tot_len
        out.append(bytes(fr))
    return out


def main():
    if not O.have_ref_bpf():
        sys.exit("oracle/_ref/mosbpf missing: run `make -C oracle ref` first (needs /root/reference)")
    rng = random.Random(0xB9F)
    frames = bpf_frames(rng, 600)
    buf, off, ln = pack_frames(frames, phase=2)
    lines = EXPRS + ["raw:" + b"".join(v).hex() for v in RAW.values()]
    names = EXPRS + [f"raw:{k}" for k in RAW]
    res = O.run_ref_bpf(lines, buf, off, ln)
    progs, plen, poff, valid, rf, ri = [], [], [], [], [], []
    for r in res:
        poff.append(sum(plen))
        plen.append(len(r["insns"]))
        progs.append(r["insns"])
        valid.append(r["validate"] if r["rc"] >= 0 else -1)
        rf.append(r["ret_frame"])
        ri.append(r["ret_ip"])
    np.savez_compressed(os.path.join(HERE, "bpf.npz"), names=np.array(names), valid=np.array(valid, np.int32),
                        prog_off=np.array(poff, np.uint32), prog_len=np.array(plen, np.uint32),
                        insns=np.concatenate(progs), frames=buf, off=off, len=ln,
                        ret_frame=np.stack(rf), ret_ip=np.stack(ri))
    print(f"bpf: {len(names)} programs ({sum(v == 1 for v in valid)} valid), {len(frames)} frames")


if __name__ == "__main__":
    main()
