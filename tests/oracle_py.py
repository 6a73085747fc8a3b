"""ctypes access to the oracle (TEST INFRASTRUCTURE ONLY).

Loads oracle/libmosrx_oracle.so (the C restatement) and, when it was built in
this container, runs oracle/_ref/mosref (mOS's own compiled rx path).  Only
tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use this.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
import tempfile

import numpy as np

from pktlib import RESULT_DTYPE, read_ref_results, write_ref_trace

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_SO = os.path.join(ROOT, "oracle", "libmosrx_oracle.so")
REF_BIN = os.path.join(ROOT, "oracle", "_ref", "mosref")
REF_BPF_BIN = os.path.join(ROOT, "oracle", "_ref", "mosbpf")
BPF_INSN = np.dtype([("code", "<u2"), ("jt", "u1"), ("jf", "u1"), ("k", "<u4")])   # struct sfbpf_insn

MS_KEY = bytes([0x6d, 0x5a, 0x56, 0xda, 0x25, 0x5b, 0x0e, 0xc2, 0x41, 0x67, 0x25, 0x3d, 0x43, 0xa3,
                0x8f, 0xb0, 0xd0, 0xca, 0x2b, 0xcb, 0xae, 0x7b, 0x30, 0xb4, 0x77, 0xcb, 0x2d, 0xa3,
                0x80, 0x30, 0xf2, 0x0c, 0x6a, 0x42, 0xb7, 0x3b, 0xbe, 0xac, 0x01, 0xfa])


class Params(C.Structure):
    _fields_ = [("num_msp", C.c_uint32), ("num_esp", C.c_uint32), ("forward", C.c_int32),
                ("num_queues", C.c_int32), ("queue_mode", C.c_int32), ("skip_tcp_csum", C.c_int32),
                ("rss_key_len", C.c_uint32), ("rss_key", C.c_uint8 * 52),
                ("num_local", C.c_uint32), ("local_ip", C.c_uint32 * 16)]


TCPINFO_DTYPE = np.dtype([("seq", "<u4"), ("ack_seq", "<u4"), ("window", "<u2"), ("ip_len", "<u2")])


def ip_raw(a: str) -> int:
    """Dotted quad -> the raw u32 mOS stores (network order loaded little-endian)."""
    return int.from_bytes(bytes(int(x) for x in a.split(".")), "little")


def params(num_msp=1, num_esp=0, forward=1, num_queues=1, queue_mode=1, skip_tcp_csum=0,
           key=b"\x05" * 40, local=()) -> Params:
    p = Params()
    p.num_msp, p.num_esp, p.forward = num_msp, num_esp, forward
    p.num_queues, p.queue_mode, p.skip_tcp_csum = num_queues, queue_mode, skip_tcp_csum
    p.rss_key_len = len(key)
    for i, b in enumerate(key):
        p.rss_key[i] = b
    p.num_local = len(local)
    for i, a in enumerate(local):
        p.local_ip[i] = ip_raw(a) if isinstance(a, str) else a
    return p


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(ORACLE_SO):
            subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle")])
        L = C.CDLL(ORACLE_SO)
        L.mo_ip_fast_csum.restype = C.c_uint16
        L.mo_ip_fast_csum.argtypes = [C.c_char_p, C.c_uint]
        L.mo_tcp_csum.restype = C.c_uint16
        L.mo_tcp_csum.argtypes = [C.c_char_p, C.c_uint16, C.c_uint32, C.c_uint32]
        L.mo_rss_key_cache.argtypes = [C.c_char_p, C.POINTER(C.c_uint32)]
        L.mo_rss_hash.restype = C.c_uint32
        L.mo_rss_hash.argtypes = [C.POINTER(C.c_uint32), C.c_uint32, C.c_uint32, C.c_uint16, C.c_uint16]
        L.mo_rss_queue.restype = C.c_int
        L.mo_rss_queue.argtypes = [C.c_uint32, C.c_int, C.c_int]
        L.mo_classify.restype = C.c_int
        L.mo_classify.argtypes = [C.POINTER(Params), C.c_void_p, C.c_uint64, C.c_void_p, C.c_void_p,
                                  C.c_uint32, C.c_void_p]
        L.mo_classify_mt.restype = C.c_int
        L.mo_classify_mt.argtypes = L.mo_classify.argtypes + [C.c_int]
        L.mo_classify_fh.restype = C.c_int
        L.mo_classify_fh.argtypes = L.mo_classify.argtypes + [C.c_void_p]
        L.mo_classify_ex.restype = C.c_int
        L.mo_classify_ex.argtypes = L.mo_classify.argtypes + [C.c_void_p, C.c_void_p]
        L.mo_superfasthash.restype = C.c_uint32
        L.mo_superfasthash.argtypes = [C.c_char_p, C.c_int]
        L.mo_bpf_filter.restype = C.c_uint32
        L.mo_bpf_filter.argtypes = [C.c_void_p, C.c_char_p, C.c_uint32, C.c_uint32]
        L.mo_bpf_validate.restype = C.c_int
        L.mo_bpf_validate.argtypes = [C.c_void_p, C.c_int]
        L.mo_tx_csum.restype = C.c_int
        L.mo_tx_csum.argtypes = [C.c_void_p, C.c_uint64, C.c_void_p, C.c_void_p, C.c_uint32, C.c_int]
        L.mo_bpf_returns.restype = C.c_int
        L.mo_bpf_returns.argtypes = [C.c_void_p, C.c_uint32, C.c_int, C.c_void_p, C.c_uint64, C.c_void_p,
                                     C.c_void_p, C.c_uint32, C.c_void_p]
        L.mo_bpf_eval.restype = C.c_int
        L.mo_bpf_eval.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p, C.c_uint64, C.c_void_p, C.c_void_p,
                                  C.c_uint32, C.c_void_p]
        _lib = L
    return _lib


def rss_hash(key: bytes, sip: int, dip: int, sp: int, dp: int) -> int:
    cache = (C.c_uint32 * 96)()
    lib().mo_rss_key_cache(key, cache)
    return lib().mo_rss_hash(cache, sip, dip, sp, dp)


def classify(buf, off, ln, p: Params | None = None, nthreads: int = 1) -> np.ndarray:
    p = p or params()
    buf = np.ascontiguousarray(buf, np.uint8)
    off = np.ascontiguousarray(off, np.uint32)
    ln = np.ascontiguousarray(ln, np.uint16)
    out = np.zeros(len(off), RESULT_DTYPE)
    args = (C.byref(p), buf.ctypes.data, len(buf), off.ctypes.data, ln.ctypes.data, len(off),
            out.ctypes.data)
    rc = lib().mo_classify_mt(*args, nthreads) if nthreads > 1 else lib().mo_classify(*args)
    if rc:
        raise OSError(-rc, "mo_classify failed")
    return out


def classify_fh(buf, off, ln, p: Params | None = None):
    """Records + the FindStream flow hash (HashFlow before masking) per frame."""
    p = p or params()
    buf = np.ascontiguousarray(buf, np.uint8)
    off = np.ascontiguousarray(off, np.uint32)
    ln = np.ascontiguousarray(ln, np.uint16)
    out = np.zeros(len(off), RESULT_DTYPE)
    fh = np.zeros(len(off), np.uint32)
    rc = lib().mo_classify_fh(C.byref(p), buf.ctypes.data, len(buf), off.ctypes.data, ln.ctypes.data,
                              len(off), out.ctypes.data, fh.ctypes.data)
    if rc:
        raise OSError(-rc, "mo_classify_fh failed")
    return out, fh


def classify_ex(buf, off, ln, p: Params | None = None):
    """Records + flow hash + pkt_info TCP fields (mosrx_tcpinfo) per frame."""
    p = p or params()
    buf = np.ascontiguousarray(buf, np.uint8)
    off = np.ascontiguousarray(off, np.uint32)
    ln = np.ascontiguousarray(ln, np.uint16)
    out = np.zeros(len(off), RESULT_DTYPE)
    fh = np.zeros(len(off), np.uint32)
    ti = np.zeros(len(off), TCPINFO_DTYPE)
    rc = lib().mo_classify_ex(C.byref(p), buf.ctypes.data, len(buf), off.ctypes.data, ln.ctypes.data,
                              len(off), out.ctypes.data, fh.ctypes.data, ti.ctypes.data)
    if rc:
        raise OSError(-rc, "mo_classify_ex failed")
    return out, fh, ti


def tx_csum(buf, off, ln, flags: int) -> np.ndarray:
    """A rewritten copy of `buf` (mo_tx_csum: the MOS_UPDATE_*_CHKSUM rewrite)."""
    out = np.array(buf, np.uint8, copy=True)
    off = np.ascontiguousarray(off, np.uint32)
    ln = np.ascontiguousarray(ln, np.uint16)
    lib().mo_tx_csum(out.ctypes.data, len(out), off.ctypes.data, ln.ctypes.data, len(off), flags)
    return out


def have_ref() -> bool:
    return os.path.exists(REF_BIN)


def run_ref(buf, off, ln, *, num_msp=1, num_esp=0, num_queues=1, queue_mode=1, local=(), forward=0,
            listen_port=None):
    """Run mOS's own compiled rx path over the frames.  `local`: the netdev
    addresses (dotted quads) ICMP frames count as "to me" for; `forward`: mos.conf
    `forward` (the record's `fwd` is 1 where ProcessPacket called ForwardIPPacket /
    ForwardEthernetFrame, recorded by the harness instead of sent); `listen_port`:
    an end-host socket listening on that port (INADDR_ANY)."""
    env = dict(os.environ)
    env.pop("MOSREF_LISTENER", None)
    if listen_port is not None:
        env["MOSREF_LISTENER"] = str(listen_port)
    with tempfile.TemporaryDirectory() as d:
        tin, tout = os.path.join(d, "t.in"), os.path.join(d, "t.out")
        write_ref_trace(tin, buf, off, ln, num_msp=num_msp, num_esp=num_esp, forward=forward,
                        num_queues=num_queues, queue_mode=queue_mode,
                        local=[ip_raw(a) if isinstance(a, str) else a for a in local])
        subprocess.run([REF_BIN, tin, tout], check=True, stdout=subprocess.DEVNULL, env=env)
        return read_ref_results(tout, len(off))


class BpfProg(C.Structure):
    """mosrx_bpf_prog (include/mosrx.h)."""
    _fields_ = [("insns", C.c_void_p), ("len", C.c_uint32), ("len_mode", C.c_int32)]


def bpf_filter(insns: np.ndarray, frame: bytes, length: int) -> int:
    """sfbpf_filter(insns, frame, length, length) restated (None/empty = no filter)."""
    insns = np.ascontiguousarray(insns, BPF_INSN)
    ptr = insns.ctypes.data if len(insns) else None
    return lib().mo_bpf_filter(ptr, bytes(frame) + bytes(8), length, length)


def bpf_validate(insns: np.ndarray) -> int:
    insns = np.ascontiguousarray(insns, BPF_INSN)
    return lib().mo_bpf_validate(insns.ctypes.data if len(insns) else None, len(insns))


def bpf_eval(progs: list, buf, off, ln) -> np.ndarray:
    """progs: list of (insns ndarray, len_mode).  Returns the per-frame match mask."""
    keep = [np.ascontiguousarray(i, BPF_INSN) for i, _ in progs]
    arr = (BpfProg * max(1, len(progs)))()
    for j, ((_, mode), ins) in enumerate(zip(progs, keep)):
        arr[j].insns = ins.ctypes.data if len(ins) else None
        arr[j].len = len(ins)
        arr[j].len_mode = mode
    buf = np.ascontiguousarray(buf, np.uint8)
    off = np.ascontiguousarray(off, np.uint32)
    ln = np.ascontiguousarray(ln, np.uint16)
    out = np.zeros(len(off), np.uint32)
    rc = lib().mo_bpf_eval(arr, len(progs), buf.ctypes.data, len(buf), off.ctypes.data, ln.ctypes.data,
                           len(off), out.ctypes.data)
    if rc:
        raise OSError(-rc, "mo_bpf_eval failed")
    return out


def bpf_returns(insns, len_mode: int, buf, off, ln) -> np.ndarray:
    """sfbpf_filter's return value per frame at a call-site length (0 where not evaluated)."""
    ins = np.ascontiguousarray(insns, BPF_INSN)
    buf = np.ascontiguousarray(buf, np.uint8)
    off = np.ascontiguousarray(off, np.uint32)
    ln = np.ascontiguousarray(ln, np.uint16)
    out = np.zeros(len(off), np.uint32)
    lib().mo_bpf_returns(ins.ctypes.data if len(ins) else None, len(ins), len_mode, buf.ctypes.data, len(buf),
                         off.ctypes.data, ln.ctypes.data, len(off), out.ctypes.data)
    return out


def have_ref_bpf() -> bool:
    return os.path.exists(REF_BPF_BIN)


def run_ref_bpf(lines: list[str], buf, off, ln) -> list[dict]:
    """Compile + evaluate with mOS's own BPF objects (oracle/_ref/mosbpf)."""
    import struct
    n = len(off)
    with tempfile.TemporaryDirectory() as d:
        te, tin, tout = (os.path.join(d, x) for x in ("e.txt", "t.in", "t.out"))
        with open(te, "w") as fh:
            fh.write("\n".join(lines) + "\n")
        with open(tin, "wb") as fh:
            fh.write(struct.pack("<II", n, len(buf)))
            fh.write(np.asarray(off, "<u4").tobytes())
            fh.write(np.asarray(ln, "<u2").tobytes())
            fh.write(np.asarray(buf, np.uint8).tobytes())
        subprocess.run([REF_BPF_BIN, te, tin, tout], check=True, stdout=subprocess.DEVNULL)
        raw = open(tout, "rb").read()
    out, p = [], 0
    for _ in lines:
        rc, val, ni = struct.unpack_from("<iiI", raw, p)
        p += 12
        insns = np.frombuffer(raw[p:p + 8 * ni], BPF_INSN).copy()
        p += 8 * ni
        rf = np.frombuffer(raw[p:p + 4 * n], "<u4").copy()
        p += 4 * n
        ri = np.frombuffer(raw[p:p + 4 * n], "<u4").copy()
        p += 4 * n
        out.append(dict(rc=rc, validate=val, insns=insns, ret_frame=rf, ret_ip=ri))
    assert p == len(raw)
    return out
