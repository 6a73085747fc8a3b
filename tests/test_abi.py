"""CPU-side checks of the C ABI: the library loads, exports every declared
symbol, validates arguments, fails loudly without a GPU, and its host-side
logic (RSS tables, queue LUT inputs, trace generator, frame sources) agrees
with the oracle.  No kernel is launched here."""
import ctypes as C
import os
import re
import struct
import tempfile

import numpy as np
import pytest

import mosrx
import oracle_py as O
from pktlib import R, pack_frames, tcp_frame

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    names = set()
    for h in ("mosrx.h", "mosrx_io_module.h", "mosrx_trace.h"):
        txt = open(os.path.join(ROOT, "include", h)).read()
        txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
        names |= set(re.findall(r"\b(mosrx_[a-z0-9_]+)\s*\(", txt))
    return sorted(names)


def test_every_declared_symbol_is_exported():
    lib = C.CDLL(mosrx.LIB_PATH)
    syms = declared_symbols()
    assert len(syms) > 30
    missing = [s for s in syms if not hasattr(lib, s)]
    assert not missing, missing
    assert hasattr(lib, "gpu_module_func")
    assert mosrx.lib().mosrx_abi_version() == 3


def test_no_oracle_in_product_library():
    lib = C.CDLL(mosrx.LIB_PATH)
    for s in ("mo_classify", "mo_tcp_csum", "mo_ip_fast_csum", "mo_rss_hash"):
        assert not hasattr(lib, s)
    src = open(os.path.join(ROOT, "mos-networking-stack_amd", "mosrx", "__init__.py")).read()
    assert "oracle" not in src


def test_struct_layouts():
    assert C.sizeof(mosrx.Params) == 148          # + num_local, local_ip[16] (ABI 2)
    assert C.sizeof(mosrx.Params) == C.sizeof(O.Params)
    assert C.sizeof(mosrx.Batch) == 56          # + layout, off0, stride, reserved (ABI 3)
    assert mosrx.Batch.layout.offset == 40 and mosrx.Batch.stride.offset == 48
    assert mosrx.RESULT_DTYPE.itemsize == 16
    assert mosrx.TCPINFO_DTYPE.itemsize == 12


def test_batch_size_limit():
    """frames_bytes past MOSRX_MAX_FRAMES_BYTES is refused (-E2BIG) before any device
    work: the 16-byte-rounded buffer range must stay below the no-load offset."""
    chk = mosrx.lib().mosrx__check_batch
    chk.restype, chk.argtypes = C.c_int, [C.POINTER(mosrx.Batch), C.c_int]
    buf = np.zeros(64, np.uint8)
    off = np.zeros(1, np.uint32)
    ln = np.full(1, 60, np.uint16)
    for fb, rc in [(64, 0), (0xFFFFFFE0, 0), (0xFFFFFFE1, -7), (0xFFFFFFF0, -7), (1 << 32, -7)]:
        b = mosrx.Batch(buf.ctypes.data, fb, off.ctypes.data, ln.ctypes.data, 1, 60)
        assert chk(C.byref(b), 0) == rc, hex(fb)


@pytest.mark.skipif(os.path.exists("/dev/kfd") and os.access("/dev/kfd", os.R_OK),
                    reason="a GPU is visible")
def test_open_without_gpu_fails_loudly():
    with pytest.raises(mosrx.MosrxError) as e:
        mosrx.Context(0)
    assert e.value.errno == 19  # ENODEV: no CPU fallback


def test_param_validation_before_device():
    h = C.c_void_p()
    for kw in (dict(num_queues=0), dict(num_queues=257), dict(queue_mode=5), dict(num_local=17)):
        p = mosrx.default_params(**kw)
        assert mosrx.lib().mosrx_open(0, C.byref(p), C.byref(h)) == -22
    p = mosrx.default_params()
    p.rss_key_len = 8
    assert mosrx.lib().mosrx_open(0, C.byref(p), C.byref(h)) == -22
    assert mosrx.lib().mosrx_classify_dev(None, None, None, None) == -22


def test_defaults_match_simple_firewall_state():
    p = mosrx.default_params()
    assert (p.num_msp, p.num_esp, p.forward, p.num_queues, p.queue_mode) == (1, 0, 1, 1, 1)
    assert bytes(p.rss_key[:40]) == b"\x05" * 40 and p.rss_key_len == 40


@pytest.mark.parametrize("key", [b"\x05" * 40, mosrx.MS_KEY, bytes(range(1, 53))])
def test_rss_nibble_tables_equal_key_cache_hash(key):
    tab = mosrx.rss_tables(key).reshape(24, 16)
    rng = np.random.default_rng(7)
    for _ in range(200):
        sip, dip = (int(x) for x in rng.integers(0, 2**32, 2, dtype=np.uint64))
        sp, dp = (int(x) for x in rng.integers(0, 2**16, 2))
        tup = struct.pack("!IIHH", sip, dip, sp, dp)
        h = 0
        for k, b in enumerate(tup):
            h ^= int(tab[2 * k][b >> 4]) ^ int(tab[2 * k + 1][b & 15])
        assert h == O.rss_hash(key, sip, dip, sp, dp)


def test_trace_generator_layout_and_content():
    for kind, n, cap in [(mosrx.TRACE_S64, 3000, {60}), (mosrx.TRACE_M1500, 700, {1514}),
                         (mosrx.TRACE_IMIX, 2400, {60, 590, 1514})]:
        t = mosrx.Trace(kind, n, nflows=5000)
        assert t.n == n and set(np.unique(t.len).tolist()) == cap
        assert np.all(t.off % 16 == 2)
        assert np.all(t.off[1:] >= t.off[:-1] + t.len[:-1])
        assert t.off[-1] + t.len[-1] <= t.frames_bytes
        res = O.classify(t.frames, t.off, t.len, O.params())
        idx = np.arange(n)
        bad_ip, bad_tcp = idx % 1024 == 511, idx % 1024 == 1023
        assert np.all(res["reason"][bad_ip] == R["IP_BADCSUM"])
        assert np.all(res["reason"][bad_tcp] == R["TCP_BADCSUM"])
        assert np.all(res["reason"][~bad_ip & ~bad_tcp] == R["TCP_OK"])
    imix = mosrx.Trace(mosrx.TRACE_IMIX, 12000, nflows=1000)
    assert abs(imix.caplen_sum / imix.n - 357.83) < 0.01


def test_trace_is_deterministic():
    a = mosrx.Trace(mosrx.TRACE_IMIX, 500, nflows=100)
    b = mosrx.Trace(mosrx.TRACE_IMIX, 500, nflows=100)
    assert np.array_equal(a.frames, b.frames) and np.array_equal(a.off, b.off)
    c = mosrx.Trace(mosrx.TRACE_IMIX, 500, nflows=100, seed=99)
    assert not np.array_equal(a.frames, c.frames)


def _drain(src, cap=4096):
    buf = np.zeros(cap, np.uint8)
    out = []
    while True:
        n = mosrx.lib().mosrx_source_next(src, buf.ctypes.data, cap)
        if n <= 0:
            return out
        out.append(bytes(buf[:n]))


def test_mem_source_replays_frames():
    frames = [tcp_frame(payload=bytes([i]) * i) for i in range(1, 9)]
    buf, off, ln = pack_frames(frames)
    src = mosrx.lib().mosrx_source_mem(buf.ctypes.data, off.ctypes.data, ln.ctypes.data, len(frames), 2)
    assert src
    got = _drain(src)
    mosrx.lib().mosrx_source_close(src)
    assert got == frames * 2


@pytest.mark.parametrize("swap,nsec", [(False, False), (True, False), (False, True)])
def test_pcap_source_reads_classic_pcap(swap, nsec):
    frames = [tcp_frame(payload=b"p" * i) for i in range(0, 40, 7)]
    e = ">" if swap else "<"
    magic = 0xA1B23C4D if nsec else 0xA1B2C3D4
    with tempfile.TemporaryDirectory() as d:
        path = os.path.join(d, "t.pcap")
        with open(path, "wb") as fh:
            fh.write(struct.pack(e + "IHHiIII", magic, 2, 4, 0, 0, 65535, 1))
            for i, f in enumerate(frames):
                fh.write(struct.pack(e + "IIII", i, 0, len(f), len(f)) + f)
        src = mosrx.lib().mosrx_source_pcap(path.encode(), 1)
        assert src
        got = _drain(src)
        mosrx.lib().mosrx_source_close(src)
    assert got == frames
    assert not mosrx.lib().mosrx_source_pcap(b"/nonexistent.pcap", 1)


def test_pcap_source_replays_and_stops_at_a_truncated_record():
    """Replays wrap to the first record; a last record cut short by the end of
    the file ends each replay (as pcap_next does); an empty capture yields
    nothing, however many replays are asked for."""
    frames = [tcp_frame(payload=bytes([i]) * (i * 13)) for i in range(9)]
    with tempfile.TemporaryDirectory() as d:
        path = os.path.join(d, "t.pcap")
        with open(path, "wb") as fh:
            fh.write(struct.pack("<IHHiIII", 0xA1B2C3D4, 2, 4, 0, 0, 65535, 1))
            for i, f in enumerate(frames):
                fh.write(struct.pack("<IIII", i, 0, len(f), len(f)) + f)
            fh.write(struct.pack("<IIII", 99, 0, 500, 500) + b"cut")   # truncated record
        src = mosrx.lib().mosrx_source_pcap(path.encode(), 3)
        assert _drain(src) == frames * 3
        mosrx.lib().mosrx_source_close(src)
        empty = os.path.join(d, "e.pcap")
        with open(empty, "wb") as fh:
            fh.write(struct.pack("<IHHiIII", 0xA1B2C3D4, 2, 4, 0, 0, 65535, 1))
        src = mosrx.lib().mosrx_source_pcap(empty.encode(), 5)
        assert _drain(src) == []
        mosrx.lib().mosrx_source_close(src)


def test_module_struct_layouts_match_the_header(tmp_path):
    """The ctypes mirrors of the backend's structs have the C sizes and offsets."""
    import subprocess
    src = tmp_path / "lay.c"
    src.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "mosrx_io_module.h"\n'
                   'int main(void){printf("%zu %zu %zu %zu %zu %zu\\n", sizeof(mosrx_gpu_module_cfg),'
                   ' offsetof(mosrx_gpu_module_cfg, group_bytes), sizeof(mosrx_gpu_module_stats),'
                   ' offsetof(mosrx_gpu_module_stats, device), sizeof(mosrx_rx_state), sizeof(mosrx_bpf_set_arg));'
                   'return 0;}\n')
    exe = tmp_path / "lay"
    subprocess.run(["gcc", "-I" + os.path.join(ROOT, "include"), "-o", str(exe), str(src)], check=True)
    got = list(map(int, subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split()))
    assert got == [C.sizeof(mosrx.ModuleCfg), mosrx.ModuleCfg.group_bytes.offset, C.sizeof(mosrx.ModuleStats),
                   mosrx.ModuleStats.device.offset, 24, 16]


@pytest.mark.skipif(not os.path.exists(os.path.join(ROOT, "oracle", "_ref", "mos_rx_mos.o")),
                    reason="needs oracle/_ref (make -C oracle ref)")
def test_mos_rx_consumer_exports_its_header():
    """include/mosrx_mos_rx.h's functions are defined by csrc/mos_rx.c as built inside
    mOS's tree (the object a maintainer links into libmtcp)."""
    import subprocess
    txt = re.sub(r"/\*.*?\*/", "", open(os.path.join(ROOT, "include", "mosrx_mos_rx.h")).read(), flags=re.S)
    want = set(re.findall(r"\b(mosrx_[a-z0-9_]+)\s*\(", txt))
    nm = subprocess.run(["nm", "-g", "--defined-only", os.path.join(ROOT, "oracle", "_ref", "mos_rx_mos.o")],
                        capture_output=True, text=True, check=True).stdout
    have = {ln.split()[-1] for ln in nm.splitlines() if ln.strip()}
    assert want and want <= have, want - have


def test_pinned_range_registry():
    """Host regions are merged into one PCIe copy only inside one known pinned
    allocation (a borrowed run next to the staging block must not be
    copied together with it): the registry answers which allocation holds a span."""
    L = mosrx.lib()
    add, dele, of = L.mosrx__host_range_add, L.mosrx__host_range_del, L.mosrx__host_range_of
    add.argtypes, dele.argtypes, of.argtypes = [C.c_void_p, C.c_uint64], [C.c_void_p], [C.c_void_p, C.c_uint64]
    add.restype, dele.restype, of.restype = None, None, C.c_uint64
    a, b = 0x7F0000000000, 0x7F0000100000            # two adjacent "allocations" of 1 MiB
    add(a, 1 << 20)
    add(b, 1 << 20)
    try:
        ia, ib = of(a, 1 << 20), of(b + 4096, 4096)
        assert ia and ib and ia != ib
        assert of(a + (1 << 20) - 16, 32) == 0          # spans the boundary between the two
        assert of(a - 1, 2) == 0 and of(b + (1 << 20), 1) == 0
    finally:
        dele(a)
        dele(b)
    assert of(a, 16) == 0 and of(b, 16) == 0


def test_pinned_range_registry_nested_and_many():
    """The sorted registry (binary search under a read lock): a registered
    sub-range inside another allocation (a NIC ring registered within a larger
    mapping) does not hide the outer one from spans outside it, and hundreds
    of ranges added and removed in any order keep every answer right."""
    import random
    L = mosrx.lib()
    add, dele, of = L.mosrx__host_range_add, L.mosrx__host_range_del, L.mosrx__host_range_of
    add.argtypes, dele.argtypes, of.argtypes = [C.c_void_p, C.c_uint64], [C.c_void_p], [C.c_void_p, C.c_uint64]
    add.restype, dele.restype, of.restype = None, None, C.c_uint64
    outer, inner = 0x7E0000000000, 0x7E0000200000
    add(outer, 8 << 20)
    add(inner, 1 << 20)
    try:
        io, ii = of(outer, 4096), of(inner + 64, 64)
        assert io and ii and io != ii
        assert of(inner + (2 << 20), 4096) == io            # past the inner range, still in the outer one
        assert of(inner - 4096, 8192) == io                 # straddling the inner start: the outer one holds it
        assert of(outer + (8 << 20) - 8, 16) == 0
    finally:
        dele(inner)
        dele(outer)
    rnd = random.Random(5)
    base = 0x7D0000000000
    slots = list(range(300))
    rnd.shuffle(slots)
    for k in slots:
        add(base + k * (1 << 20), 4096 * (1 + k % 7))
    try:
        for k in range(300):
            a = base + k * (1 << 20)
            assert of(a, 4096 * (1 + k % 7)) != 0
            assert of(a + 4096 * (1 + k % 7), 1) == 0       # just past its end: nobody's
        for k in slots[:150]:
            dele(base + k * (1 << 20))
        gone = set(slots[:150])
        for k in range(300):
            assert (of(base + k * (1 << 20), 16) == 0) == (k in gone)
    finally:
        for k in slots[150:]:
            dele(base + k * (1 << 20))
