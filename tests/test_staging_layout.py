"""The backend's staging layout (csrc/mosrx_source.h mosrx__frame_at), on the CPU.

gpu_module_func copies every batch it does not borrow zero-copy into its
staging block through mosrx_source_fill: frames of up to 128 bytes back to
back (a 60-byte frame takes 60 bytes over PCIe and from HBM, not 64), longer
ones at the next 16-byte boundary + 2.  Checked here for the three ways a batch
is filled: the in-memory source's runs, its frame-by-frame path (frames
truncated to max_frame) and the pcap file source; the kernels' side of it
(any alignment) is the GPU suite's layout tests and bench.py's packed rows.
"""
import ctypes as C
import struct

import numpy as np
import pytest

import mosrx

SIZES = [60, 60, 61, 64, 100, 128, 129, 1514, 60, 66, 576, 60, 127, 1500, 60, 60]


def frames_of(sizes, seed=5):
    rng = np.random.default_rng(seed)
    fr = [rng.integers(0, 256, n, dtype=np.uint8) for n in sizes]
    off = np.cumsum([0] + sizes[:-1]).astype(np.uint32) + 16
    buf = np.zeros(int(off[-1]) + sizes[-1] + 64, np.uint8)
    for o, f in zip(off, fr):
        buf[o:o + len(f)] = f
    return fr, buf, off, np.array(sizes, np.uint16)


def fill(src, max_n, max_frame, cap=1 << 20):
    dst = np.zeros(cap, np.uint8)
    off = np.zeros(max_n, np.uint32)
    ln = np.zeros(max_n, np.uint16)
    end = C.c_uint64(0)
    k = mosrx.lib().mosrx_source_fill(src, dst.ctypes.data, cap, off.ctypes.data, ln.ctypes.data, max_n, max_frame,
                                      C.byref(end))
    assert k >= 0
    return dst, off[:k], ln[:k], end.value


def check_layout(dst, off, ln, end, want):
    assert len(off) == len(want)
    assert off[0] == 2 or (ln[0] > 128 and off[0] % 16 == 2)
    for i, (o, n) in enumerate(zip(off.tolist(), ln.tolist())):
        assert bytes(dst[o:o + n]) == bytes(want[i][:n]), i
        if n > 128:
            assert o % 16 == 2, (i, o)                             # longer frames: 16-byte boundary + 2
        if i:
            prev_end = int(off[i - 1]) + int(ln[i - 1])
            assert o >= prev_end
            if n <= 128:
                assert o == prev_end, (i, o, prev_end)             # short frames: back to back
            else:
                assert o - prev_end < 16
    assert end == int(off[-1]) + int(ln[-1])


@pytest.mark.parametrize("mode", [mosrx.SRC_FILL, mosrx.SRC_PER_FRAME])
def test_mem_source_layout(mode):
    fr, buf, off, ln = frames_of(SIZES)
    src = mosrx.mem_source(buf, off, ln, loops=1, mode=mode)
    try:
        dst, o, n, end = fill(src, 64, 2048)
        check_layout(dst, o, n, end, fr)
    finally:
        mosrx.lib().mosrx_source_close(src)


def test_mem_source_truncating_path():
    """max_frame below the longest frame: the per-frame path, frames cut to max_frame,
    placed by their cut length."""
    fr, buf, off, ln = frames_of(SIZES)
    src = mosrx.mem_source(buf, off, ln, loops=1)
    try:
        dst, o, n, end = fill(src, 64, 100)
        assert n.tolist() == [min(s, 100) for s in SIZES]
        check_layout(dst, o, n, end, fr)
    finally:
        mosrx.lib().mosrx_source_close(src)


def test_pcap_source_layout(tmp_path):
    fr, _, _, _ = frames_of(SIZES, seed=9)
    path = tmp_path / "t.pcap"
    with open(path, "wb") as fh:
        fh.write(struct.pack("<IHHiIII", 0xA1B2C3D4, 2, 4, 0, 0, 65535, 1))
        for i, f in enumerate(fr):
            fh.write(struct.pack("<IIII", i, 0, len(f), len(f)) + f.tobytes())
    src = mosrx.lib().mosrx_source_pcap(str(path).encode(), 1)
    assert src
    try:
        dst, o, n, end = fill(src, 64, 2048)
        check_layout(dst, o, n, end, fr)
        # the batch is bounded by the room: a small cap takes a prefix, never past cap
        src2 = mosrx.lib().mosrx_source_pcap(str(path).encode(), 1)
        d2, o2, n2, end2 = fill(src2, 64, 2048, cap=3000)
        mosrx.lib().mosrx_source_close(src2)
        assert 0 < len(o2) < len(fr) and end2 <= 3000
        check_layout(d2, o2, n2, end2, fr[:len(o2)])
    finally:
        mosrx.lib().mosrx_source_close(src)


def test_packed_64b_batch_bytes():
    """A batch of 60-byte frames stages 60 bytes per frame (the round-3 layout took 64)."""
    fr, buf, off, ln = frames_of([60] * 1000)
    src = mosrx.mem_source(buf, off, ln, loops=1)
    try:
        _, o, n, end = fill(src, 1000, 2048)
        assert len(o) == 1000 and end == 2 + 60 * 1000
    finally:
        mosrx.lib().mosrx_source_close(src)


def test_mem_source_runs_across_replay_loops():
    """A batch longer than the replay buffer takes several runs of it: each run
    is copied whole at the source's alignment mod 16, so its long frames stay
    at 16 B + 2; between runs at most 15 bytes of gap."""
    fr, buf, off, ln = frames_of(SIZES)
    src = mosrx.mem_source(buf, off, ln, loops=4, mode=mosrx.SRC_FILL)
    try:
        dst, o, n, end = fill(src, 3 * len(SIZES), 2048)
        assert len(o) == 3 * len(SIZES)
        want = fr * 3
        for i, (a, m) in enumerate(zip(o.tolist(), n.tolist())):
            assert bytes(dst[a:a + m]) == bytes(want[i][:m]), i
            if m > 128:
                assert a % 16 == 2, (i, a)
            if i:
                prev_end = int(o[i - 1]) + int(n[i - 1])
                assert 0 <= a - prev_end < 16, (i, a, prev_end)
    finally:
        mosrx.lib().mosrx_source_close(src)
