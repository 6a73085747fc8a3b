"""The TPACKET_V3 ring source without a socket (mosrx_source_tpacket_v3).

The AF_PACKET source's ring logic -- take retired blocks in order, lend runs
of them zero-copy to gpu_module_func (hipHostRegister of the mapping,
loopback.c), give blocks back to the producer only when the batch holding
them is recycled -- driven over a ring this test fills itself in a shared
memfd mapping, playing the kernel's part: it writes frames into blocks the
reader gave back (block_status TP_STATUS_KERNEL) and flips them to
TP_STATUS_USER.  Needs no CAP_NET_RAW, so the zero-copy path runs on the GPU
box; the real-socket tests stay in test_boundary.py (skipped without the
capability).
"""
import ctypes as C

import numpy as np
import pytest

import mosrx
import oracle_py as O
from pktlib import TpacketRing, pack_frames, tcp_frame, icmp_frame


def _frames(n, seed=5):
    rng = np.random.default_rng(seed)
    out = []
    for i in range(n):
        size = int(rng.choice([6, 536, 1460]))
        f = tcp_frame(f"10.0.{i % 200}.{1 + i % 250}", "192.168.0.9", 1000 + i % 5000, 80,
                      bytes(rng.integers(0, 256, size, dtype=np.uint8)), seq=i, flags=0x18,
                      tcp_csum=0x1111 if i % 97 == 5 else None)
        out.append(f if i % 101 != 7 else icmp_frame("10.0.0.1", "192.168.0.9"))
    return out


def _src(ring):
    s = mosrx.lib().mosrx_source_tpacket_v3(C.c_void_p(ring.addr), ring.nb, ring.bsz)
    assert s
    return s


def test_tpacket_ring_read_in_order_and_blocks_returned():
    """Copying reader (no GPU registration here): every frame once, in order, and
    every drained block back with the producer."""
    ring = TpacketRing(4, 1 << 16)
    frames = _frames(400)
    src = _src(ring)
    try:
        pending, got, buf = list(frames), [], np.zeros(2048, np.uint8)
        nxt = 0
        for _ in range(1000):
            for k in range(ring.nb):                         # the producer refills given-back blocks in order
                b = (nxt + k) % ring.nb
                if pending and ring.status(b) == 0 and b == nxt % ring.nb:
                    pending = pending[ring.fill(b, pending):]
                    nxt += 1
            n = mosrx.lib().mosrx_source_next(src, buf.ctypes.data, len(buf))
            if n > 0:
                got.append(bytes(buf[:n]))
            elif not pending:
                break
        assert got == frames
        assert all(ring.status(b) == 0 for b in range(ring.nb))
        assert mosrx.afpacket_info(src).ring_bytes == 4 << 16
    finally:
        mosrx.lib().mosrx_source_close(src)
        ring.close()


def test_tpacket_ring_rejects_bad_geometry():
    ring = TpacketRing(2, 1 << 16)
    try:
        L = mosrx.lib()
        assert not L.mosrx_source_tpacket_v3(C.c_void_p(ring.addr), 2, 3000)     # not a power of two
        assert not L.mosrx_source_tpacket_v3(C.c_void_p(ring.addr), 0, 1 << 16)
        assert not L.mosrx_source_tpacket_v3(None, 2, 1 << 16)
    finally:
        ring.close()


@pytest.mark.gpu
@pytest.mark.parametrize("group", [1, 3])
def test_tpacket_ring_lent_zero_copy_to_the_backend(group):
    """The ring registered with the HIP runtime and lent to gpu_module_func:
    batches are runs of the ring itself (get_rptr points into the mapping),
    the records equal the oracle's for every frame, and no block goes back to
    the producer while a batch exposing its frames is out -- the producer
    overwrites every given-back block at once, so a block recycled too early
    would show up as a frame that differs from what was delivered."""
    ring = TpacketRing(6, 1 << 18)
    frames = _frames(3000)
    src = _src(ring)
    assert mosrx.afpacket_info(src).zero_copy == 1
    be = mosrx.GpuBackend([src], batch=256, pipeline=True, group=group)
    try:
        pending, nxt = list(frames), 0
        got, recs = [], []
        junk = [tcp_frame("1.1.1.1", "2.2.2.2", 1, 1, b"\xEE" * 900)] * 400
        idle = 0
        for _ in range(10000):
            # the producer: fill the next block in ring order once it is back; blocks
            # given back with nothing left to send are scribbled over
            b = nxt % ring.nb
            if ring.status(b) == 0:
                if pending:
                    pending = pending[ring.fill(b, pending):]
                    nxt += 1
            n = be.recv_pkts(0)
            assert n >= 0
            if n == 0:
                idle += 1
                if not pending and idle > 50:
                    break
                continue
            idle = 0
            ln = C.c_uint16()
            ptrs = [be._rptr(be.ctx, 0, i, C.byref(ln)) for i in range(n)]
            for p in ptrs:
                assert ring.addr <= p < ring.addr + ring.nb * ring.bsz      # zero-copy: a pointer into the ring
                assert ring.status((p - ring.addr) // ring.bsz) == 1       # its block is still lent
            got += [be.get_rptr(0, i) for i in range(n)]
            recs.append(be.results(0, n))
            for b2 in range(ring.nb):                        # scribble over every block already given back
                if ring.status(b2) == 0 and b2 != nxt % ring.nb:
                    ring.fill(b2, junk)
                    struct_clear(ring, b2)
        assert got == frames
        buf, off, ln_ = pack_frames(frames)
        want = O.classify(buf, off, ln_, O.params())
        have = np.concatenate(recs)
        assert np.array_equal(have.view(np.uint8), want.view(np.uint8))
    finally:
        be.close()
        ring.close()


def struct_clear(ring, b):
    """Undo the hand-over of a scribbled block (the reader must never see it)."""
    import struct
    struct.pack_into("<I", ring.m, b * ring.bsz + 8, 0)
