"""TX checksum rewrite: mtcp_setlastpkt's MOS_UPDATE_IP_CHKSUM /
MOS_UPDATE_TCP_CHKSUM (mos_api.c:1177-1193) over a batch, on the GPU.

tests/golden/tx_*.npz hold, per frame, whether each check is rewritten and the
value mOS's own compiled ip_fast_csum / TCPCalcChecksum give after the check
fields are zeroed (tests/golden/make_golden.py).  The inputs keep their old
(valid, corrupted or random) checks, so the zeroing step is exercised too.
"""
import os

import numpy as np
import pytest

import mosrx
import oracle_py as O

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
FIXTURES = ["tx_mixed", "tx_odd", "tx_short"]
IP, TCP = mosrx.TX_IP_CSUM, mosrx.TX_TCP_CSUM
FLAGS = [IP | TCP, IP, TCP]


def expected(z, flags):
    out = z["frames"].copy()
    for i, (o, n) in enumerate(zip(z["off"].tolist(), z["len"].tolist())):
        ihl = int(out[o + 14] & 0xF) if n > 14 else 0
        if (flags & IP) and z["ip_w"][i]:
            out[o + 24:o + 26] = np.frombuffer(np.uint16(z["ip_check"][i]).tobytes(), np.uint8)
        if (flags & TCP) and z["tcp_w"][i]:
            at = o + 30 + 4 * ihl
            out[at:at + 2] = np.frombuffer(np.uint16(z["tcp_check"][i]).tobytes(), np.uint8)
    return out


@pytest.mark.parametrize("fix", FIXTURES)
@pytest.mark.parametrize("flags", FLAGS)
def test_oracle_tx_matches_reference(fix, flags):
    z = np.load(os.path.join(GOLDEN, f"{fix}.npz"))
    np.testing.assert_array_equal(O.tx_csum(z["frames"], z["off"], z["len"], flags), expected(z, flags))


def test_tx_fixture_coverage():
    z = np.load(os.path.join(GOLDEN, "tx_mixed.npz"))
    # rewrites, untouched frames, and inputs whose old checks were wrong all occur
    assert 0 < z["tcp_w"].sum() < z["ip_w"].sum() < len(z["off"])
    after = O.tx_csum(z["frames"], z["off"], z["len"], IP | TCP)
    assert (after != z["frames"]).any()


def test_tx_short_segments_fixture():
    """tx_short: segments shorter than a TCP header (doff < 5, short tot_len), so
    tcph->check lies past the bytes TCPCalcChecksum sums -- wholly, or by its
    second byte -- and its old value must not count (found by the round-3 soak)."""
    z = np.load(os.path.join(GOLDEN, "tx_short.npz"))
    seg = np.array([((int(z["frames"][o + 16]) << 8) | int(z["frames"][o + 17])) - 20 for o in z["off"].tolist()])
    assert z["tcp_w"].all() and (seg <= 16).any() and (seg == 17).any() and (seg >= 18).any()


def test_tx_rewritten_frames_verify():
    # property: every rewritten TCP frame then passes mOS's checks (TCP_OK) in the oracle
    z = np.load(os.path.join(GOLDEN, "tx_mixed.npz"))
    after = O.tx_csum(z["frames"], z["off"], z["len"], IP | TCP)
    res = O.classify(after, z["off"], z["len"], O.params(forward=0))
    ok = z["tcp_w"] & (res["reason"] != mosrx.R["IP_BADVER"]) & (res["reason"] != mosrx.R["IP_SHORT"])
    assert np.all(res["reason"][ok] == mosrx.R["TCP_OK"])


# ---------------------------------------------------------------- GPU parity
@pytest.mark.gpu
@pytest.mark.parametrize("fix", FIXTURES)
@pytest.mark.parametrize("flags", FLAGS)
def test_tx_golden(gpu_ctx, fix, flags):
    z = np.load(os.path.join(GOLDEN, f"{fix}.npz"))
    exp = expected(z, flags)
    np.testing.assert_array_equal(gpu_ctx.tx_csum_host(z["frames"], z["off"], z["len"], flags), exp)
    db = gpu_ctx.upload(z["frames"], z["off"], z["len"])
    gpu_ctx.tx_csum_dev(db, flags)
    np.testing.assert_array_equal(db.frames(len(z["frames"])), exp)
    db.free()


@pytest.mark.gpu
@pytest.mark.parametrize("variant", [mosrx.shape_variant(mosrx.KIND_SMALL), mosrx.shape_variant(mosrx.KIND_S13)])
@pytest.mark.parametrize("fix", FIXTURES)
def test_tx_forced_shapes(gpu_ctx, variant, fix):
    z = np.load(os.path.join(GOLDEN, f"{fix}.npz"))
    gpu_ctx.set_variant(variant)
    try:
        got = gpu_ctx.tx_csum_host(z["frames"], z["off"], z["len"], IP | TCP)
    finally:
        gpu_ctx.set_variant(2)
    np.testing.assert_array_equal(got, expected(z, IP | TCP))


@pytest.mark.gpu
@pytest.mark.parametrize("kind,n", [(mosrx.TRACE_S64, 32_768), (mosrx.TRACE_M1500, 65_536),
                                    (mosrx.TRACE_IMIX, 262_144)])
def test_tx_full_size_traces(gpu_ctx, kind, n):
    t = mosrx.Trace(kind, n)
    exp = O.tx_csum(t.frames, t.off, t.len, IP | TCP)
    db = gpu_ctx.upload(t.frames, t.off, t.len, frames_bytes=t.frames_bytes, max_len=t.max_len)
    gpu_ctx.tx_csum_dev(db)
    got = db.frames(len(t.frames))
    np.testing.assert_array_equal(got, exp)
    # size-independent property: the generator's corrupted frames (1/1024 IP, 1/1024 TCP) are repaired
    gpu_ctx.set_params(mosrx.default_params())
    gpu_ctx.classify_dev(db)
    assert np.all(db.results()["reason"] == mosrx.R["TCP_OK"])
    db.free()


@pytest.mark.gpu
@pytest.mark.parametrize("shift", [0, 1, 3])
def test_tx_host_records_full_size(gpu_ctx, shift):
    """mosrx_tx_csum_host brings back 8-byte check records and writes them into
    the caller's frames on the host (csrc/mosrx_api.c tx_patch): the frames
    equal the oracle's rewrite and the device's in-place one, at every frame
    alignment (odd starts store the check words byte by byte on the GPU)."""
    t = mosrx.Trace(mosrx.TRACE_IMIX, 65_536)
    buf = np.zeros(len(t.frames) + 8, np.uint8)
    buf[shift:shift + len(t.frames)] = t.frames
    off = (t.off + shift).astype(np.uint32)
    exp = O.tx_csum(buf, off, t.len, IP | TCP)
    got = gpu_ctx.tx_csum_host(buf, off, t.len, IP | TCP)
    np.testing.assert_array_equal(got, exp)
    for flags in (IP, TCP):
        np.testing.assert_array_equal(gpu_ctx.tx_csum_host(buf, off, t.len, flags), O.tx_csum(buf, off, t.len, flags))
    db = gpu_ctx.upload(buf, off, t.len)
    gpu_ctx.tx_csum_dev(db, IP | TCP)
    np.testing.assert_array_equal(db.frames(len(buf)), exp)
    db.free()


def apply_checks(buf, off, checks):
    """The host side of mosrx_tx_check records: the words into a copy of the frames."""
    out = np.array(buf, np.uint8, copy=True)
    for o, r in zip(off.tolist(), checks):
        if r["what"] & 1:
            out[o + 24] = r["ip_check"] & 0xFF
            out[o + 25] = r["ip_check"] >> 8
        if r["what"] & 2:
            at = o + 30 + 4 * int(r["ihl"])
            out[at] = r["tcp_check"] & 0xFF
            out[at + 1] = r["tcp_check"] >> 8
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("fix", FIXTURES)
@pytest.mark.parametrize("flags", FLAGS)
def test_tx_dev_checks_golden(gpu_ctx, fix, flags):
    """mosrx_tx_csum_dev_checks: the frames stay as they were, and the records
    written into them give mOS's rewrite (the reference's own fixtures)."""
    z = np.load(os.path.join(GOLDEN, f"{fix}.npz"))
    db = gpu_ctx.upload(z["frames"], z["off"], z["len"])
    checks = gpu_ctx.tx_csum_dev_checks(db, flags)
    np.testing.assert_array_equal(db.frames(len(z["frames"])), z["frames"])
    np.testing.assert_array_equal(apply_checks(z["frames"], z["off"], checks), expected(z, flags))
    db.free()


@pytest.mark.gpu
@pytest.mark.parametrize("kind,n", [(mosrx.TRACE_M1500, 65_536), (mosrx.TRACE_IMIX, 262_144)])
def test_tx_dev_checks_full_size(gpu_ctx, kind, n):
    t = mosrx.Trace(kind, n)
    db = gpu_ctx.upload(t.frames, t.off, t.len, frames_bytes=t.frames_bytes, max_len=t.max_len)
    checks = gpu_ctx.tx_csum_dev_checks(db)
    np.testing.assert_array_equal(apply_checks(t.frames, t.off, checks), O.tx_csum(t.frames, t.off, t.len, IP | TCP))
    assert not gpu_ctx.tx_csum_dev_checks(db, 0)["what"].any()
    db.free()


def fuzz_frames(seed, n=8192):
    """Header-mutated frames at every alignment: IPv4 mostly, ihl mostly 5 but any
    nibble, tot_len equal to / around / far from the capture, TCP mostly with any
    doff, captures cut anywhere (inside Ethernet, IP, TCP, options)."""
    rng = np.random.default_rng(seed)
    cls = rng.integers(0, 10, n)
    lens = np.where(cls == 0, rng.integers(0, 34, n),
                    np.where(cls < 4, rng.integers(34, 80, n), rng.integers(60, 1515, n))).astype(np.uint16)
    gaps = rng.integers(0, 8, n)
    off = (np.cumsum(np.concatenate([[0], lens[:-1].astype(np.int64) + gaps[:-1]])) + 1).astype(np.uint32)
    buf = rng.integers(0, 256, int(off[-1]) + int(lens[-1]) + 64, dtype=np.uint8)
    for i in range(n):
        o, m = int(off[i]), int(lens[i])
        if m >= 14 and rng.random() < 0.85:
            buf[o + 12], buf[o + 13] = 0x08, 0x00
        if m >= 15:
            ihl = 5 if rng.random() < 0.7 else int(rng.integers(0, 16))
            buf[o + 14] = (0x40 if rng.random() < 0.9 else int(rng.integers(0, 16)) << 4) | ihl
            if m >= 18:
                r = rng.random()
                tl = m - 14 if r < 0.6 else (m - 14 + int(rng.integers(-24, 25)) if r < 0.85
                                              else int(rng.integers(0, 65536)))
                tl &= 0xFFFF
                buf[o + 16], buf[o + 17] = tl >> 8, tl & 0xFF
            if m >= 24 and rng.random() < 0.8:
                buf[o + 23] = 6
            d = o + 14 + 4 * ihl + 12
            if d < o + m and rng.random() < 0.8:
                buf[d] = (5 if rng.random() < 0.6 else int(rng.integers(0, 16))) << 4
    return buf, off, lens


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [1, 2, 3])
def test_tx_fuzz_headers(gpu_ctx, seed):
    """Mutated headers through all three TX forms (in place on the device, host
    records, device records applied on the host), each equal to the oracle's
    rewrite for every flag combination; the frames are never touched by the
    records form."""
    buf, off, lens = fuzz_frames(seed)
    db = gpu_ctx.upload(buf, off, lens)
    for flags in FLAGS:
        exp = O.tx_csum(buf, off, lens, flags)
        assert (exp != buf).any()
        np.testing.assert_array_equal(gpu_ctx.tx_csum_host(buf, off, lens, flags), exp)
        checks = gpu_ctx.tx_csum_dev_checks(db, flags)
        np.testing.assert_array_equal(db.frames(len(buf)), buf)
        np.testing.assert_array_equal(apply_checks(buf, off, checks), exp)
    gpu_ctx.tx_csum_dev(db, IP | TCP)
    np.testing.assert_array_equal(db.frames(len(buf)), O.tx_csum(buf, off, lens, IP | TCP))
    db.free()


def test_tx_fuzz_frames_cover_edges():
    """The fuzz input holds the cases the rewrite must tell apart (oracle only)."""
    buf, off, lens = fuzz_frames(1)
    after = O.tx_csum(buf, off, lens, IP | TCP)
    changed = np.array([(after[o:o + m] != buf[o:o + m]).any() for o, m in zip(off.tolist(), lens.tolist())])
    ihl = np.array([buf[o + 14] & 0xF if m > 14 else 0 for o, m in zip(off.tolist(), lens.tolist())])
    assert 0.2 < changed.mean() < 0.95
    assert (lens < 34).any() and (ihl < 5).any() and (ihl > 5).any() and (off % 2 == 1).any()
