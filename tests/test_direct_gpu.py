"""Direct groups (mosrx_set_direct, cfg.direct_kb): a small group launches with
no copies -- the kernel reads the pinned frames, descriptors and batch table in
place over PCIe and writes pinned outputs in place.  The records must be the
ones the copying path makes (the oracle's, bit for bit) for every output form,
and the kernel must see what the host wrote into the same pinned buffers
since the previous launch (no stale reads through the GPU's caches): each
round below rewrites one pinned block with new frames, descriptors and a new
batch table and checks every record.  The backend (gpu_module_func) takes small
groups direct by default; its records match with and without."""
import ctypes as C

import numpy as np
import pytest

import mosrx
import oracle_py as O
from test_bpf import load, program_sets
from test_bpf_groups import _set, project8
from test_parity_gpu import assert_records_equal

pytestmark = pytest.mark.gpu

BIG = 1 << 30


def _pinned_like(ctx, dtype, n):
    p, arr = ctx.host_alloc(max(n, 1) * np.dtype(dtype).itemsize)
    return p, arr.view(dtype)[:n]


@pytest.mark.parametrize("kind,n,nb", [(mosrx.TRACE_IMIX, 20_000, 4), (mosrx.TRACE_S64, 16_384, 3),
                                       (mosrx.TRACE_M1500, 3_000, 2)])
@pytest.mark.parametrize("form", ["ex", "c8", "bpf_fused", "bpf_interp"])
@pytest.mark.parametrize("outs", ["pinned", "pageable"])
def test_direct_group_equals_oracle(gpu_ctx, kind, n, nb, form, outs):
    """Every output form of a direct group (full records + pkt_info + flow hashes;
    8-byte records; with a filter set, fused or interpreted) equals the oracle,
    outputs written in place (pinned) or copied back (pageable)."""
    t = mosrx.Trace(kind, n, nflows=1500, seed=11)
    gpu_ctx.set_params(mosrx.default_params())
    bpf = form.startswith("bpf")
    ps = program_sets(*load())[0][0][:8] if bpf else None
    gpu_ctx.bpf_set_engine(mosrx.BPF_ENGINE_INTERP if form == "bpf_interp" else mosrx.BPF_ENGINE_JIT)
    frees = []
    try:
        if bpf:
            _set(gpu_ctx, ps)
            assert gpu_ctx.bpf_fused() == (form == "bpf_fused"), gpu_ctx.bpf_jit_log()
        base, blk = gpu_ctx.host_alloc(t.frames_bytes + 8 * t.n + 256 * (nb + 1))
        frees.append(base)
        batches, parts = _stage(blk, base, t, nb)

        def arr(dtype, k, fill=0):
            if outs == "pageable":
                return np.full(k, fill, dtype) if np.dtype(dtype).names is None else np.zeros(k, dtype)
            p, a = _pinned_like(gpu_ctx, dtype, k)
            frees.append(p)
            a[...] = fill if np.dtype(dtype).names is None else np.zeros(k, dtype)
            return a

        rdt = mosrx.RESULT8_DTYPE if form != "ex" else mosrx.RESULT_DTYPE
        recs = [arr(rdt, b.n) for b in batches]
        fhs = [arr(np.uint32, b.n) for b in batches]
        tis = [arr(mosrx.TCPINFO_DTYPE, b.n) for b in batches]
        mts = [arr(np.uint32, b.n, 0xDEADBEEF) for b in batches]
        gpu_ctx.set_direct(BIG)
        if form == "ex":
            gpu_ctx.group_submit_ex(1, batches, [r.ctypes.data for r in recs], [x.ctypes.data for x in tis],
                                    [f.ctypes.data for f in fhs])
        elif form == "c8":
            gpu_ctx.group_submit_c8(1, batches, [r.ctypes.data for r in recs], [f.ctypes.data for f in fhs])
        else:
            gpu_ctx.group_submit_c8(1, batches, [r.ctypes.data for r in recs], [f.ctypes.data for f in fhs],
                                    [m.ctypes.data for m in mts])
        gpu_ctx.group_wait(1)
        assert gpu_ctx.slot_direct(1)
        for i, (fr, o, ln, fb) in enumerate(parts):
            orec, ofh, oti = O.classify_ex(fr[:fb], o, ln, O.params())
            if form == "ex":
                assert_records_equal(recs[i], orec, f"batch {i}")
                np.testing.assert_array_equal(tis[i], oti)
            else:
                assert np.array_equal(recs[i].view(np.uint8), project8(orec).view(np.uint8)), f"batch {i}"
            np.testing.assert_array_equal(fhs[i], ofh)
            if bpf:
                np.testing.assert_array_equal(mts[i], O.bpf_eval(ps, fr[:fb], o, ln))
    finally:
        gpu_ctx.set_direct(0)
        for p in frees:
            gpu_ctx.host_free(p)
        if bpf:
            gpu_ctx.bpf_set_async([])
        gpu_ctx.bpf_set_engine(mosrx.BPF_ENGINE_JIT)


def _stage(arr, base, t, nb, pos0=0):
    """Trace t as nb batches laid out in arr (host address base) from pos0:
    frames | off | len per batch, 16-byte aligned; the Batch list and parts."""
    per = -(-t.n // nb)
    parts = mosrx.split_batches(t.frames, t.off, t.len, per)
    batches, pos = [], pos0
    for fr, o, ln, fb in parts:
        fa = (fb + 15) & ~15
        arr[pos:pos + fb] = fr[:fb]
        arr[pos + fa:pos + fa + 4 * len(o)].view(np.uint32)[:] = o
        arr[pos + fa + 4 * len(o):pos + fa + 6 * len(o)].view(np.uint16)[:] = ln
        batches.append(mosrx.Batch(base + pos, fb, base + pos + fa, base + pos + fa + 4 * len(o), len(o),
                                   int(ln.max())))
        pos += ((fa + 6 * len(o)) + 255) & ~255
    return batches, parts


@pytest.mark.parametrize("memory", ["host_alloc", "registered"])
def test_direct_reads_what_the_host_rewrote(gpu_ctx, memory):
    """One pinned block rewritten every round (new frames of a different kind,
    new descriptors, a new batch table and group shape) and one pinned record
    array reused: every round's records equal the oracle's for that round's
    frames -- the kernel never sees a previous round's bytes, and the host
    never reads a previous round's records."""
    size = 24 << 20
    keep = None
    if memory == "host_alloc":
        base, arr = gpu_ctx.host_alloc(size)
    else:
        keep = np.zeros(size + 4096, np.uint8)
        base = (keep.ctypes.data + 4095) & ~4095
        arr = keep[base - keep.ctypes.data:base - keep.ctypes.data + size]
        gpu_ctx.host_register(base, size)
    rp, rarr = gpu_ctx.host_alloc(64_000 * 16)
    gpu_ctx.set_params(mosrx.default_params())
    gpu_ctx.set_direct(BIG)
    try:
        kinds = [mosrx.TRACE_IMIX, mosrx.TRACE_S64, mosrx.TRACE_M1500, mosrx.TRACE_FW64]
        for rnd in range(12):
            kind = kinds[rnd % 4]
            n = {mosrx.TRACE_M1500: 6_000}.get(kind, 30_000 + 1_000 * rnd)
            t = mosrx.Trace(kind, n, nflows=500 + rnd, seed=100 + rnd)
            nb = 1 + rnd % 5
            batches, parts = _stage(arr, base, t, nb, pos0=(rnd % 3) * 4096)
            rarr[:] = 0xA5
            recs, pre = [], 0
            for b in batches:
                recs.append(rarr[pre * 16:(pre + b.n) * 16].view(mosrx.RESULT_DTYPE))
                pre += b.n
            slot = rnd & 1
            gpu_ctx.group_submit_ex(slot, batches, [rp + 16 * sum(x.n for x in batches[:i]) for i in range(nb)])
            gpu_ctx.group_wait(slot)
            assert gpu_ctx.slot_direct(slot), f"round {rnd}"
            for i, (fr, o, ln, fb) in enumerate(parts):
                assert_records_equal(recs[i], O.classify(fr[:fb], o, ln, O.params()), f"round {rnd} batch {i}")
    finally:
        gpu_ctx.set_direct(0)
        gpu_ctx.host_free(rp)
        if memory == "host_alloc":
            gpu_ctx.host_free(base)
        else:
            gpu_ctx.host_unregister(base)
    del keep


def test_direct_only_within_its_bounds(gpu_ctx):
    """A group over the byte or frame limit, a frame buffer off 16-byte
    alignment, or pageable input is copied as before (slot_direct false), and
    its records are the same."""
    t = mosrx.Trace(mosrx.TRACE_IMIX, 8_000, nflows=300, seed=4)
    gpu_ctx.set_params(mosrx.default_params())
    base, arr = gpu_ctx.host_alloc(8 << 20)
    rp, rec = _pinned_like(gpu_ctx, mosrx.RESULT_DTYPE, t.n)
    try:
        batches, parts = _stage(arr, base, t, 1)
        total = batches[0].frames_bytes + 6 * t.n
        ora = O.classify(parts[0][0][:parts[0][3]], parts[0][1], parts[0][2], O.params())
        for limit, frames, direct in ((total, t.n, True), (total - 1, t.n, False), (0, t.n, False),
                                      (total, t.n - 1, False)):
            gpu_ctx.set_direct(limit, frames)
            rec[...] = np.zeros(t.n, mosrx.RESULT_DTYPE)
            gpu_ctx.group_submit_ex(0, batches, [rp])
            gpu_ctx.group_wait(0)
            assert gpu_ctx.slot_direct(0) == direct, (limit, frames)
            assert_records_equal(rec, ora, f"limit {limit} / {frames}")
        gpu_ctx.set_direct(BIG)
        # frames 2 bytes past a 16-byte boundary (offsets relative to the buffer),
        # descriptors aligned elsewhere in the block
        fr, o, ln, fb = parts[0]
        fpos, opos = (7 << 19) + 2, 7 << 20     # past the staged batch (~3 MB)
        arr[fpos:fpos + fb] = fr[:fb]
        arr[opos:opos + 4 * t.n].view(np.uint32)[:] = o
        arr[opos + 4 * t.n:opos + 6 * t.n].view(np.uint16)[:] = ln
        b2 = [mosrx.Batch(base + fpos, fb, base + opos, base + opos + 4 * t.n, t.n, int(ln.max()))]
        rec[...] = np.zeros(t.n, mosrx.RESULT_DTYPE)
        gpu_ctx.group_submit_ex(0, b2, [rp])
        gpu_ctx.group_wait(0)
        assert not gpu_ctx.slot_direct(0)
        assert_records_equal(rec, ora, "unaligned")
        # records 8 bytes off their 16-byte alignment: the inputs are read in place,
        # the records made on the device and copied back (never stored misaligned)
        rp2, rbuf = gpu_ctx.host_alloc(16 * t.n + 64)
        try:
            rec2 = rbuf[8:8 + 16 * t.n].view(mosrx.RESULT_DTYPE)
            gpu_ctx.group_submit_ex(0, batches, [rp2 + 8])
            gpu_ctx.group_wait(0)
            assert gpu_ctx.slot_direct(0)
            assert_records_equal(rec2, ora, "misaligned records")
        finally:
            gpu_ctx.host_free(rp2)
        # pageable frames and descriptors
        pfr = np.ascontiguousarray(fr)
        poff = np.ascontiguousarray(o, np.uint32)
        pln = np.ascontiguousarray(ln, np.uint16)
        b3 = [mosrx.Batch(pfr.ctypes.data, fb, poff.ctypes.data, pln.ctypes.data, t.n, int(pln.max()))]
        rec[...] = np.zeros(t.n, mosrx.RESULT_DTYPE)
        gpu_ctx.group_submit_ex(1, b3, [rp])
        gpu_ctx.group_wait(1)
        assert not gpu_ctx.slot_direct(1)
        assert_records_equal(rec, ora, "pageable")
    finally:
        gpu_ctx.set_direct(0)
        gpu_ctx.host_free(rp)
        gpu_ctx.host_free(base)


@pytest.mark.parametrize("mode", [mosrx.SRC_BEST, mosrx.SRC_FILL])
@pytest.mark.parametrize("direct_kb", [0, 1024])
@pytest.mark.parametrize("group", [1, 2])
def test_backend_small_groups_direct(mode, direct_kb, group):
    """gpu_module_func with cfg.direct_kb: groups under the limit launch copy-free
    (stats.rx_direct_groups), lone batches included, lent (SRC_BEST) or staged
    (SRC_FILL); records and frames equal the oracle over three replays either
    way."""
    t = mosrx.Trace(mosrx.TRACE_IMIX, 9000, nflows=300, seed=2)
    src = mosrx.mem_source(t.frames, t.off, t.len, loops=3, mode=mode)
    be = mosrx.GpuBackend([src], batch=1024, pipeline=True, cpu=5, group=group, direct_kb=direct_kb)
    try:
        ora = O.classify(t.frames, t.off, t.len, O.params())
        seen = 0
        while True:
            n = be.recv_pkts(0)
            assert n >= 0
            if n == 0:
                break
            idx = (seen + np.arange(n)) % t.n
            assert_records_equal(be.results(0, n), ora[idx], f"batch@{seen}")
            j = int(idx[n - 1])
            assert be.get_rptr(0, n - 1) == bytes(t.frames[t.off[j]:t.off[j] + t.len[j]])
            seen += n
        assert seen == 3 * t.n
        st = be.stats()
        assert st.rx_groups > 0
        assert st.rx_direct_groups == (st.rx_groups if direct_kb else 0)
    finally:
        be.close()
