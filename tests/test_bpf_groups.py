"""Classify + BPF (+ flow hash) over groups of batches in one launch, and filter
sets installed without waiting for their compile.

mOS evaluates its monitors' filters per frame (ip_in.c:56-63, tcp.c:42-56,
:486-496) and hashes FindStream's tuple (fhash.c:183-214).  With a filter set
installed the backend keeps its multi-batch launches: the fused classify + BPF
queue kernel (hipRTC-built) makes records, match masks and flow hashes for a
whole group at once; while the set's compile is outstanding
(mosrx_bpf_set_async) the classify queue launch and the interpreter kernel
per batch give the same results.  Everything is compared bit for bit with the
oracle (pinned to mOS's sfbpf_filter / HashFlow by tests/golden).
"""
import time

import numpy as np
import pytest

import mosrx
import oracle_py as O
from test_bpf import load, program_sets, random_sets
from test_parity_gpu import assert_records_equal

pytestmark = pytest.mark.gpu


def _set(ctx, ps, wait=True):
    ctx.bpf_set_async(ps)
    if wait:
        ctx.bpf_wait()


def _host_group(ctx, t, nb):
    """`nb` batches of trace t staged back to back in one pinned block (frames | off | len
    per batch, as gpu_module_func stages a group): (Batch list, per-batch frame slices,
    pinned pointers to free)."""
    per = -(-t.n // nb)
    parts = mosrx.split_batches(t.frames, t.off, t.len, per)
    sizes = [((fb + 15) & ~15) + len(o) * 6 + 256 for _, o, _, fb in parts]
    base, arr = ctx.host_alloc(sum(sizes))
    batches, pos = [], 0
    for (fr, o, ln, fb), sz in zip(parts, sizes):
        fa = (fb + 15) & ~15
        arr[pos:pos + fb] = fr[:fb]
        arr[pos + fa:pos + fa + 4 * len(o)].view(np.uint32)[:] = o
        arr[pos + fa + 4 * len(o):pos + fa + 6 * len(o)].view(np.uint16)[:] = ln
        batches.append(mosrx.Batch(base + pos, fb, base + pos + fa, base + pos + fa + 4 * len(o), len(o),
                                   int(ln.max())))
        pos += sz
    return batches, parts, base


@pytest.mark.parametrize("kind,n,nb", [(mosrx.TRACE_IMIX, 40_000, 5), (mosrx.TRACE_S64, 65_536, 8),
                                       (mosrx.TRACE_M1500, 9_000, 3)])
@pytest.mark.parametrize("mode", ["fused", "interp"])
def test_group_submit_bpf(gpu_ctx, kind, n, nb, mode):
    """mosrx_classify_host_group_submit_bpf: records, flow hashes and masks of every
    batch of a group from one launch (fused) or the classify launch + the
    interpreter per batch, equal to the oracle."""
    z, progs = load()
    ps = program_sets(z, progs)[0][0][:8]
    t = mosrx.Trace(kind, n, nflows=2000)
    gpu_ctx.set_params(mosrx.default_params())
    gpu_ctx.bpf_set_engine(mosrx.BPF_ENGINE_JIT if mode == "fused" else mosrx.BPF_ENGINE_INTERP)
    try:
        _set(gpu_ctx, ps)
        assert gpu_ctx.bpf_fused() == (mode == "fused"), gpu_ctx.bpf_jit_log()
        batches, parts, base = _host_group(gpu_ctx, t, nb)
        recs = [np.zeros(b.n, mosrx.RESULT_DTYPE) for b in batches]
        fhs = [np.zeros(b.n, np.uint32) for b in batches]
        mts = [np.full(b.n, 0xDEADBEEF, np.uint32) for b in batches]
        gpu_ctx.group_submit_bpf(1, batches, [r.ctypes.data for r in recs], [f.ctypes.data for f in fhs],
                                 [m.ctypes.data for m in mts])
        gpu_ctx.group_wait(1)
        for i, (fr, o, ln, fb) in enumerate(parts):
            orec, ofh = O.classify_fh(fr[:fb], o, ln, O.params())
            assert_records_equal(recs[i], orec, f"batch {i}")
            np.testing.assert_array_equal(fhs[i], ofh)
            np.testing.assert_array_equal(mts[i], O.bpf_eval(ps, fr[:fb], o, ln))
        gpu_ctx.host_free(base)
    finally:
        gpu_ctx.bpf_set_engine(mosrx.BPF_ENGINE_JIT)


@pytest.mark.parametrize("kind,n", [(mosrx.TRACE_IMIX, 65_536), (mosrx.TRACE_S64, 32_768),
                                    (mosrx.TRACE_M1500, 16_384)])
def test_queue_with_masks(gpu_ctx, kind, n):
    """mosrx_queue_create_ex with match masks and flow hashes: the fused queue kernel
    over resident batches; after a new (uncompiled) set, the interpreter form."""
    z, progs = load()
    gpu_ctx.set_params(mosrx.default_params())
    trs = [mosrx.Trace(kind, n, nflows=1500, seed=s) for s in (0, 7, 9)]
    dbs = [gpu_ctx.upload(t.frames, t.off, t.len, frames_bytes=t.frames_bytes, max_len=t.max_len) for t in trs]
    q = gpu_ctx.queue_ex(dbs, flow_hash=True, match=True)
    try:
        for ps, wait in ((program_sets(z, progs)[0][0][:8], True), (random_sets(11, 1)[0], False)):
            _set(gpu_ctx, ps, wait)
            q.run()
            for t, d in zip(trs, dbs):
                orec, ofh = O.classify_fh(t.frames[:t.frames_bytes], t.off, t.len, O.params())
                assert_records_equal(d.results(), orec, "records")
                np.testing.assert_array_equal(d.flow_hashes(), ofh)
                np.testing.assert_array_equal(d.matches(), O.bpf_eval(ps, t.frames[:t.frames_bytes], t.off, t.len))
        gpu_ctx.bpf_wait()
    finally:
        q.destroy()
        for d in dbs:
            d.free()


def test_set_async_returns_at_once_and_interp_until_compiled(gpu_ctx):
    """A set never seen before: mosrx_bpf_set_async returns in far less than a
    compile, the set runs on the interpreter meanwhile (same masks), and the
    compiled kernels replace it once the compile thread is done."""
    gpu_ctx.set_params(mosrx.default_params())
    t = mosrx.Trace(mosrx.TRACE_IMIX, 20_000, nflows=900)
    db = gpu_ctx.upload(t.frames, t.off, t.len, frames_bytes=t.frames_bytes, max_len=t.max_len)
    ora = O.classify(t.frames[:t.frames_bytes], t.off, t.len, O.params())
    try:
        for seed in (101, 102):
            ps = random_sets(seed, 1)[0]              # content never installed before: a compile
            om = O.bpf_eval(ps, t.frames[:t.frames_bytes], t.off, t.len)
            t0 = time.perf_counter()
            gpu_ctx.bpf_set_async(ps)
            dt = time.perf_counter() - t0
            assert dt < 0.05, f"bpf_set_async took {dt * 1e3:.1f} ms"
            assert gpu_ctx.bpf_pending()
            assert gpu_ctx.bpf_engine() == mosrx.BPF_ENGINE_INTERP
            gpu_ctx.classify_bpf_dev(db)
            np.testing.assert_array_equal(db.matches(), om)
            assert_records_equal(db.results(), ora, "records (interpreter)")
            t0 = time.perf_counter()
            gpu_ctx.bpf_wait()
            compile_s = time.perf_counter() - t0
            assert not gpu_ctx.bpf_pending()
            assert gpu_ctx.bpf_engine() == mosrx.BPF_ENGINE_JIT and gpu_ctx.bpf_fused(), gpu_ctx.bpf_jit_log()
            gpu_ctx.classify_bpf_dev(db)
            np.testing.assert_array_equal(db.matches(), om)
            assert_records_equal(db.results(), ora, "records (fused)")
            print(f"set_async {dt * 1e6:.0f} us, compile behind it {compile_s * 1e3:.0f} ms")
            # the same content again: from the cache, no compile
            gpu_ctx.bpf_set_async([])
            t0 = time.perf_counter()
            gpu_ctx.bpf_set_async(ps)
            assert not gpu_ctx.bpf_pending() and gpu_ctx.bpf_fused()
            assert time.perf_counter() - t0 < 0.05
    finally:
        db.free()


def test_back_to_back_sets_while_compiling(gpu_ctx):
    """Sets replaced faster than they compile: each is in effect when installed
    (the interpreter, then its own kernels), never an older set's kernels."""
    gpu_ctx.set_params(mosrx.default_params())
    t = mosrx.Trace(mosrx.TRACE_S64, 32_768, nflows=500)
    db = gpu_ctx.upload(t.frames, t.off, t.len, frames_bytes=t.frames_bytes, max_len=t.max_len)
    try:
        sets = [random_sets(200 + s, 1)[0] for s in range(4)]
        for ps in sets + sets[::-1]:
            gpu_ctx.bpf_set_async(ps)
            gpu_ctx.classify_bpf_dev(db)
            np.testing.assert_array_equal(db.matches(), O.bpf_eval(ps, t.frames[:t.frames_bytes], t.off, t.len))
        gpu_ctx.bpf_wait()
        gpu_ctx.classify_bpf_dev(db)
        np.testing.assert_array_equal(db.matches(), O.bpf_eval(sets[0], t.frames[:t.frames_bytes], t.off, t.len))
    finally:
        db.free()


@pytest.mark.parametrize("group", [0, 3])
def test_backend_with_filters_keeps_groups_and_flow_hash(group):
    """gpu_module_func with monitor filters installed: groups of several batches per
    launch (auto and explicit), records, masks and flow hashes per batch through
    dev_ioctl, equal to the oracle."""
    z, progs = load()
    ps = program_sets(z, progs)[0][0][:8]
    t = mosrx.Trace(mosrx.TRACE_IMIX, 24_000, nflows=800)
    ora, ofh = O.classify_fh(t.frames, t.off, t.len, O.params())
    om = O.bpf_eval(ps, t.frames[:t.frames_bytes], t.off, t.len)
    src = mosrx.mem_source(t.frames, t.off, t.len, loops=1)
    be = mosrx.GpuBackend([src], batch=2000, pipeline=True, cpu=7, bpf=ps, group=group, flowhash=True,
                          timing=True)
    try:
        seen = 0
        while (n := be.recv_pkts(0)) > 0:
            assert_records_equal(be.results(0, n), ora[seen:seen + n], f"batch@{seen}")
            np.testing.assert_array_equal(be.matches(0, n), om[seen:seen + n])
            np.testing.assert_array_equal(be.fhashes(0, n), ofh[seen:seen + n])
            seen += n
        assert seen == t.n
        st = be.stats()
        assert st.rx_batches == -(-t.n // 2000)
        assert st.kernel_launches < st.rx_batches        # several batches per launch, filters or not
    finally:
        be.close()


def test_backend_set_bpf_ioctl_is_async():
    """dev_ioctl(MOSRX_PKT_SET_BPF) of a set never compiled returns at once (the
    mTCP thread does not wait for hipRTC) and the next batches carry its masks."""
    import ctypes as C
    t = mosrx.Trace(mosrx.TRACE_IMIX, 16_000, nflows=600)
    ora = O.classify(t.frames, t.off, t.len, O.params())
    src = mosrx.mem_source(t.frames, t.off, t.len, loops=1)
    be = mosrx.GpuBackend([src], batch=1000, pipeline=True, cpu=9, group=2)
    try:
        ps = random_sets(303, 1)[0]
        arr, keep = mosrx._bpf_progs(ps)

        class SetArg(C.Structure):
            _fields_ = [("progs", C.c_void_p), ("nprog", C.c_uint32)]
        a = SetArg(C.addressof(arr[0]), len(ps))
        n = be.recv_pkts(0)
        seen = n
        t0 = time.perf_counter()
        assert be.ioctl_raw(0, mosrx.PKT_SET_BPF, C.byref(a)) == 0
        dt = time.perf_counter() - t0
        assert dt < 0.05, f"SET_BPF took {dt * 1e3:.1f} ms"
        om = O.bpf_eval(ps, t.frames[:t.frames_bytes], t.off, t.len)
        while (n := be.recv_pkts(0)) > 0:
            assert_records_equal(be.results(0, n), ora[seen:seen + n], f"batch@{seen}")
            np.testing.assert_array_equal(be.matches(0, n), om[seen:seen + n])
            seen += n
        assert seen == t.n
    finally:
        be.close()


# ---------------------------------------------------------------- compact records
def project8(rec):
    """The oracle's 16-byte records projected onto mosrx_result8's fields."""
    out = np.zeros(len(rec), mosrx.RESULT8_DTYPE)
    for f in ("rss", "reason", "queue", "verdict", "tcp_flags"):
        out[f] = rec[f]
    return out


@pytest.mark.parametrize("skip_tcp", [1, 0])
@pytest.mark.parametrize("kind,n", [(mosrx.TRACE_S64, 32_768), (mosrx.TRACE_FW64, 10_000),
                                    (mosrx.TRACE_IMIX, 50_000)])
def test_compact_records(gpu_ctx, kind, n, skip_tcp):
    """8-byte records (one launch and the batch queue) equal the oracle's full
    records projected, header-only (config #2) and full verdict."""
    p = mosrx.default_params(skip_tcp_csum=skip_tcp)
    gpu_ctx.set_params(p)
    trs = [mosrx.Trace(kind, n, nflows=1000, seed=s) for s in (0, 3)]
    dbs = [gpu_ctx.upload(t.frames, t.off, t.len, frames_bytes=t.frames_bytes, max_len=t.max_len) for t in trs]
    try:
        exp = [project8(O.classify(t.frames[:t.frames_bytes], t.off, t.len, O.params(skip_tcp_csum=skip_tcp)))
               for t in trs]
        for d, e in zip(dbs, exp):
            gpu_ctx.classify_dev_compact(d)
            assert np.array_equal(d.results8().view(np.uint8), e.view(np.uint8))
            d.d_out8.upload(np.zeros(d.n * 8, np.uint8))
        q = gpu_ctx.queue_ex(dbs, compact=True)
        q.run()
        q.destroy()
        for d, e in zip(dbs, exp):
            assert np.array_equal(d.results8().view(np.uint8), e.view(np.uint8))
    finally:
        for d in dbs:
            d.free()
        gpu_ctx.set_params(mosrx.default_params())


def test_compact_records_golden(gpu_ctx):
    """The reference fixtures' frames (the ihl 0..4 quirk, options, mutations)
    under their stack states, compact records against mOS's own values."""
    import os
    z = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "edge.npz"))
    frames, off, ln = z["frames"], z["off"], z["len"]
    for p in (mosrx.default_params(), mosrx.default_params(num_msp=0), mosrx.default_params(skip_tcp_csum=1)):
        gpu_ctx.set_params(p)
        op = O.params(num_msp=p.num_msp, skip_tcp_csum=p.skip_tcp_csum)
        db = gpu_ctx.upload(frames, off, ln)
        gpu_ctx.classify_dev_compact(db)
        got = db.results8()
        db.free()
        assert np.array_equal(got.view(np.uint8), project8(O.classify(frames, off, ln, op)).view(np.uint8))
    gpu_ctx.set_params(mosrx.default_params())


@pytest.mark.parametrize("kind,n,nb", [(mosrx.TRACE_IMIX, 40_000, 5), (mosrx.TRACE_S64, 65_536, 8)])
@pytest.mark.parametrize("mode", ["fused", "interp", "nofilter"])
def test_group_submit_c8(gpu_ctx, kind, n, nb, mode):
    """mosrx_classify_host_group_submit_c8 / _bpf_c8: a group's 8-byte records, flow
    hashes and (with a set) masks from one launch (the fused kernel's 8-byte form)
    or the classify launch + the interpreter per batch, equal to the oracle."""
    z, progs = load()
    ps = program_sets(z, progs)[0][0][:8]
    t = mosrx.Trace(kind, n, nflows=2000, seed=5)
    gpu_ctx.set_params(mosrx.default_params())
    gpu_ctx.bpf_set_engine(mosrx.BPF_ENGINE_INTERP if mode == "interp" else mosrx.BPF_ENGINE_JIT)
    try:
        if mode != "nofilter":
            _set(gpu_ctx, ps)
            assert gpu_ctx.bpf_fused() == (mode == "fused"), gpu_ctx.bpf_jit_log()
        batches, parts, base = _host_group(gpu_ctx, t, nb)
        recs = [np.zeros(b.n, mosrx.RESULT8_DTYPE) for b in batches]
        fhs = [np.zeros(b.n, np.uint32) for b in batches]
        mts = [np.full(b.n, 0xDEADBEEF, np.uint32) for b in batches]
        gpu_ctx.group_submit_c8(0, batches, [r.ctypes.data for r in recs], [f.ctypes.data for f in fhs],
                                None if mode == "nofilter" else [m.ctypes.data for m in mts])
        gpu_ctx.group_wait(0)
        for i, (fr, o, ln, fb) in enumerate(parts):
            orec, ofh = O.classify_fh(fr[:fb], o, ln, O.params())
            assert np.array_equal(recs[i].view(np.uint8), project8(orec).view(np.uint8)), f"batch {i}"
            np.testing.assert_array_equal(fhs[i], ofh)
            if mode != "nofilter":
                np.testing.assert_array_equal(mts[i], O.bpf_eval(ps, fr[:fb], o, ln))
        gpu_ctx.host_free(base)
    finally:
        gpu_ctx.bpf_set_async([])
        gpu_ctx.bpf_set_engine(mosrx.BPF_ENGINE_JIT)


def test_queue_compact_with_masks_and_hashes(gpu_ctx):
    """A resident queue with 8-byte records, flow hashes and masks (ABI 3 lifts
    the compact queue's side-array restriction)."""
    z, progs = load()
    gpu_ctx.set_params(mosrx.default_params())
    trs = [mosrx.Trace(mosrx.TRACE_IMIX, 30_000, nflows=1500, seed=s) for s in (1, 2)]
    dbs = [gpu_ctx.upload(t.frames, t.off, t.len, frames_bytes=t.frames_bytes, max_len=t.max_len) for t in trs]
    q = gpu_ctx.queue_ex(dbs, flow_hash=True, match=True, compact=True)
    try:
        ps = program_sets(z, progs)[0][0][:8]
        _set(gpu_ctx, ps)
        q.run()
        for t, d in zip(trs, dbs):
            orec, ofh = O.classify_fh(t.frames[:t.frames_bytes], t.off, t.len, O.params())
            assert np.array_equal(d.results8().view(np.uint8), project8(orec).view(np.uint8))
            np.testing.assert_array_equal(d.flow_hashes(), ofh)
            np.testing.assert_array_equal(d.matches(), O.bpf_eval(ps, t.frames[:t.frames_bytes], t.off, t.len))
    finally:
        q.destroy()
        gpu_ctx.bpf_set_async([])
        for d in dbs:
            d.free()


@pytest.mark.parametrize("group", [0, 3])
def test_backend_compact_with_filters(group):
    """gpu_module_func with cfg.compact and monitor filters: 8-byte records, masks
    and flow hashes per batch through dev_ioctl, equal to the oracle."""
    z, progs = load()
    ps = program_sets(z, progs)[0][0][:8]
    t = mosrx.Trace(mosrx.TRACE_IMIX, 24_000, nflows=800, seed=3)
    ora, ofh = O.classify_fh(t.frames, t.off, t.len, O.params())
    om = O.bpf_eval(ps, t.frames[:t.frames_bytes], t.off, t.len)
    src = mosrx.mem_source(t.frames, t.off, t.len, loops=1)
    be = mosrx.GpuBackend([src], batch=2000, pipeline=True, cpu=8, bpf=ps, group=group, flowhash=True,
                          compact=True)
    try:
        seen = 0
        while (n := be.recv_pkts(0)) > 0:
            got = be.results8(0, n)
            assert np.array_equal(got.view(np.uint8), project8(ora[seen:seen + n]).view(np.uint8)), f"@{seen}"
            np.testing.assert_array_equal(be.matches(0, n), om[seen:seen + n])
            np.testing.assert_array_equal(be.fhashes(0, n), ofh[seen:seen + n])
            seen += n
        assert seen == t.n
    finally:
        be.close()
