"""GPU parity: the HIP path (through the C ABI) against the oracle and the
reference-generated golden vectors.  Bit-exact on all 16 bytes of every record.

Runs on the MI355X box (`pytest -m gpu`).  The oracle is the checker only."""
import os
import random
import struct

import numpy as np
import pytest

import mosrx
import oracle_py as O
from pktlib import NREASON, R, REF_FIELDS, icmp_frame, pack_frames, tcp_frame
from test_oracle_golden import FIXTURES, GOLDEN, LOCAL, STATES, compare_with_ref

pytestmark = pytest.mark.gpu


def oparams(p: mosrx.Params) -> O.Params:
    q = O.Params()
    for f, _ in mosrx.Params._fields_:
        setattr(q, f, getattr(p, f))
    return q


def assert_records_equal(gpu, ora, what=""):
    g = gpu.view(np.uint8).reshape(-1, 16)
    o = ora.view(np.uint8).reshape(-1, 16)
    bad = np.nonzero(np.any(g != o, axis=1))[0]
    if len(bad):
        i = bad[0]
        raise AssertionError(f"{what}: {len(bad)} records differ; first #{i}: gpu={gpu[i]} oracle={ora[i]}")


def run_both(ctx, buf, off, ln, p, frames_bytes=None, dev=True, max_len=None, side=False):
    """Records through classify_host and classify_dev against the oracle; with
    `side`, also the flow hashes and pkt_info TCP fields (classify_*_ex)."""
    ctx.set_params(p)
    fb = len(buf) if frames_bytes is None else frames_bytes
    ora, ofh, oti = O.classify_ex(buf[:fb], off, ln, oparams(p))
    host = ctx.classify_host(buf, off, ln, frames_bytes=fb, max_len=max_len or 0)
    assert_records_equal(host, ora, "classify_host")
    if side:
        host, fh, ti = ctx.classify_host_ex(buf, off, ln, frames_bytes=fb, max_len=max_len or 0)
        assert_records_equal(host, ora, "classify_host_ex")
        np.testing.assert_array_equal(fh, ofh)
        np.testing.assert_array_equal(ti, oti)
    if dev:
        db = ctx.upload(buf, off, ln, frames_bytes=fb, max_len=max_len)
        ctx.classify_dev(db)
        assert_records_equal(db.results(), ora, "classify_dev")
        if side:
            ctx.classify_dev(db, flow_hash=True, tcpinfo=True)
            assert_records_equal(db.results(), ora, "classify_dev_ex")
            np.testing.assert_array_equal(db.flow_hashes(), ofh)
            np.testing.assert_array_equal(db.tcpinfo(), oti)
        db.free()
    return ora


def state_params(state, **kw):
    msp, esp, nq, qm, loc = STATES[state]
    return mosrx.default_params(num_msp=msp, num_esp=esp, forward=0, num_queues=nq, queue_mode=qm,
                                local=loc, **kw)


@pytest.mark.parametrize("fix", FIXTURES)
@pytest.mark.parametrize("state", list(STATES))
def test_golden_fixtures(gpu_ctx, fix, state):
    """Every record field, the flow hash and pkt_info's TCP fields against mOS's
    own outputs (ProcessPacket, ip_fast_csum, TCPCalcChecksum, GetRSSHash /
    GetRSSCPUCore, HashFlow, FillPacketContextTCPInfo) under all 11 stack states."""
    z = np.load(os.path.join(GOLDEN, f"{fix}.npz"))
    p = state_params(state)
    gpu_ctx.set_params(p)
    out, fh, ti = gpu_ctx.classify_host_ex(z["frames"], z["off"], z["len"])
    ref = {k: z[f"{state}__{k}"] for k in REF_FIELDS}
    compare_with_ref(out, ref, p, fh, ti)                          # against mOS itself
    ora, ofh, oti = O.classify_ex(z["frames"], z["off"], z["len"], oparams(p))
    assert_records_equal(out, ora, fix)
    np.testing.assert_array_equal(fh, ofh)
    np.testing.assert_array_equal(ti, oti)
    # the device-resident form on the same frames, every shape
    for v in (mosrx.shape_variant(mosrx.KIND_SMALL), mosrx.shape_variant(mosrx.KIND_S13), 2):
        gpu_ctx.set_variant(v)
        try:
            db = gpu_ctx.upload(z["frames"], z["off"], z["len"])
            gpu_ctx.classify_dev(db, flow_hash=True, tcpinfo=True)
            res, dfh, dti = db.results(), db.flow_hashes(), db.tcpinfo()
            db.free()
        finally:
            gpu_ctx.set_variant(2)
        assert_records_equal(res, ora, f"{fix} dev variant {v}")
        np.testing.assert_array_equal(dfh, ofh)
        np.testing.assert_array_equal(dti, oti)


@pytest.mark.parametrize("fix", FIXTURES)
@pytest.mark.parametrize("state", ["msp1", "noverify", "msp1_esp1_listen", "msp1_local"])
def test_golden_forward_on(gpu_ctx, fix, state):
    """mos.conf `forward = 1`: the GPU verdicts against mOS's own ProcessPacket
    with forwarding on (tests/golden/forward.npz), and the frames the rx loop's
    forwarding rule picks from the GPU records against the frames mOS forwarded."""
    from test_forwarding import FSTATES, FWD, check
    z = np.load(os.path.join(GOLDEN, f"{fix}.npz"))
    msp, esp, loc, listen = FSTATES[state]
    p = mosrx.default_params(num_msp=msp, num_esp=esp, forward=1, local=loc)
    k = f"{fix}__{state}__"
    for v in (mosrx.shape_variant(mosrx.KIND_SMALL), mosrx.shape_variant(mosrx.KIND_S13)):
        gpu_ctx.set_variant(v)
        try:
            out = run_both(gpu_ctx, z["frames"], z["off"], z["len"], p)
            gpu = gpu_ctx.classify_host(z["frames"], z["off"], z["len"])
        finally:
            gpu_ctx.set_variant(2)
        assert_records_equal(gpu, out, f"{fix} variant {v}")
        check(gpu, FWD[k + "verdict"], FWD[k + "fwd"], FWD[k + "have"], msp, listen)


@pytest.mark.parametrize("kind,n", [(mosrx.TRACE_FW64, 10_000), (mosrx.TRACE_S64, 32_768),
                                    (mosrx.TRACE_M1500, 65_536), (mosrx.TRACE_IMIX, 262_144)])
def test_baseline_configs_full_size(gpu_ctx, kind, n):
    t = mosrx.Trace(kind, n)
    p = mosrx.default_params()
    ora = run_both(gpu_ctx, t.frames, t.off, t.len, p, frames_bytes=t.frames_bytes, max_len=t.max_len)
    idx = np.arange(n)
    assert np.all(ora["reason"][idx % 1024 == 511] == R["IP_BADCSUM"])
    assert np.all(ora["reason"][idx % 1024 == 1023] == R["TCP_BADCSUM"])
    # size-independent property: the verdict census equals the generator's corruption schedule
    assert (ora["verdict"] == 1).sum() == n - ((idx % 1024 == 511) | (idx % 1024 == 1023)).sum()


def test_skip_tcp_mode_config2(gpu_ctx):
    t = mosrx.Trace(mosrx.TRACE_S64, 32_768)
    p = mosrx.default_params(skip_tcp_csum=1)
    ora = run_both(gpu_ctx, t.frames, t.off, t.len, p, frames_bytes=t.frames_bytes, max_len=t.max_len)
    assert np.all(ora["tcp_csum"] == 0)
    assert set(np.unique(ora["reason"]).tolist()) == {R["TCP_LEN_OK"], R["IP_BADCSUM"]}


@pytest.mark.parametrize("msp,esp,fwd,nq,qm", [(1, 0, 1, 1, 1), (0, 0, 1, 1, 1), (0, 1, 0, 1, 1),
                                               (1, 0, 0, 8, 1), (1, 1, 1, 5, 0), (1, 0, 1, 256, 1)])
def test_stack_states(gpu_ctx, msp, esp, fwd, nq, qm):
    z = np.load(os.path.join(GOLDEN, "edge.npz"))
    p = mosrx.default_params(num_msp=msp, num_esp=esp, forward=fwd, num_queues=nq, queue_mode=qm)
    run_both(gpu_ctx, z["frames"], z["off"], z["len"], p)


@pytest.mark.parametrize("key", [mosrx.MS_KEY, bytes(range(100, 152)), b"\xff" * 16])
def test_rss_keys(gpu_ctx, key):
    t = mosrx.Trace(mosrx.TRACE_IMIX, 20_000, nflows=5000)
    run_both(gpu_ctx, t.frames, t.off, t.len, mosrx.default_params(key=key, num_queues=16))


def test_msdn_vectors_through_the_kernel(gpu_ctx):
    z = np.load(os.path.join(GOLDEN, "rss_msdn_kat.npz"))
    frames = []
    for v in z["kat"]:
        s = ".".join(str(b) for b in struct.pack("!I", int(v["sip"])))
        d = ".".join(str(b) for b in struct.pack("!I", int(v["dip"])))
        frames.append(tcp_frame(s, d, int(v["sp"]), int(v["dp"]), b"kat"))
    buf, off, ln = pack_frames(frames)
    gpu_ctx.set_params(mosrx.default_params(key=mosrx.MS_KEY))
    out = gpu_ctx.classify_host(buf, off, ln)
    assert out["rss"].tolist() == [int(h) for h in z["kat"]["hash"]]


@pytest.mark.parametrize("phase", [0, 1, 3, 5, 7, 13])
def test_misaligned_layouts(gpu_ctx, phase):
    rng = random.Random(phase)
    from golden.make_golden import random_frames
    frames = random_frames(rng, 200, 0) + random_frames(rng, 100, 2) + random_frames(rng, 100, 1)
    rng.shuffle(frames)
    buf, off, ln = pack_frames(frames, align=rng.choice([1, 2, 4, 16]), phase=phase, gap=rng.randint(0, 5))
    run_both(gpu_ctx, buf, off, ln, mosrx.default_params(forward=0))


def test_buffer_end_exact(gpu_ctx):
    """Last frame ends exactly at frames_bytes (not a multiple of 16): no byte is lost."""
    for plen in range(0, 40):
        f = tcp_frame(payload=bytes(range(plen)), doff=8)
        buf, off, ln = pack_frames([tcp_frame(payload=b"x" * 100), f], phase=plen % 16)
        fb = int(off[-1]) + int(ln[-1])
        run_both(gpu_ctx, buf, off, ln, mosrx.default_params(), frames_bytes=fb)


def test_random_offsets_and_garbage(gpu_ctx):
    rng = np.random.default_rng(11)
    buf = rng.integers(0, 256, 300_000, dtype=np.uint8)
    n = 5000
    off = rng.integers(0, len(buf), n).astype(np.uint32)
    ln = rng.integers(0, 2000, n).astype(np.uint16)
    # make many of them reach deep paths: IPv4 ethertype, version 4, plausible ihl/tot_len
    for i in range(0, n, 2):
        o = int(off[i])
        if o + 40 < len(buf):
            buf[o + 12:o + 14] = (0x08, 0x00)
            buf[o + 14] = 0x40 | rng.integers(0, 16)
            tl = int(rng.integers(0, 1600))
            buf[o + 16:o + 18] = (tl >> 8, tl & 0xFF)
            buf[o + 23] = 6 if rng.random() < 0.8 else 17
    run_both(gpu_ctx, buf, off, ln, mosrx.default_params())
    run_both(gpu_ctx, buf, off, ln, mosrx.default_params(num_msp=0, num_esp=0))


def test_jumbo_and_max_lengths(gpu_ctx):
    frames = [tcp_frame(payload=bytes(range(256)) * (k // 256) + bytes(k % 256), doff=rng_d)
              for k, rng_d in [(8952, 5), (9000 - 52, 8), (65535 - 60, 5), (65535 - 20 - 60, 15), (30000, 6)]]
    frames = [f[:65535] for f in frames]
    buf, off, ln = pack_frames(frames)
    run_both(gpu_ctx, buf, off, ln, mosrx.default_params())


def test_empty_and_single(gpu_ctx):
    gpu_ctx.set_params(mosrx.default_params())
    out = gpu_ctx.classify_host(np.zeros(16, np.uint8), np.zeros(0, np.uint32), np.zeros(0, np.uint16))
    assert len(out) == 0
    buf, off, ln = pack_frames([tcp_frame(payload=b"one")])
    run_both(gpu_ctx, buf, off, ln, mosrx.default_params())


def test_counters_match_records(gpu_ctx):
    t = mosrx.Trace(mosrx.TRACE_IMIX, 50_000, nflows=1000)
    gpu_ctx.set_params(mosrx.default_params())
    out = gpu_ctx.classify_host(t.frames, t.off, t.len, frames_bytes=t.frames_bytes)
    cnt = gpu_ctx.last_counters()
    assert cnt.tolist() == np.bincount(out["reason"], minlength=NREASON).tolist()


def test_repeatable(gpu_ctx):
    t = mosrx.Trace(mosrx.TRACE_M1500, 8192, nflows=1000)
    gpu_ctx.set_params(mosrx.default_params())
    db = gpu_ctx.upload(t.frames, t.off, t.len, frames_bytes=t.frames_bytes, max_len=t.max_len)
    gpu_ctx.classify_dev(db)
    a = db.results()
    for _ in range(3):
        gpu_ctx.classify_dev(db)
        assert np.array_equal(a, db.results())
    db.free()


@pytest.mark.parametrize("pipeline", [True, False])
def test_gpu_io_module_rx_loop(pipeline):
    t = mosrx.Trace(mosrx.TRACE_IMIX, 30_000, nflows=2000)
    src = mosrx.mem_source(t.frames, t.off, t.len, loops=1)
    be = mosrx.GpuBackend([src], batch=4096, pipeline=pipeline, cpu=1 if pipeline else 2)
    try:
        st = be.run_loop()
    finally:
        be.close()
    ora = O.classify(t.frames, t.off, t.len, O.params())
    assert st.rx_packets == t.n
    assert st.rx_bytes == int(t.len.astype(np.uint64).sum()) + 24 * t.n
    assert st.rx_errors == int((ora["verdict"] < 0).sum())
    assert list(st.by_reason) == np.bincount(ora["reason"], minlength=NREASON).tolist()
    assert st.batches == (t.n + 4095) // 4096


@pytest.mark.parametrize("mode", [mosrx.SRC_BEST, mosrx.SRC_FILL, mosrx.SRC_PER_FRAME])
@pytest.mark.parametrize("max_frame", [2048, 600])
def test_gpu_io_module_replay_runs(max_frame, mode):
    """The in-memory source's batch fill (loopback.c mem_fill): runs of the
    replay buffer copied whole into the staging block and rebased, wrapping
    inside a batch across replay loops; with max_frame below the longest frame
    the per-frame truncating path runs instead.  Records match the oracle over
    the replayed (truncated) stream.  Every way a batch reaches the stage: the
    pinned replay buffer lent zero-copy, copied in runs, copied per frame."""
    t = mosrx.Trace(mosrx.TRACE_IMIX, 7000, nflows=300)
    src = mosrx.mem_source(t.frames, t.off, t.len, loops=3, mode=mode)
    be = mosrx.GpuBackend([src], batch=4096, max_frame=max_frame, pipeline=True, cpu=4)
    ln = np.minimum(t.len, max_frame).astype(np.uint16)
    ora = O.classify(t.frames, t.off, ln, O.params())
    try:
        seen = 0
        while True:
            n = be.recv_pkts(0)
            assert n >= 0
            if n == 0:
                break
            idx = (seen + np.arange(n)) % t.n
            assert_records_equal(be.results(0, n), ora[idx], f"batch@{seen}")
            for i in (0, n // 2, n - 1):
                j = int(idx[i])
                assert be.get_rptr(0, i) == bytes(t.frames[t.off[j]:t.off[j] + ln[j]])
            seen += n
        assert seen == 3 * t.n
    finally:
        be.close()


def test_gpu_io_module_batches_and_ioctl():
    t = mosrx.Trace(mosrx.TRACE_IMIX, 10_000, nflows=500)
    src = mosrx.mem_source(t.frames, t.off, t.len, loops=1)
    be = mosrx.GpuBackend([src], batch=3000, pipeline=True, cpu=3)
    ora = O.classify(t.frames, t.off, t.len, O.params())
    try:
        seen = 0
        while True:
            n = be.recv_pkts(0)
            assert n >= 0
            if n == 0:
                break
            res = be.results(0, n)
            assert_records_equal(res, ora[seen:seen + n], f"batch@{seen}")
            for i in (0, min(n, 128) - 1):
                assert be.get_rptr(0, i) == bytes(t.frames[t.off[seen + i]:t.off[seen + i] + t.len[seen + i]])
                assert be.rss_of(0, i) == int(ora["rss"][seen + i])
            assert be.get_rptr(0, n) is None
            seen += n
        assert seen == t.n
        assert be.recv_pkts(5) == -1          # bad ifidx, pcap_module.c:37-38
    finally:
        be.close()


@pytest.mark.parametrize("kind,sizes", [(mosrx.TRACE_S64, [5_000, 300, 70_001, 256, 1]),
                                        (mosrx.TRACE_IMIX, [3_000, 64, 9_100, 65])])
def test_batch_queue_unequal_batches(gpu_ctx, kind, sizes):
    """Batches of different tile counts: workgroups find their batch by the
    binary search of tile_base[] (equal batches take the division path)."""
    gpu_ctx.set_params(mosrx.default_params())
    trs = [mosrx.Trace(kind, n, nflows=2000, seed=300 + i) for i, n in enumerate(sizes)]
    dbs = [gpu_ctx.upload(t.frames, t.off, t.len, frames_bytes=t.frames_bytes, max_len=t.max_len) for t in trs]
    q = gpu_ctx.queue(dbs)
    q.run()
    for t, d in zip(trs, dbs):
        assert_records_equal(d.results(), O.classify(t.frames, t.off, t.len, O.params()), "queue (unequal)")
    q.destroy()
    for d in dbs:
        d.free()


@pytest.mark.parametrize("kind,n,nb", [(mosrx.TRACE_S64, 32_768, 8), (mosrx.TRACE_IMIX, 9_000, 5),
                                       (mosrx.TRACE_M1500, 9_000, 4)])
def test_batch_queue_one_launch(gpu_ctx, kind, n, nb):
    gpu_ctx.set_params(mosrx.default_params())
    trs = [mosrx.Trace(kind, n - 7 * i, nflows=4000, seed=100 + i) for i in range(nb)]
    dbs = [gpu_ctx.upload(t.frames, t.off, t.len, frames_bytes=t.frames_bytes, max_len=t.max_len) for t in trs]
    q = gpu_ctx.queue(dbs)
    q.run()
    for t, d in zip(trs, dbs):
        assert_records_equal(d.results(), O.classify(t.frames, t.off, t.len, O.params()), "queue")
    q.destroy()
    for d in dbs:
        d.free()


def test_dispatch_stamped_kernel_timing(gpu_ctx):
    """The bench's roofline duration (mosrx_time_op_dispatch / _queue_dispatch):
    every launch stamped by its own dispatch, so never longer than the same
    launches timed back to back with events around them (dispatch gaps
    included); the BPF op (the set's own kernel, or the interpreter) is one
    launch and is stamped too, with the oracle's masks; the stamped launches
    leave the same records."""
    gpu_ctx.set_params(mosrx.default_params())
    trs = [mosrx.Trace(mosrx.TRACE_M1500, 4096, nflows=4000, seed=200 + i) for i in range(2)]
    dbs = [gpu_ctx.upload(t.frames, t.off, t.len, frames_bytes=t.frames_bytes, max_len=t.max_len) for t in trs]
    stamped = gpu_ctx.time_op_dispatch(mosrx.OP_CLASSIFY, dbs, 64)
    b2b = gpu_ctx.time_dev_streams(dbs, 64, 1) / 64
    assert 0 < stamped <= b2b * 1.02, (stamped, b2b)
    for t, d in zip(trs, dbs):
        assert_records_equal(d.results(), O.classify(t.frames, t.off, t.len, O.params()), "stamped")
    # the stamp's reading for an empty kernel of the same grid (the bench's short-row floor):
    # positive, and no longer than the classify launch it is stated against
    floor = gpu_ctx.probe_stamp_floor(dbs[0], 64)
    assert 0 < floor <= stamped * 1.05, (floor, stamped)
    gpu_ctx.time_op(mosrx.OP_CLASSIFY_FH, dbs, 2, kernels=False)                # side buffers allocated
    assert gpu_ctx.time_op_dispatch(mosrx.OP_CLASSIFY_FH, dbs, 16) > 0
    progs = [(np.array([(0x28, 0, 0, 12), (0x15, 0, 1, 0x800), (0x06, 0, 0, 1), (0x06, 0, 0, 0)],
                       mosrx.BPF_INSN), 0)]
    gpu_ctx.bpf_set(progs)
    for d in dbs:
        gpu_ctx.bpf_dev(d)                                                   # match buffers allocated
    assert gpu_ctx.time_op_dispatch(mosrx.OP_BPF, dbs, 4) > 0
    for t, d in zip(trs, dbs):
        np.testing.assert_array_equal(d.matches(), O.bpf_eval(progs, t.frames[:t.frames_bytes], t.off, t.len))
    gpu_ctx.bpf_set([])
    q = gpu_ctx.queue(dbs)
    qs = q.time_dispatch(16)
    qb = q.time(16, kernels=False)[0] / 16
    assert 0 < qs <= qb * 1.02, (qs, qb)
    q.destroy()
    for d in dbs:
        d.free()


# kernel shapes forced through variant bits 2-6 (value - 1: SMALL, S13) with both tail-load
# cache policies; every shape must be exact on every frame mix
STREAM_VARIANTS = [mosrx.shape_variant(mosrx.KIND_S13), mosrx.shape_variant(mosrx.KIND_S13, False)]
ALL_VARIANTS = [2, 0, mosrx.shape_variant(mosrx.KIND_SMALL), mosrx.shape_variant(mosrx.KIND_SMALL, False)] + STREAM_VARIANTS


@pytest.mark.parametrize("variant", ALL_VARIANTS)
@pytest.mark.parametrize("kind,n", [(mosrx.TRACE_S64, 20_000), (mosrx.TRACE_M1500, 9_000),
                                    (mosrx.TRACE_IMIX, 30_000)])
def test_forced_kernel_shapes(gpu_ctx, variant, kind, n):
    t = mosrx.Trace(kind, n, seed=variant)
    gpu_ctx.set_variant(variant)
    try:
        run_both(gpu_ctx, t.frames, t.off, t.len, mosrx.default_params(),
                 frames_bytes=t.frames_bytes, max_len=t.max_len)
        z = np.load(os.path.join(GOLDEN, "rand_mid.npz"))
        run_both(gpu_ctx, z["frames"], z["off"], z["len"], mosrx.default_params(forward=0))
    finally:
        gpu_ctx.set_variant(2)


@pytest.mark.parametrize("fix", FIXTURES)
def test_flow_hash_golden(gpu_ctx, fix):
    # HashFlow bucket (fhash.c:72-92) of FindStream's reversed tuple (tcp.c:185-190)
    z = np.load(os.path.join(GOLDEN, f"{fix}.npz"))
    p = mosrx.default_params(forward=0)
    gpu_ctx.set_params(p)
    out, fh = gpu_ctx.classify_host_fh(z["frames"], z["off"], z["len"])
    ref = {k: z[f"msp1__{k}"] for k in REF_FIELDS}
    compare_with_ref(out, ref, p, fh)                               # against mOS itself
    ora, ofh = O.classify_fh(z["frames"], z["off"], z["len"], oparams(p))
    assert_records_equal(out, ora, fix)
    np.testing.assert_array_equal(fh, ofh)


@pytest.mark.parametrize("variant", ALL_VARIANTS)
@pytest.mark.parametrize("kind,n", [(mosrx.TRACE_S64, 32_768), (mosrx.TRACE_M1500, 16_384),
                                    (mosrx.TRACE_IMIX, 65_536)])
def test_flow_hash_device(gpu_ctx, variant, kind, n):
    t = mosrx.Trace(kind, n, nflows=5000)
    p = mosrx.default_params()
    gpu_ctx.set_params(p)
    gpu_ctx.set_variant(variant)
    try:
        db = gpu_ctx.upload(t.frames, t.off, t.len, frames_bytes=t.frames_bytes, max_len=t.max_len)
        gpu_ctx.classify_dev(db, flow_hash=True)
        res, fh = db.results(), db.flow_hashes()
        gpu_ctx.classify_dev(db, flow_hash=True, tcpinfo=True)
        res2, fh2, ti = db.results(), db.flow_hashes(), db.tcpinfo()
        db.free()
    finally:
        gpu_ctx.set_variant(2)
    ora, ofh, oti = O.classify_ex(t.frames[:t.frames_bytes], t.off, t.len, oparams(p))
    assert_records_equal(res, ora, "classify_dev_fh")
    np.testing.assert_array_equal(fh, ofh)
    assert_records_equal(res2, ora, "classify_dev_ex")
    np.testing.assert_array_equal(fh2, ofh)
    np.testing.assert_array_equal(ti, oti)
    # size-independent property: the generator advances seq by the payload per flow and acks 1
    tcp = ora["payload_off"] != 0
    assert np.all(ti["ip_len"][tcp] == t.len[tcp] - 14)
    # size-independent property: frames of one flow share a bucket; 5000 flows -> <= 5000 buckets
    assert len(np.unique(fh[ora["payload_off"] != 0] & 0x1FFFF)) <= 5000


# Stream shapes on the layouts that stress the span walk: tight packing at any
# alignment (owners change inside a wave load), jumbo frames longer than a
# streamer's run (one frame flushed by several streamers), frames out of buffer
# order (the per-frame fallback), the last frame ending at the buffer end.
@pytest.mark.parametrize("variant", STREAM_VARIANTS)
def test_stream_shapes_layouts(gpu_ctx, variant):
    gpu_ctx.set_variant(variant)
    try:
        rng = random.Random(variant)
        from golden.make_golden import random_frames
        for phase in (0, 1, 2, 7):
            frames = random_frames(rng, 300, 0) + random_frames(rng, 150, 2) + random_frames(rng, 150, 1)
            rng.shuffle(frames)
            buf, off, ln = pack_frames(frames, align=rng.choice([1, 2, 16]), phase=phase, gap=rng.randint(0, 3))
            run_both(gpu_ctx, buf, off, ln, mosrx.default_params(forward=0))
            # same frames, descriptors in reverse buffer order: unsorted tiles
            run_both(gpu_ctx, buf, off[::-1].copy(), ln[::-1].copy(), mosrx.default_params(forward=0))
        big = [tcp_frame(payload=bytes(rng.getrandbits(8) for _ in range(k)), doff=5)
               for k in (65535 - 54, 30000, 9000, 3000, 1500, 600, 10)]
        buf, off, ln = pack_frames(big * 3, phase=3)
        run_both(gpu_ctx, buf, off, ln, mosrx.default_params())
        for plen in (0, 1, 15, 16, 17, 1000, 1447):
            f = tcp_frame(payload=bytes(range(256)) * (plen // 256) + bytes(plen % 256), doff=8)
            buf, off, ln = pack_frames([tcp_frame(payload=b"x" * 1400), f], phase=plen % 16)
            run_both(gpu_ctx, buf, off, ln, mosrx.default_params(), frames_bytes=int(off[-1]) + int(ln[-1]))
        rb = np.random.default_rng(variant)
        buf = rb.integers(0, 256, 200_000, dtype=np.uint8)
        off = np.sort(rb.integers(0, len(buf) - 2000, 3000)).astype(np.uint32)
        ln = rb.integers(0, 2000, 3000).astype(np.uint16)          # sorted offsets, overlapping captures
        run_both(gpu_ctx, buf, off, ln, mosrx.default_params())
    finally:
        gpu_ctx.set_variant(2)


def test_bogus_offsets_after_sorted_frames(gpu_ctx):
    """Descriptors in buffer order whose last entries point past the buffer (or
    carry zero length): the tail span stops at the last frame with a tail."""
    frames = [tcp_frame(payload=bytes(range(200)) * 7) for _ in range(70)]
    buf, off, ln = pack_frames(frames)
    off = np.concatenate([off, np.array([len(buf) + 5, 0xFFFF0000, 0xFFFFFFF0], np.uint32)])
    ln = np.concatenate([ln, np.array([1500, 1500, 0], np.uint16)])
    for variant in STREAM_VARIANTS + [2]:
        gpu_ctx.set_variant(variant)
        try:
            run_both(gpu_ctx, buf, off, ln, mosrx.default_params())
        finally:
            gpu_ctx.set_variant(2)


@pytest.mark.parametrize("layout", ["frames_off_len", "off_len_frames", "gaps", "too_sparse", "overlap"])
def test_host_one_block_layouts(gpu_ctx, layout):
    """classify_host with frames and descriptors in one block (the gpu_module
    staging layout): one H2D copy of the span (mosrx_api.c batch_span), device
    pointers at the same relative offsets.  Sparse blocks, and descriptors lying
    inside frames_bytes, take the three-copy path; every layout gives the
    oracle's records and counters."""
    t = mosrx.Trace(mosrx.TRACE_IMIX, 5000, nflows=500)
    n, fb = t.n, int(t.frames_bytes)
    fa = (fb + 15) & ~15
    off, ln = np.asarray(t.off, np.uint32), np.asarray(t.len, np.uint16)
    gap = {"gaps": 4000, "too_sparse": 10 * fb}.get(layout, 0)
    if layout == "off_len_frames":
        d = (n * 6 + 15) & ~15
        blk = np.zeros(d + fb, np.uint8)
        o_at, l_at, f_at = 0, n * 4, d
    else:
        blk = np.zeros(fa + gap + n * 6 + 16, np.uint8)
        o_at, l_at, f_at = fa + gap, fa + gap + n * 4 + (16 if gap else 0), 0
    blk[f_at:f_at + fb] = np.asarray(t.frames[:fb], np.uint8)
    ov = blk[o_at:o_at + n * 4].view(np.uint32)
    lv = blk[l_at:l_at + n * 2].view(np.uint16)
    ov[:] = off
    lv[:] = ln
    if layout == "overlap":           # frames_bytes covers the descriptors too
        fb = len(blk) - f_at
    frames = blk[f_at:f_at + fb]
    p = mosrx.default_params()
    gpu_ctx.set_params(p)
    ora = O.classify(frames.copy(), off, ln, oparams(p))
    got = gpu_ctx.classify_host(frames, ov, lv, frames_bytes=fb, max_len=int(ln.max()))
    assert_records_equal(got, ora, layout)
    cnt = np.asarray(gpu_ctx.last_counters())
    assert cnt.sum() == n and np.array_equal(cnt, np.bincount(ora["reason"], minlength=len(cnt)))


def _options_frames(seed):
    """IP options of every length (ihl 5..15) and TCP options (doff 5..15) with
    segments ending inside the header window, just past it and far past it: the
    segment start 14+4*ihl then falls before, at and after the stream tile's
    split (frame byte 47..62) and the SMALL tile's (63..78), so the option bytes
    past the split are summed by the tail streamers and taken out again."""
    rng = random.Random(seed)
    frames = []
    for ihl in range(5, 16):
        for doff in (5, 8, 15):
            for plen in (0, 1, 7, 16, 33, 64, 95, 300, 1400 - 4 * (ihl + doff)):
                f = bytearray(tcp_frame(payload=bytes(rng.getrandbits(8) for _ in range(plen)), ihl=ihl, doff=doff,
                                        seq=rng.getrandbits(32)))
                if rng.random() < 0.3:                          # corrupt a byte of the segment or the options
                    f[rng.randint(14 + 20, len(f) - 1)] ^= 1 << rng.randint(0, 7)
                frames.append(bytes(f))
    rng.shuffle(frames)
    return frames


@pytest.mark.parametrize("variant", ALL_VARIANTS)
@pytest.mark.parametrize("phase", [0, 1, 2, 5, 9, 14])
def test_ip_options_across_the_split(gpu_ctx, variant, phase):
    frames = _options_frames(phase)
    buf, off, ln = pack_frames(frames, phase=phase, align=16)
    gpu_ctx.set_variant(variant)
    try:
        ora = run_both(gpu_ctx, buf, off, ln, mosrx.default_params(forward=0), side=True)
    finally:
        gpu_ctx.set_variant(2)
    # the trace reaches both verdicts of the TCP checksum on option-bearing frames
    ihl = (ora["ihl_doff"] >> 4)
    assert ((ihl > 5) & (ora["reason"] == R["TCP_OK"])).sum() > 50
    assert ((ihl > 5) & (ora["reason"] == R["TCP_BADCSUM"])).sum() > 5


@pytest.mark.parametrize("variant", [mosrx.shape_variant(mosrx.KIND_SMALL), mosrx.shape_variant(mosrx.KIND_S13)])
def test_ip_options_tx_rewrite(gpu_ctx, variant):
    """The TX rewrite shares the in-window sum: checks of option-bearing frames
    rewritten on the GPU equal the oracle's (mOS's arithmetic), both shapes."""
    frames = _options_frames(99)
    buf, off, ln = pack_frames(frames, phase=3)
    flags = mosrx.TX_IP_CSUM | mosrx.TX_TCP_CSUM
    exp = O.tx_csum(buf, off, ln, flags)
    gpu_ctx.set_variant(variant)
    try:
        np.testing.assert_array_equal(gpu_ctx.tx_csum_host(buf, off, ln, flags), exp)
    finally:
        gpu_ctx.set_variant(2)
