"""The uniform-layout hint (mosrx_batch.layout = MOSRX_BATCH_UNIFORM, ABI 3).

A batch packed at a fixed stride (an rx ring of fixed-size buffers, the
backend's stage of equal 64 B frames) may say so; the SMALL tile then loads
each frame's header window from off0 + i * stride together with its
descriptor instead of behind it.  off[] still decides: a lane whose offset
differs reloads, so a wrong hint may cost time but never changes a record.
Checked here against the oracle with right hints, hints wrong for a few lanes,
wholly wrong hints and hints outside the 16-bit packing, through the single
launch, the compact records and the batch queue (hinted and unhinted batches
mixed in one launch).  References: eth_in.c:27-87, ip_in.c:30-101, tcp.c:408-445
(the records), core.c:899-906 (the rx batches the hint describes)."""
import numpy as np
import pytest

import mosrx
import oracle_py as O
from test_parity_gpu import assert_records_equal, oparams

pytestmark = pytest.mark.gpu


def uniform_trace(n=32_768, kind=mosrx.TRACE_S64, seed=0):
    t = mosrx.Trace(kind, n, seed=seed)
    assert mosrx.uniform_layout(t.off) is not None
    return t


def relocate(t, lanes):
    """A copy of t's buffer with frames `lanes` moved past the end (their offsets
    changed), so the original layout hint is wrong exactly for those lanes."""
    frames = np.concatenate([t.frames[:t.frames_bytes], np.zeros(len(lanes) * 64 + 64, np.uint8)])
    off = t.off.copy()
    at = (t.frames_bytes + 15) & ~15
    for i in lanes:
        o, ln = int(t.off[i]), int(t.len[i])
        frames[at + 2:at + 2 + ln] = t.frames[o:o + ln]
        frames[o:o + ln] = 0xA5                      # the hinted address now holds garbage
        off[i] = at + 2
        at += 64
    return frames, off, t.len.copy(), at


def check(ctx, frames, off, ln, fb, hint, p, compact=False):
    ctx.set_params(p)
    ora = O.classify(frames[:fb], off, ln, oparams(p))
    db = ctx.upload(frames, off, ln, frames_bytes=fb, hint=hint)
    try:
        ctx.classify_dev(db)
        assert_records_equal(db.results(), ora, f"classify_dev hint={hint}")
        if compact:
            ctx.classify_dev_compact(db)
            r8 = db.results8()
            for f in ("rss", "reason", "queue", "verdict", "tcp_flags"):
                np.testing.assert_array_equal(r8[f], ora[f], err_msg=f"compact {f} hint={hint}")
    finally:
        db.free()
    return ora


@pytest.mark.parametrize("skip", [0, 1])
def test_right_hint_matches_oracle(gpu_ctx, skip):
    t = uniform_trace()
    check(gpu_ctx, t.frames, t.off, t.len, t.frames_bytes, mosrx.uniform_layout(t.off),
          mosrx.default_params(skip_tcp_csum=skip), compact=True)


@pytest.mark.parametrize("lanes", [[0], [63], [64, 65, 200], list(range(1000, 1256)), [32_767],
                                   list(range(0, 32_768, 97))])
def test_hint_wrong_for_some_lanes(gpu_ctx, lanes):
    """The hint describes the original layout; the listed frames were moved and
    their hinted addresses overwritten with garbage: those lanes must reload."""
    t = uniform_trace(seed=5)
    frames, off, ln, fb = relocate(t, lanes)
    check(gpu_ctx, frames, off, ln, fb, mosrx.uniform_layout(t.off), mosrx.default_params(), compact=True)


@pytest.mark.parametrize("hint", [(2, 60), (18, 64), (0, 64), (2, 1), (2, 0xFFFF), (0xFFFF, 64),
                                  (0x10000, 64), (2, 0x10000), (0xFFFFFFF0, 64)])
def test_wholly_wrong_or_unpackable_hint(gpu_ctx, hint):
    t = uniform_trace(n=20_000, seed=9)
    check(gpu_ctx, t.frames, t.off, t.len, t.frames_bytes, hint, mosrx.default_params(), compact=True)


def test_hint_on_non_small_batches_and_random_layouts(gpu_ctx):
    """Frames past the SMALL window (the stream tile takes no hint) and an
    irregular layout with a made-up hint: records unchanged."""
    t = mosrx.Trace(mosrx.TRACE_IMIX, 30_000, nflows=5000)
    check(gpu_ctx, t.frames, t.off, t.len, t.frames_bytes, (2, 64), mosrx.default_params())
    rng = np.random.default_rng(3)
    u = uniform_trace(n=5000, seed=3)
    perm = rng.permutation(u.n)                      # frames in shuffled descriptor order
    check(gpu_ctx, u.frames, u.off[perm].copy(), u.len[perm].copy(), u.frames_bytes,
          mosrx.uniform_layout(u.off), mosrx.default_params())


def test_tail_batches_and_tiny(gpu_ctx):
    for n in (1, 2, 63, 255, 256, 257, 1000):
        t = uniform_trace(n=max(n, 2), seed=n)
        off, ln = t.off[:n].copy(), t.len[:n].copy()
        fb = int(off[-1]) + int(ln[-1])
        check(gpu_ctx, t.frames, off, ln, fb, (int(t.off[0]), int(t.off[1]) - int(t.off[0])),
              mosrx.default_params())


@pytest.mark.parametrize("compact", [False, True])
def test_queue_mixes_hinted_and_plain_batches(gpu_ctx, compact):
    p = mosrx.default_params()
    gpu_ctx.set_params(p)
    dbs, oras = [], []
    for i in range(6):
        t = uniform_trace(n=32_768 if i % 2 else 20_000, seed=40 + i)
        frames, off, ln, fb = t.frames, t.off, t.len, t.frames_bytes
        hint = "auto" if i % 3 == 0 else None if i % 3 == 1 else mosrx.uniform_layout(t.off)
        if i == 5:                                   # a hinted batch whose hint is wrong for some lanes
            frames, off, ln, fb = relocate(t, [7, 300, 9000])
            hint = mosrx.uniform_layout(t.off)
        oras.append(O.classify(frames[:fb], off, ln, oparams(p)))
        dbs.append(gpu_ctx.upload(frames, off, ln, frames_bytes=fb, hint=hint))
    q = gpu_ctx.queue_ex(dbs, compact=compact)
    try:
        q.run()
        for d, ora in zip(dbs, oras):
            if compact:
                r8 = d.results8()
                for f in ("rss", "reason", "queue", "verdict", "tcp_flags"):
                    np.testing.assert_array_equal(r8[f], ora[f])
            else:
                assert_records_equal(d.results(), ora, "queue")
    finally:
        q.destroy()
        for d in dbs:
            d.free()


@pytest.mark.parametrize("group", [1, 4, 0])
def test_backend_stage_carries_the_hint(gpu_ctx, group):
    """The gpu_module backend's stage of equal 60 B frames (packed back to back
    by the fill) is handed over with its stride, through one launch per batch,
    explicit groups and auto groups; the records equal the oracle's."""
    t = uniform_trace(n=50_000, seed=77)
    p = mosrx.default_params()
    src = mosrx.mem_source(t.frames, t.off, t.len, loops=1, mode=mosrx.SRC_FILL)
    be = mosrx.GpuBackend([src], params=p, batch=8192, pipeline=True, group=group)
    try:
        got = []
        while True:
            n = be.recv_pkts(0)
            if n <= 0:
                break
            got.append(be.results(0, n).copy())
    finally:
        be.close()
    out = np.concatenate(got)
    assert len(out) == t.n
    assert_records_equal(out, O.classify(t.frames[:t.frames_bytes], t.off, t.len, oparams(p)), "backend")
