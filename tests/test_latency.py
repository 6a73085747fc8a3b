"""CPU tests of the drop-in path's latency instruments:
the paced source (csrc/loopback.c mosrx_source_paced), the residency probe
(csrc/rx_loop.c, mosrx_rx_loop_opts.probe) and the latency cap of the auto-group
policy (csrc/gpu_module.c group_cap, cfg.group_max_us), the last run through
gpu_module_func over the CPU stand-in for the GPU (oracle/_ref/libbackend_emul.so:
the oracle makes the records), so no GPU is needed.  The measured residencies
on the MI355X are bench.py's e2e.backend_latency legs."""
import ctypes as C
import os
import time

import numpy as np
import pytest

import mosrx

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EMUL = os.path.join(ROOT, "oracle", "_ref", "libbackend_emul.so")


def _now_ns():
    return time.clock_gettime_ns(time.CLOCK_MONOTONIC)


def test_paced_source_releases_frames_at_its_rate():
    tr = mosrx.Trace(mosrx.TRACE_S64, 4096)
    src = mosrx.paced_source(mosrx.mem_source(tr.frames, tr.off, tr.len, loops=0), 200_000.0)
    L = mosrx.lib()
    buf = np.zeros(1 << 22, np.uint8)
    off = np.zeros(65536, np.uint32)
    ln = np.zeros(65536, np.uint16)
    end = C.c_uint64()
    try:
        got = L.mosrx_source_fill(src, buf.ctypes.data, buf.nbytes, off.ctypes.data, ln.ctypes.data, 65536, 2048,
                                  C.byref(end))
        assert got == 1                       # frame 0 arrives at the first receive, the next 5 us later
        t0, nspf, rel = C.c_uint64(), C.c_double(), C.c_uint64()
        assert L.mosrx_source_paced_info(src, C.byref(t0), C.byref(nspf), C.byref(rel)) == 0
        assert t0.value > 0 and abs(nspf.value - 5000.0) < 1e-6 and rel.value == 1
        total = got
        deadline = t0.value + 60_000_000
        while _now_ns() < deadline:
            got = L.mosrx_source_fill(src, buf.ctypes.data, buf.nbytes, off.ctypes.data, ln.ctypes.data, 65536,
                                      2048, C.byref(end))
            assert got >= 0
            total += got
            # never ahead of the wire: at most the frames that have arrived by now
            assert total <= (_now_ns() - t0.value) / 5000.0 + 1
            time.sleep(0.002)
        el = (_now_ns() - t0.value) / 5000.0
        assert total >= el - 2 * 0.002 / 5e-6 - 2, (total, el)   # and not far behind (one sleep's worth)
        # the frames come out in order, as the inner source has them
        assert L.mosrx_source_paced_info(src, None, None, C.byref(rel)) == 0 and rel.value == total
    finally:
        L.mosrx_source_close(src)


def test_paced_source_rejects_bad_rates():
    tr = mosrx.Trace(mosrx.TRACE_S64, 16)
    inner = mosrx.mem_source(tr.frames, tr.off, tr.len)
    try:
        assert not mosrx.lib().mosrx_source_paced(inner, 0.0)
        assert not mosrx.lib().mosrx_source_paced(None, 1.0)
    finally:
        mosrx.lib().mosrx_source_close(inner)


def test_latency_probe_bins_residency():
    """The rx loop's probe on made-up arrivals (a scripted backend, tests/test_rx_loop.py):
    frame k arrived at t0 + k ms with t0 2 s before the first receive; one batch of
    1000 frames, so recv -> verdict available spans the 999 ms below its largest
    value evenly, and every percentile lands within a bin (6 %) of that ramp;
    consumed >= available."""
    from test_rx_loop import FakeBackend
    fb = FakeBackend([1000, 0], nif=1)
    p = mosrx.LatencyProbe()
    p.t0_ns = _now_ns() - 2_000_000_000
    p.ns_per_frame = 1e6
    st = mosrx.RxStats()
    o = mosrx.RxLoopOpts(0, 1, 0, 0, C.addressof(p))
    assert mosrx.lib().mosrx_rx_loop_ex(C.addressof(fb.m), None, 1, C.byref(o), None, None, C.byref(st)) == 0
    assert st.rx_packets == 1000 and p.seen == p.recorded == 1000 and p.batches == 1
    hi = p.avail_max_ns / 1e3                       # frame 0's residency, us (2 s + the receive's own time)
    assert 2.0e6 <= hi < 3.0e6
    pc = p.percentiles("avail", (0.1, 50, 99.9))
    for q, want in (("p0.1_us", hi - 999_000), ("p50_us", hi - 499_500), ("p99.9_us", hi)):
        assert abs(pc[q] - want) / want < 0.07, (q, pc, hi)
    assert sum(p.avail_hist) == sum(p.done_hist) == 1000
    dc = p.percentiles("done", (50,))
    assert dc["p50_us"] >= pc["p50_us"] * 0.93
    # skip: the first frames are not recorded
    fb = FakeBackend([600, 600, 0], nif=1)
    q = mosrx.LatencyProbe()
    q.t0_ns, q.ns_per_frame, q.skip = _now_ns() - 1_000_000, 100.0, 900
    o = mosrx.RxLoopOpts(0, 1, 0, 0, C.addressof(q))
    assert mosrx.lib().mosrx_rx_loop_ex(C.addressof(fb.m), None, 1, C.byref(o), None, None, C.byref(st)) == 0
    assert q.seen == 1200 and q.recorded == 300 and sum(q.avail_hist) == 300


def _emul():
    if not os.path.exists(EMUL):
        pytest.skip("oracle/_ref/libbackend_emul.so not built (make -C oracle)")
    return mosrx.module_lib(EMUL)


def _run_paced(L, rate, group_max_us, run_ms, batch=4096, group_bytes=16 << 20, kind=mosrx.TRACE_S64):
    tr = mosrx.Trace(kind, 8192)
    src = mosrx.paced_source(mosrx.mem_source(tr.frames, tr.off, tr.len, loops=0), rate)
    be = mosrx.GpuBackend([src], batch=batch, group=0, group_bytes=group_bytes, group_max_us=group_max_us,
                          compact=True, module_lib=L)
    probe = mosrx.LatencyProbe()
    probe.src = src
    try:
        st = be.run_loop(idle_rounds=0, idle_us=50, max_us=run_ms * 1000, probe=probe)
        ms = be.stats()
    finally:
        be.close()
    return st, ms, probe


def test_emulated_backend_latency_probe_counts_every_frame():
    """A light paced load through gpu_module_func (CPU stand-in): every frame the
    rx loop receives is recorded, and residencies are short."""
    L = _emul()
    st, ms, p = _run_paced(L, 100_000.0, 0, 150)
    assert st.rx_packets > 5000 and p.seen == st.rx_packets and p.recorded == st.rx_packets
    assert sum(p.avail_hist) == sum(p.done_hist) == p.recorded
    assert ms.rx_groups >= 10
    pc = p.percentiles("done", (50, 99))
    assert 0 < pc["p50_us"] < 50_000, pc


def test_latency_cap_bounds_group_size_under_a_paced_source():
    """Offered more frames than the stand-in classifies, the uncapped auto policy
    lets a group take every frame that has arrived (up to group_bytes), while
    cfg.group_max_us caps each group at what the measured host rate walks within
    the budget (never under 4096 frames)."""
    L = _emul()
    rate = 30_000_000.0                  # far above the stand-in's rate: a backlog builds
    _, free, _ = _run_paced(L, rate, 0, 400)
    _, capped, _ = _run_paced(L, rate, 2000, 400)
    assert capped.ns_per_frame_host > 0
    bound = max(4096, 2000e3 / capped.ns_per_frame_host)
    assert capped.group_cap_frames > 0
    assert capped.max_group_frames <= 2 * bound, (capped.max_group_frames, bound)
    assert free.max_group_frames > 2 * capped.max_group_frames, (free.max_group_frames, capped.max_group_frames)
