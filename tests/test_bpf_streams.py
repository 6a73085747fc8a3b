"""BPF sets replaced while launches on a caller's stream still read the old ones.

mosrx_bpf_dev / mosrx_classify_bpf_dev take the caller's stream.  The
interpreter's staged instructions rotate over MOSRX_BPF_POOL (8) device
buffers and the compiled sets over a cache of MOSRX_BPF_JIT_CACHE (16)
modules; a buffer is rewritten, or a module unloaded, only after every launch
that may read it has finished -- on the context's streams and on any caller's
stream used since (mosrx__drain: a device synchronisation).  Here more than 8
and more than 16 distinct sets are installed one after another while a
non-blocking stream the test created holds a backlog of launches of the
previous sets; every launch's masks must be those of the set installed when it
was enqueued (the oracle, pinned to mOS's sfbpf_filter by tests/test_bpf.py).
Reference: EVAL_BPFFILTER / sfbpf_filter, include/bpf/sfbpf.h:84,
bpf/sf_bpf_filter.c:214-536."""
import ctypes as C

import numpy as np
import pytest

import mosrx
import oracle_py as O
from test_bpf import load, runnable

pytestmark = pytest.mark.gpu

NSETS = 18          # past the interpreter pool (8) and the compiled-set cache (16)
LAUNCHES = 24       # per set, queued on the caller's stream behind each other


def distinct_sets(n):
    """n distinct sets of 6 mOS-compiled programs (rotations over the runnable ones)."""
    z, progs = load()
    js = runnable(z)
    sets = []
    for i in range(n):
        pick = [js[(7 * i + 3 * k) % len(js)] for k in range(6)]
        sets.append([(progs[j], (i + k) % 2) for k, j in enumerate(pick)])
    return sets


@pytest.fixture
def caller_stream():
    hip = C.CDLL("libamdhip64.so")
    s = C.c_void_p()
    assert hip.hipStreamCreateWithFlags(C.byref(s), 1) == 0        # hipStreamNonBlocking
    yield hip, s.value
    hip.hipStreamSynchronize(C.c_void_p(s.value))
    hip.hipStreamDestroy(C.c_void_p(s.value))


@pytest.mark.parametrize("engine,fused", [(0, False), (1, False), (1, True)])
def test_sets_replaced_under_a_caller_stream_backlog(caller_stream, engine, fused):
    hip, stream = caller_stream
    t = mosrx.Trace(mosrx.TRACE_IMIX, 65_536, nflows=4000, seed=21)
    sets = distinct_sets(NSETS)
    want = [O.bpf_eval(st, t.frames[:t.frames_bytes], t.off, t.len) for st in sets]
    with mosrx.Context(0) as ctx:
        ctx.bpf_set_engine(engine)
        dbs = [ctx.upload(t.frames, t.off, t.len, frames_bytes=t.frames_bytes, max_len=t.max_len)
               for _ in range(NSETS)]
        try:
            for i, st in enumerate(sets):
                # installed while the previous sets' launches are still queued on the caller's
                # stream (the interpreter's set is staged at once; a compiled one after its compile)
                ctx.bpf_set(st) if engine else ctx.bpf_set_async(st)
                for _ in range(LAUNCHES):
                    if fused:
                        ctx.classify_bpf_dev(dbs[i], sync=False, stream=stream)
                    else:
                        ctx.bpf_dev(dbs[i], sync=False, stream=stream)
            assert hip.hipStreamSynchronize(C.c_void_p(stream)) == 0
            for i, d in enumerate(dbs):
                got = d.matches()
                bad = np.nonzero(got != want[i])[0]
                assert len(bad) == 0, f"set {i}: {len(bad)} masks differ (first frame {bad[0]})"
        finally:
            for d in dbs:
                d.free()
