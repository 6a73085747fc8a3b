"""Batched BPF: mOS's sfbpf_filter per frame, on the GPU.

tests/golden/bpf.npz holds programs compiled by mOS's own sfbpf_compile plus
hand-assembled ones, mixed frames, and the return values of mOS's own
sfbpf_filter at both call-site lengths (tests/golden/make_golden_bpf.py).
CPU tests pin the oracle restatement to them; GPU tests compare the kernel
(through the C ABI) with both, bit-exact on every match bit.
"""
import os
import random
import struct

import numpy as np
import pytest

import mosrx
import oracle_py as O
from pktlib import pack_frames, tcp_frame

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load():
    z = np.load(os.path.join(GOLDEN, "bpf.npz"))
    progs = [z["insns"][o:o + n] for o, n in zip(z["prog_off"], z["prog_len"])]
    return z, progs


def runnable(z):
    """Programs the reference compiled, validated and ran (ip6 fails to compile there)."""
    return [j for j, v in enumerate(z["valid"]) if v == 1]


def program_sets(z, progs):
    """Sets of <= 32 programs, alternating the two call-site lengths, plus the
    expected match masks from the reference's return values."""
    js = runnable(z)
    sets = []
    for start in range(0, len(js), 32):
        chunk = js[start:start + 32]
        modes = [(start + b) % 2 for b in range(len(chunk))]
        exp = np.zeros(len(z["off"]), np.uint32)
        for b, (j, m) in enumerate(zip(chunk, modes)):
            r = z["ret_ip"][j] if m == mosrx.BPF_LEN_IP else z["ret_frame"][j]
            exp |= (r != 0).astype(np.uint32) << np.uint32(b)
        sets.append(([(progs[j], m) for j, m in zip(chunk, modes)], exp))
    return sets


I_ = lambda code, k=0, jt=0, jf=0: (code, jt, jf, k & 0xFFFFFFFF)  # noqa: E731


def prog(*ins):
    return np.array(list(ins), mosrx.BPF_INSN)


# ---------------------------------------------------------------- CPU: oracle pinned
def test_oracle_bpf_filter_matches_reference_returns():
    z, progs = load()
    buf, off, ln = z["frames"], z["off"], z["len"]
    for j in runnable(z):
        for mode, key in ((mosrx.BPF_LEN_FRAME, "ret_frame"), (mosrx.BPF_LEN_IP, "ret_ip")):
            np.testing.assert_array_equal(O.bpf_returns(progs[j], mode, buf, off, ln), z[key][j],
                                          err_msg=f"{z['names'][j]} {key}")


def test_oracle_bpf_filter_single_frame():
    z, progs = load()
    buf, off, ln = z["frames"], z["off"], z["len"]
    for i in range(0, len(off), 37):
        f = bytes(buf[off[i]:off[i] + ln[i]])
        for j in runnable(z)[::5]:
            assert O.bpf_filter(progs[j], f, int(ln[i])) == z["ret_frame"][j][i], (z["names"][j], i)
        if f[12:14] == b"\x08\x00" and len(f) >= 18:
            lip = 14 + struct.unpack("!H", f[16:18])[0]
            if lip <= len(f):
                assert O.bpf_filter(progs[0], f, lip) == z["ret_ip"][0][i]


def test_oracle_validate_matches_reference():
    z, progs = load()
    for j, v in enumerate(z["valid"]):
        if v >= 0:
            assert O.bpf_validate(progs[j]) == v, z["names"][j]


def test_oracle_batch_eval_masks():
    z, progs = load()
    for ps, exp in program_sets(z, progs):
        np.testing.assert_array_equal(O.bpf_eval(ps, z["frames"], z["off"], z["len"]), exp)


def test_reference_validate_accepts_constant_div0():
    # sf_bpf_filter.c:628 tests BPF_RVAL (code & 0x18) instead of BPF_SRC, so ALU|DIV|K
    # with k == 0 passes sfbpf_validate (and would SIGFPE in sfbpf_filter)
    p = prog(I_(0x34, 0), I_(0x16))
    assert O.bpf_validate(p) == 1
    assert mosrx.bpf_check(p) == -22


def test_fixture_coverage():
    z, progs = load()
    js = runnable(z)
    assert len(js) >= 60
    codes = set(np.concatenate([progs[j]["code"] for j in js]).tolist())
    # every opcode sfbpf_filter executes appears in some runnable program
    executable = {0x06, 0x16, 0x20, 0x28, 0x30, 0x80, 0x81, 0x40, 0x48, 0x50, 0xb1, 0x00, 0x01, 0x60, 0x61,
                  0x02, 0x03, 0x05, 0x25, 0x35, 0x15, 0x45, 0x2d, 0x3d, 0x1d, 0x4d, 0x0c, 0x1c, 0x2c, 0x3c,
                  0x5c, 0x4c, 0x6c, 0x7c, 0x04, 0x14, 0x24, 0x34, 0x54, 0x44, 0x64, 0x74, 0x84, 0x07, 0x87}
    assert executable - codes == set()
    # both outcomes occur for most programs
    both = sum(1 for j in js if 0 < (z["ret_frame"][j] != 0).sum() < len(z["off"]))
    assert both >= 40


# ---------------------------------------------------------------- CPU: admission check
@pytest.mark.parametrize("name,p,ok", [
    ("ret", prog(I_(0x06, 1)), True),
    ("empty", prog(), False),
    ("no_ret_end", prog(I_(0x00, 1)), False),
    ("jump_out", prog(I_(0x15, 1, 5, 0), I_(0x06, 1)), False),
    ("ja_wrap", prog(I_(0x05, 0xFFFFFFFF), I_(0x06, 1)), False),     # u_int-wrap backward jump
    ("mem16", prog(I_(0x60, 16), I_(0x16)), False),
    ("div_k0", prog(I_(0x34, 0), I_(0x16)), False),
    ("div_k1", prog(I_(0x34, 1), I_(0x16)), True),
    ("ld_h_len", prog(I_(0x88), I_(0x16)), False),                   # validate ok, abort() in filter
    ("neg_x", prog(I_(0x8c), I_(0x16)), False),
    ("ret_x", prog(I_(0x0e)), False),
    ("st_bits", prog(I_(0x22, 1), I_(0x16)), False),
    ("misc_other", prog(I_(0x27), I_(0x16)), False),
    ("alu_mod", prog(I_(0x94, 3), I_(0x16)), False),
    # absolute loads whose k wraps sfbpf_filter's int bounds check (reads before the frame)
    ("ld_w_abs_m1", prog(I_(0x20, 0xFFFFFFFF), I_(0x16)), False),
    ("ld_w_abs_m4", prog(I_(0x20, 0xFFFFFFFC), I_(0x16)), False),
    ("ld_w_abs_m5", prog(I_(0x20, 0xFFFFFFFB), I_(0x16)), True),     # fails the check: returns 0 there too
    ("ld_h_abs_m2", prog(I_(0x28, 0xFFFFFFFE), I_(0x16)), False),
    ("ld_h_abs_m3", prog(I_(0x28, 0xFFFFFFFD), I_(0x16)), True),
    ("ld_b_abs_m1", prog(I_(0x30, 0xFFFFFFFF), I_(0x16)), True),     # k >= buflen as u_int: returns 0
])
def test_bpf_check(name, p, ok):
    assert (mosrx.bpf_check(p) == 0) == ok, name
    if ok:
        assert O.bpf_validate(p) == 1


def test_bpf_check_admits_every_reference_runnable_program():
    z, progs = load()
    for j in runnable(z):
        assert mosrx.bpf_check(progs[j]) == 0, z["names"][j]
    for j, v in enumerate(z["valid"]):
        if v == 0:
            assert mosrx.bpf_check(progs[j]) != 0, z["names"][j]


def test_bpf_jit_compiles_every_golden_set():
    """Every admitted program becomes gfx950 code through hipRTC (compile only, no GPU)."""
    z, progs = load()
    sets = [ps for ps, _ in program_sets(z, progs)]
    sets.append([(p, m) for p, m in ((prog(I_(0x81), I_(0x40, 0xFFFFFFFC), I_(0x16)), 0),
                                     (prog(I_(0x81), I_(0x50, 0xFFFFFFFF), I_(0x44, 0x100), I_(0x16)), 1),
                                     (None, 0))])
    for ps in sets:
        rc, size, log = mosrx.bpf_jit_compile(ps)
        assert rc == 0 and size > 0, log
        src = mosrx.bpf_jit_source(ps)
        assert src.count("/* program ") == len(ps)


# random admitted programs: every opcode sfbpf_filter runs, forward jumps to
# anywhere later, loads in / past the LDS stage / past the frame, scratch slots
_LOADS = [0x20, 0x28, 0x30, 0x40, 0x48, 0x50, 0xb1, 0x80, 0x81]
_ALU = [0x04, 0x14, 0x24, 0x34, 0x44, 0x54, 0x64, 0x74, 0x0c, 0x1c, 0x2c, 0x3c, 0x4c, 0x5c, 0x6c, 0x7c, 0x84]
_JMP = [0x15, 0x25, 0x35, 0x45, 0x1d, 0x2d, 0x3d, 0x4d]
_MISC = [0x00, 0x01, 0x60, 0x61, 0x02, 0x03, 0x07, 0x87]


def random_program(rng, n):
    ins = []
    for i in range(n - 1):
        left = n - 2 - i                       # last valid jump offset
        r = rng.random()
        if r < 0.30:
            code = rng.choice(_LOADS)
            mode = code & 0xe0
            k = (rng.randint(0, 80) if rng.random() < 0.8 else rng.choice([rng.randint(80, 2000), 0xFFFFFFF0]))
            if mode == 0x40:
                k = rng.randint(0, 60)
            elif code == 0xb1:
                k = rng.choice([14, rng.randint(0, 100)])
            ins.append(I_(code, k))
        elif r < 0.55:
            code = rng.choice(_ALU)
            k = rng.getrandbits(32)
            if code in (0x64, 0x74):
                k = rng.randint(0, 40)
            if code == 0x34 and k == 0:
                k = 3
            ins.append(I_(code, k))
        elif r < 0.80:
            code = rng.choice(_JMP + [0x05])
            if code == 0x05:
                ins.append(I_(code, rng.randint(0, left)))
            else:
                k = rng.choice([0, 0x800, 6, rng.getrandbits(8), rng.getrandbits(32)])
                ins.append(I_(code, k, rng.randint(0, left), rng.randint(0, left)))
        elif r < 0.95:
            code = rng.choice(_MISC)
            k = rng.randint(0, 15) if code in (0x60, 0x61, 0x02, 0x03) else rng.getrandbits(32)
            ins.append(I_(code, k))
        else:
            ins.append(I_(rng.choice([0x06, 0x16]), rng.choice([0, 1, rng.getrandbits(32)])))
    ins.append(I_(rng.choice([0x06, 0x16]), rng.choice([1, 0xFFFF, rng.getrandbits(32)])))
    return prog(*ins)


def random_sets(seed, nsets=2):
    rng = random.Random(seed)
    return [[(random_program(rng, rng.randint(2, 48)), b % 2) for b in range(32)] for _ in range(nsets)]


def test_random_programs_admitted_and_compiled():
    for ps in random_sets(7):
        for p, _ in ps:
            assert mosrx.bpf_check(p) == 0, p
        rc, size, log = mosrx.bpf_jit_compile(ps)
        assert rc == 0 and size > 0, log


def test_fused_classify_bpf_compiles():
    """The classify kernel source embedded in libmosrx.so + each set's hook
    compile with hipRTC (no GPU needed)."""
    z, progs = load()
    for ps in [ps for ps, _ in program_sets(z, progs)] + random_sets(11, 1):
        rc, size, log = mosrx.bpf_jit_compile_fused(ps)
        assert rc == 0 and size > 0, log


# ---------------------------------------------------------------- GPU parity
@pytest.fixture(params=[mosrx.BPF_ENGINE_JIT, mosrx.BPF_ENGINE_INTERP], ids=["jit", "interp"])
def engine(gpu_ctx, request):
    """Both GPU engines: the hipRTC-compiled set and the interpreter kernel."""
    gpu_ctx.bpf_set_engine(request.param)
    yield request.param
    gpu_ctx.bpf_set_engine(mosrx.BPF_ENGINE_JIT)


def bpf_set(ctx, engine, ps):
    ctx.bpf_set(ps)
    if any(p is not None and len(p) for p, _ in ps):
        assert ctx.bpf_engine() == engine, ctx.bpf_jit_log()


@pytest.mark.gpu
def test_bpf_golden_sets(gpu_ctx, engine):
    z, progs = load()
    for ps, exp in program_sets(z, progs):
        bpf_set(gpu_ctx, engine, ps)
        got = gpu_ctx.bpf_host(z["frames"], z["off"], z["len"])
        np.testing.assert_array_equal(got, exp)
        db = gpu_ctx.upload(z["frames"], z["off"], z["len"])
        gpu_ctx.bpf_dev(db)
        np.testing.assert_array_equal(db.matches(), exp)
        db.free()


@pytest.mark.gpu
@pytest.mark.parametrize("phase,align", [(0, 1), (1, 1), (3, 4), (7, 16), (13, 2)])
def test_bpf_misaligned_layouts(gpu_ctx, engine, phase, align):
    z, progs = load()
    frames = [bytes(z["frames"][o:o + n]) for o, n in zip(z["off"], z["len"])]
    buf, off, ln = pack_frames(frames, align=align, phase=phase)
    ps = program_sets(z, progs)[0][0]
    bpf_set(gpu_ctx, engine, ps)
    np.testing.assert_array_equal(gpu_ctx.bpf_host(buf, off, ln), O.bpf_eval(ps, buf, off, ln))


@pytest.mark.gpu
def test_bpf_buffer_end_and_truncation(gpu_ctx, engine):
    # loads of the very last frame bytes, with frames_bytes ending mid-dword
    last = prog(I_(0x81), I_(0x40, 0xFFFFFFFC), I_(0x16))
    lastb = prog(I_(0x81), I_(0x50, 0xFFFFFFFF), I_(0x44, 0x100), I_(0x16))
    ps = [(last, 0), (lastb, 0), (last, 1), (lastb, 1)]
    bpf_set(gpu_ctx, engine, ps)
    for plen in range(0, 24):
        f = tcp_frame(payload=bytes(range(1, plen + 1)))
        buf, off, ln = pack_frames([tcp_frame(payload=b"x" * 50), f], phase=plen % 16)
        fb = int(off[-1]) + int(ln[-1])
        got = gpu_ctx.bpf_host(buf, off, ln, frames_bytes=fb)
        np.testing.assert_array_equal(got, O.bpf_eval(ps, buf[:fb], off, ln))


@pytest.mark.gpu
def test_bpf_empty_and_nofilter(gpu_ctx, engine):
    buf, off, ln = pack_frames([tcp_frame(payload=b"a"), tcp_frame(ethertype=0x86DD, pad_to=60)])
    bpf_set(gpu_ctx, engine, [(None, 0), (None, 1), (prog(I_(0x06, 0)), 0)])
    assert gpu_ctx.bpf_host(buf, off, ln).tolist() == [0b011, 0b001]   # LEN_IP only on IPv4
    gpu_ctx.bpf_set([])
    assert gpu_ctx.bpf_host(buf, off, ln).tolist() == [0, 0]
    with pytest.raises(mosrx.MosrxError):
        gpu_ctx.bpf_set([(prog(I_(0x34, 0), I_(0x16)), 0)])


@pytest.mark.gpu
@pytest.mark.parametrize("kind,n", [(mosrx.TRACE_IMIX, 262_144), (mosrx.TRACE_M1500, 65_536),
                                    (mosrx.TRACE_S64, 32_768)])
def test_bpf_full_size_traces(gpu_ctx, engine, kind, n):
    z, progs = load()
    t = mosrx.Trace(kind, n, nflows=3000)
    ps = program_sets(z, progs)[0][0]
    bpf_set(gpu_ctx, engine, ps)
    db = gpu_ctx.upload(t.frames, t.off, t.len, frames_bytes=t.frames_bytes, max_len=t.max_len)
    gpu_ctx.bpf_dev(db)
    got = db.matches()
    db.free()
    np.testing.assert_array_equal(got, O.bpf_eval(ps, t.frames[:t.frames_bytes], t.off, t.len))


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [1, 2, 3])
def test_bpf_random_programs(gpu_ctx, engine, seed):
    """Random admitted programs on both engines against the oracle (itself pinned to
    mOS's sfbpf_filter by the golden returns): every opcode, jump shape and bound."""
    z, _ = load()
    t = mosrx.Trace(mosrx.TRACE_IMIX, 4096, nflows=500, seed=seed)
    for buf, off, ln in ((z["frames"], z["off"], z["len"]), (t.frames[:t.frames_bytes], t.off, t.len)):
        for ps in random_sets(seed):
            bpf_set(gpu_ctx, engine, ps)
            np.testing.assert_array_equal(gpu_ctx.bpf_host(buf, off, ln), O.bpf_eval(ps, buf, off, ln))


# ---------------------------------------------------------------- fused classify + BPF
def fused_check(ctx, buf, off, ln, ps, frames_bytes=None, max_len=None):
    fb = len(buf) if frames_bytes is None else frames_bytes
    db = ctx.upload(buf, off, ln, frames_bytes=fb, max_len=max_len)
    ctx.classify_bpf_dev(db)
    rec, got = db.results(), db.matches()
    db.free()
    np.testing.assert_array_equal(got, O.bpf_eval(ps, buf[:fb], off, ln))
    ora = O.classify(buf[:fb], off, ln, O.params())
    assert np.array_equal(rec.view(np.uint8), ora.view(np.uint8)), "records differ from the oracle"


@pytest.mark.gpu
def test_classify_bpf_fused_golden(gpu_ctx, engine):
    """One pass: records bit-exact with the oracle, match masks with mOS's returns."""
    z, progs = load()
    gpu_ctx.set_params(mosrx.default_params())
    for ps, exp in program_sets(z, progs):
        bpf_set(gpu_ctx, engine, ps)
        assert gpu_ctx.bpf_fused() == (engine == mosrx.BPF_ENGINE_JIT), gpu_ctx.bpf_jit_log()
        db = gpu_ctx.upload(z["frames"], z["off"], z["len"])
        gpu_ctx.classify_bpf_dev(db)
        np.testing.assert_array_equal(db.matches(), exp)
        ora = O.classify(z["frames"], z["off"], z["len"], O.params())
        assert np.array_equal(db.results().view(np.uint8), ora.view(np.uint8))
        db.free()


@pytest.mark.gpu
@pytest.mark.parametrize("kind,n", [(mosrx.TRACE_IMIX, 100_000), (mosrx.TRACE_M1500, 20_000),
                                    (mosrx.TRACE_S64, 32_768)])
def test_classify_bpf_fused_traces(gpu_ctx, engine, kind, n):
    z, progs = load()
    gpu_ctx.set_params(mosrx.default_params())
    t = mosrx.Trace(kind, n, nflows=3000)
    for ps in (program_sets(z, progs)[0][0], random_sets(5, 1)[0]):
        bpf_set(gpu_ctx, engine, ps)
        fused_check(gpu_ctx, t.frames, t.off, t.len, ps, frames_bytes=t.frames_bytes, max_len=t.max_len)


@pytest.mark.gpu
@pytest.mark.parametrize("phase,align", [(1, 1), (3, 4), (13, 2)])
def test_classify_bpf_fused_layouts(gpu_ctx, phase, align):
    """Misaligned frames (window realignment inside the hook) and reversed
    descriptors (the unsorted-tile path of the stream kernel)."""
    z, progs = load()
    gpu_ctx.set_params(mosrx.default_params())
    frames = [bytes(z["frames"][o:o + n]) for o, n in zip(z["off"], z["len"])]
    buf, off, ln = pack_frames(frames, align=align, phase=phase)
    for ps in (program_sets(z, progs)[1][0], random_sets(phase, 1)[0]):
        bpf_set(gpu_ctx, mosrx.BPF_ENGINE_JIT, ps)
        fused_check(gpu_ctx, buf, off, ln, ps)
        fused_check(gpu_ctx, buf, off[::-1].copy(), ln[::-1].copy(), ps)


@pytest.mark.gpu
def test_classify_bpf_host_and_backend(gpu_ctx):
    """Host path (H2D, one pass, D2H) and the io_module backend with monitor
    filters: records and match masks per batch, through dev_ioctl."""
    z, progs = load()
    ps = program_sets(z, progs)[0][0]
    t = mosrx.Trace(mosrx.TRACE_IMIX, 20_000, nflows=800)
    ora = O.classify(t.frames, t.off, t.len, O.params())
    om = O.bpf_eval(ps, t.frames[:t.frames_bytes], t.off, t.len)
    gpu_ctx.set_params(mosrx.default_params())
    bpf_set(gpu_ctx, mosrx.BPF_ENGINE_JIT, ps)
    rec, m = gpu_ctx.classify_bpf_host(t.frames, t.off, t.len, frames_bytes=t.frames_bytes)
    np.testing.assert_array_equal(m, om)
    assert np.array_equal(rec.view(np.uint8), ora.view(np.uint8))
    src = mosrx.mem_source(t.frames, t.off, t.len, loops=1)
    be = mosrx.GpuBackend([src], batch=3000, pipeline=True, cpu=4, bpf=ps)
    try:
        seen = 0
        while (n := be.recv_pkts(0)) > 0:
            assert np.array_equal(be.results(0, n).view(np.uint8), ora[seen:seen + n].view(np.uint8))
            np.testing.assert_array_equal(be.matches(0, n), om[seen:seen + n])
            seen += n
        assert seen == t.n
    finally:
        be.close()
