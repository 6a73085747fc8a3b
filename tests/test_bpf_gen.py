"""The BPF code generator's output, run on the CPU.

csrc/bpf_jit.c turns a program set into gfx950 source.  Its program bodies are
plain C once the packet-load helpers are defined, so this test compiles the
generated text with gcc, one frame at a time (a wave with a single lane), and
checks it against mOS's own sfbpf_filter results (tests/golden/bpf.npz) and the
oracle.  Both code shapes are covered -- the if-converted programs
(MOSRX_BPF_PRED=1) and the branchy form (default) -- and both consumers: the
standalone kernel's programs and the fused classify kernel's hook (its
window registers, the X = 4 * ihl speculation, the LDS window copy for other
indexed loads).  A generator error shows here, apart from anything the GPU
compiler does with the text.  No GPU.
"""
import ctypes as C
import os
import subprocess

import numpy as np
import pytest

import mosrx
import oracle_py as O
from test_bpf import load, program_sets, random_sets

HARNESS = r"""
#include <stdbool.h>
#include <stdint.h>
#include <string.h>
typedef uint32_t u32; typedef uint64_t u64; typedef uint16_t u16; typedef uint8_t u8;
static const u8 *g_fr;
static u32 ld(u64 k) { u32 v; memcpy(&v, g_fr + k, 4); return v; }
static u32 be32(u32 v) { return __builtin_bswap32(v); }
static u32 be16(u32 v) { return ((v & 0xFFu) << 8) | ((v >> 8) & 0xFFu); }
#define W32(k) ld(k)
#define fr_le32(win, sh, rs, o, k, size) ld(k)
#define __any(x) (x)
void eval(const u8 *buf, u32 nbytes, const u32 *off, const u16 *len, u32 n, u32 *out)
{
  static const u8 zero[1 << 17];
  for (u32 p = 0; p < n; p++) {
    const bool live = true;
    const u32 o = off[p], l = len[p];
    const u32 cap = (o >= nbytes) ? 0u : (l < nbytes - o ? l : nbytes - o);
    const int rs = 0, sh = 0; const u32 *win = 0;
    u32 lip = 0, match = 0;
    (void)rs; (void)sh; (void)win;
    g_fr = o >= nbytes ? zero : buf + o;
    if (cap >= 18u && (ld(12) & 0xFFFFu) == 0x0008u) {
      lip = 14u + be16(ld(16));
      if (lip > cap) lip = 0;
    }
    BODY
    out[p] = match;
  }
}
"""


HOOK_HARNESS = r"""
#include <stdbool.h>
#include <string.h>
static unsigned buf_ld(const unsigned char *rs, unsigned a) { unsigned v; memcpy(&v, rs + a, 4); return v; }
#define __amdgpu_buffer_rsrc_t const unsigned char *
#define __builtin_amdgcn_raw_buffer_load_b32(rs, a, x, y) buf_ld(rs, a)
#define __builtin_amdgcn_alignbyte(h, l, s) \
  ((unsigned)((((unsigned long long)(h) << 32) | (unsigned)(l)) >> (8u * ((s) & 3u))))
#define __device__
#define __shared__ static
#define __any(x) (x)
static struct { unsigned x; } threadIdx;
static unsigned be16hi(unsigned w) { return ((w >> 8) & 0xFF00u) | (w >> 24); }
HOOK
extern "C" void eval(const unsigned char *buf, unsigned nbytes, const unsigned *off, const unsigned short *len,
                     unsigned n, unsigned *out)
{
  for (unsigned p = 0; p < n; p++) {
    const unsigned o = off[p] < nbytes ? off[p] : nbytes, l = len[p];
    const unsigned cap = (off[p] >= nbytes) ? 0u : (l < nbytes - o ? l : nbytes - o);
    unsigned w[23];
    threadIdx.x = p & 255u;
    for (unsigned j = 0; j < 23; j++) w[j] = buf_ld(buf, o + 2u + 4u * j);
    out[p] = mosrx_bpf_hook<256u>(w, o, cap, true, buf);
  }
}
"""


def build_hook(tmp_path, ps, pred):
    os.environ["MOSRX_BPF_PRED"] = str(pred)
    try:
        src = mosrx.bpf_jit_hook_source(ps)
    finally:
        del os.environ["MOSRX_BPF_PRED"]
    return compile_c(tmp_path, f"hook{pred}", HOOK_HARNESS.replace("HOOK", src), cxx=True)   # (a template)


def compile_c(tmp_path, name, text, cxx=False):
    c = tmp_path / (f"{name}.cc" if cxx else f"{name}.c")
    c.write_text(text)
    so = tmp_path / f"{name}.so"
    r = subprocess.run(["g++" if cxx else "gcc", "-O1", "-shared", "-fPIC", "-w", "-o", str(so), str(c)],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-2000:]
    return C.CDLL(str(so))


def build(tmp_path, ps, pred):
    os.environ["MOSRX_BPF_PRED"] = str(pred)
    try:
        src = mosrx.bpf_jit_source(ps)
    finally:
        del os.environ["MOSRX_BPF_PRED"]
    body = src[src.index("  u32 match = 0;\n") + len("  u32 match = 0;\n"):src.index("  if (live) match_out[p]")]
    return compile_c(tmp_path, f"gen{pred}", HARNESS.replace("BODY", body))


def run(lib, buf, off, ln):
    # the if-converted programs load every constant offset below 65536 (zero padding, as the GPU's
    # buffer descriptor returns zeros past the end)
    padded = np.zeros(len(buf) + 70000, np.uint8)
    padded[:len(buf)] = buf
    off = np.ascontiguousarray(off, np.uint32)
    ln = np.ascontiguousarray(ln, np.uint16)
    out = np.zeros(len(off), np.uint32)
    lib.eval(padded.ctypes.data_as(C.c_void_p), C.c_uint32(len(buf)), off.ctypes.data_as(C.c_void_p),
             ln.ctypes.data_as(C.c_void_p), C.c_uint32(len(off)), out.ctypes.data_as(C.c_void_p))
    return out


@pytest.mark.parametrize("fused", [0, 1])
@pytest.mark.parametrize("pred", [1, 0])
def test_generated_golden_sets(tmp_path, pred, fused):
    z, progs = load()
    for i, (ps, exp) in enumerate(program_sets(z, progs)):
        d = tmp_path / str(i)
        d.mkdir()
        lib = (build_hook if fused else build)(d, ps, pred)
        got = run(lib, z["frames"], z["off"], z["len"])
        bad = np.nonzero(got != exp)[0]
        assert not len(bad), (i, bad[:5], hex(int(got[bad[0]] ^ exp[bad[0]])))


@pytest.mark.parametrize("fused", [0, 1])
@pytest.mark.parametrize("pred", [1, 0])
@pytest.mark.parametrize("seed", [3, 11, 19, 27])
def test_generated_random_programs(tmp_path, pred, seed, fused):
    z, _ = load()
    for i, ps in enumerate(random_sets(seed)):
        d = tmp_path / str(i)
        d.mkdir()
        lib = (build_hook if fused else build)(d, ps, pred)
        got = run(lib, z["frames"], z["off"], z["len"])
        exp = O.bpf_eval(ps, z["frames"], z["off"], z["len"])
        bad = np.nonzero(got != exp)[0]
        assert not len(bad), (i, bad[:5], hex(int(got[bad[0]] ^ exp[bad[0]])))


def test_hook_window_and_lds_copy():
    """The fused hook's window (MOSRX_BPF_WEND) and LDS copy follow the set
    (bpf_jit.c hook_wend / x_provenance): header filters whose indexed loads
    take X = 4 * ihl read registers of the stream tile's 62-byte window and
    copy nothing to LDS; a payload-offset load (X computed from the TCP data
    offset, mOS's HTTP-GET filter) sizes the window for IPv4 + a timestamped
    TCP header (78) and reads the hook's LDS copy of it."""
    import bench
    progs = bench.bpf_bench_programs()
    names = [e for e, _ in bench.BPF_BENCH]
    get = names.index("tcp[((tcp[12:1] & 0xf0) >> 2):4] = 0x47455420")
    header = [p for j, p in enumerate(progs) if j != get]
    src = mosrx.bpf_jit_hook_source(header)
    assert "#define MOSRX_BPF_WEND 62" in src and "s_bw" not in src and "hk_ind_le32<HL>(bw" not in src
    assert "X == 20u ? RW32(" in src                       # the ihl = 5 speculation
    src = mosrx.bpf_jit_hook_source([progs[get]])
    assert "#define MOSRX_BPF_WEND 78" in src and "__shared__ u32 s_bw" in src and "hk_ind_le32<HL>(bw" in src
    # the same filter's X = 4 * ihl load (tcp[12:1]) still takes the register speculation
    assert "X == 20u ? RW32(46u)" in src


def test_standalone_stage_follows_the_set():
    """The standalone kernel stages what the set reads (stage_pieces): header
    filters keep their bytes in registers only (no LDS stage; X = 4 * ihl loads
    speculate ihl = 5), a payload-offset load adds the LDS stage of the frame's
    first 80 bytes."""
    import bench
    progs = bench.bpf_bench_programs()
    names = [e for e, _ in bench.BPF_BENCH]
    get = names.index("tcp[((tcp[12:1] & 0xf0) >> 2):4] = 0x47455420")
    header = [p for j, p in enumerate(progs) if j != get]
    src = mosrx.bpf_jit_source(header)
    assert "#define STAGE_LDS 0" in src and "#define STAGE_V 4u" in src   # tcp[13] at X + 27: bytes [0, 61)
    assert "X == 20u ? W32(" in src
    src = mosrx.bpf_jit_source(progs)
    assert "#define STAGE_LDS 1" in src and "#define STAGE_V 5u" in src


def test_compiled_sets_shared_in_process():
    """A set compiled once in the process is not compiled again (bpf_jit.c
    rtc_cache_*): every mTCP thread's context installs the same filters, and
    after the first only loads the code object."""
    import time
    import bench
    ps = bench.bpf_bench_programs()[2:5]
    rc, size, log = mosrx.bpf_jit_compile_fused(ps)
    assert rc == 0 and size > 0, log
    t0 = time.perf_counter()
    rc2, size2, _ = mosrx.bpf_jit_compile_fused(ps)
    assert (rc2, size2) == (0, size) and time.perf_counter() - t0 < 0.02
