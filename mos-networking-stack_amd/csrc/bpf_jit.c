/*
 * bpf_jit.c — compiled BPF program sets.
 *
 * mosrx_bpf_set hands the admitted program set here: every program becomes
 * straight-line gfx950 code — one labelled block per instruction, jumps as
 * gotos (forward only, so the control flow is a DAG the compiler structurizes
 * for divergent lanes), A / X / the used scratch slots as registers, packet
 * loads at constant offsets resolved at generation time to registers (the
 * staged bytes realigned once per frame), to the LDS stage (sized to what the
 * set reads; loads at X + k) or to memory — and the whole set is one kernel,
 * compiled with hipRTC
 * for gfx950 and loaded as a module.  Same semantics as the interpreter in
 * mosrx_bpf.hip (itself pinned to mOS's sfbpf_filter, bpf/sf_bpf_filter.c:
 * 214-536): the staging, bounds checks and return conventions are generated
 * from the same rules, and tests/test_bpf.py runs both engines against the
 * reference's own results.
 *
 * Compiled sets are cached per context by content hash, so re-installing a set
 * costs a lookup.  When hipRTC is unavailable or fails the set runs on the
 * interpreter (mosrx_bpf_engine() reports which engine is installed).
 *
 * The same generator writes the fused form (mosrx__bpf_jit_hook_source): the
 * set as a device function the classify tiles' header wave calls on its
 * realigned window.  There, constant-offset loads read the window's registers;
 * an indexed load whose X can only be 4 * ihl (x_provenance) speculates ihl = 5
 * and reads registers too; any other indexed load reads a copy of the window
 * the hook writes to LDS.  MOSRX_BPF_PRED=1 emits the programs if-converted
 * (gen_pred) instead of branchy; tests/test_bpf_gen.py runs both forms of both
 * outputs on the CPU against mOS's results.
 */
#include <errno.h>
#include <pthread.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "mosrx_ctx.h"
#include <hip/hiprtc.h>

/* hip/hip_ext.h is C++ only: its C-linkage launcher with dispatch-stamped events */
hipError_t hipExtModuleLaunchKernel(hipFunction_t f, uint32_t globalWorkSizeX, uint32_t globalWorkSizeY,
                                    uint32_t globalWorkSizeZ, uint32_t localWorkSizeX, uint32_t localWorkSizeY,
                                    uint32_t localWorkSizeZ, size_t sharedMemBytes, hipStream_t hStream,
                                    void **kernelParams, void **extra, hipEvent_t startEvent, hipEvent_t stopEvent,
                                    uint32_t flags);

enum {
	LD = 0, LDX = 1, ST = 2, STX = 3, ALU = 4, JMP = 5, RET = 6, MISC = 7,
	W = 0, H = 8, B = 0x10, IMM = 0, ABS = 0x20, IND = 0x40, MEM = 0x60, LEN = 0x80, MSH = 0xa0,
	ADD = 0, SUB = 0x10, MUL = 0x20, DIV = 0x30, OR = 0x40, AND = 0x50, LSH = 0x60, RSH = 0x70, NEG = 0x80,
	JA = 0, JEQ = 0x10, JGT = 0x20, JGE = 0x30, JSET = 0x40, K = 0, X = 8, A = 0x10, TAX = 0, TXA = 0x80,
};

/* ---- growable text buffer ---- */
struct sbuf {
	char *p;
	size_t n, cap;
	int err;
};

static void sb_printf(struct sbuf *s, const char *fmt, ...)
{
	va_list ap;
	int k;
	if (s->err)
		return;
	for (;;) {
		va_start(ap, fmt);
		k = vsnprintf(s->p ? s->p + s->n : NULL, s->p ? s->cap - s->n : 0, fmt, ap);
		va_end(ap);
		if (k < 0) {
			s->err = 1;
			return;
		}
		if (s->p && s->n + (size_t)k < s->cap) {
			s->n += (size_t)k;
			return;
		}
		{
			size_t nc = (s->cap ? s->cap * 2 : 1 << 16) + (size_t)k;
			char *np = realloc(s->p, nc);
			if (!np) {
				s->err = 1;
				return;
			}
			s->p = np;
			s->cap = nc;
		}
	}
}

/* Device preamble: staging and packet loads exactly as mosrx_bpf.hip. */
static const char k_preamble[] =
	"typedef unsigned int u32;\n"
	"typedef unsigned long long u64;\n"
	"typedef unsigned short u16;\n"
	"typedef unsigned char u8;\n"
	"typedef u32 u32x4 __attribute__((ext_vector_type(4)));\n"
	"static __device__ __attribute__((always_inline)) inline u32 ld_le32(__amdgpu_buffer_rsrc_t rs, u32 a) {\n"
	"  const u32 a4 = a & ~3u;\n"
	"  const u32 lo = __builtin_amdgcn_raw_buffer_load_b32(rs, a4, 0, 0);\n"
	"  const u32 hi = __builtin_amdgcn_raw_buffer_load_b32(rs, a4 + 4u, 0, 0);\n"
	"  return __builtin_amdgcn_alignbyte(hi, lo, a & 3u);\n"
	"}\n"
	"/* frame bytes [k, k+4): the LDS stage (sets with loads at an X not 4 * ihl), else memory */\n"
	"static __device__ __attribute__((always_inline)) inline u32 fr_le32(const u32 *win, u32 sh, __amdgpu_buffer_rsrc_t rs, u32 o,\n"
	"                                              u32 k, u32 size) {\n"
	"#if STAGE_LDS\n"
	"  if (k + size <= STAGE_B) {\n"
	"    const u32 a = sh + k;\n"
	"    return __builtin_amdgcn_alignbyte(win[(a >> 2) + 1u], win[a >> 2], a & 3u);\n"
	"  }\n"
	"#endif\n"
	"  return ld_le32(rs, o + k);\n"
	"}\n"
	"#define STAGE_W (4u * STAGE_V - 1u)\n"
	"/* little-endian dword of frame bytes [k, k+4), k constant, from the registers */\n"
	"#define W32(k) ((k) % 4u == 0u ? w[(k) / 4u] : __builtin_amdgcn_alignbyte(w[(k) / 4u + 1u], w[(k) / 4u], (k) % 4u))\n"
	"static __device__ __attribute__((always_inline)) inline u32 be32(u32 v) { return __builtin_bswap32(v); }\n"
	"static __device__ __attribute__((always_inline)) inline u32 be16(u32 v) { return ((v & 0xFFu) << 8) | ((v >> 8) & 0xFFu); }\n"
	"extern \"C\" __global__ __launch_bounds__(256) void mosrx_bpf_jit(const u8 *frames, const u32 *offs,\n"
	"    const u16 *lens, u32 *match_out, u32 nbytes, u32 n) {\n"
	"#if STAGE_LDS\n"
	"  __shared__ u32 s_win[STAGE_LD * 256];\n"
	"#endif\n"
	"  const u32 t = threadIdx.x;\n"
	"  const u32 p = blockIdx.x * 256u + t;\n"
	"  const bool live = p < n;\n"
	"  const __amdgpu_buffer_rsrc_t rs =\n"
	"      __builtin_amdgcn_make_buffer_rsrc((void *)frames, (short)0, (int)((nbytes + 15u) & ~15u), 0x00020000);\n"
	"  u32 o = 0, cap = 0, lip = 0;\n"
	"  if (live) {\n"
	"    o = offs[p];\n"
	"    const u32 l = lens[p];\n"
	"    cap = (o >= nbytes) ? 0u : (l < nbytes - o ? l : nbytes - o);\n"
	"  }\n"
	"#if STAGE_LDS\n"
	"  u32 *win = s_win + STAGE_LD * t;\n"
	"#else\n"
	"  const u32 *win = nullptr;\n"
	"#endif\n"
	"  const u32 sh = o & 3u;\n"
	"  u32 w[STAGE_W];   /* frame bytes [4i, 4i + 4) in w[i]: constant-offset loads read registers */\n"
	"  {\n"
	"    const u32 base = live ? (o & ~3u) : nbytes + 16u;\n"
	"    u32x4 v[STAGE_V];\n"
	"#pragma unroll\n"
	"    for (u32 m = 0; m < STAGE_V; m++) v[m] = __builtin_amdgcn_raw_buffer_load_b128(rs, base + 16u * m, 0, 0);\n"
	"    u32 r[4 * STAGE_V];\n"
	"#pragma unroll\n"
	"    for (u32 m = 0; m < STAGE_V; m++) {\n"
	"      r[4 * m + 0] = v[m].x; r[4 * m + 1] = v[m].y; r[4 * m + 2] = v[m].z; r[4 * m + 3] = v[m].w;\n"
	"#if STAGE_LDS\n"
	"      win[4 * m + 0] = v[m].x; win[4 * m + 1] = v[m].y; win[4 * m + 2] = v[m].z; win[4 * m + 3] = v[m].w;\n"
	"#endif\n"
	"    }\n"
	"#pragma unroll\n"
	"    for (u32 i = 0; i < STAGE_W; i++) w[i] = __builtin_amdgcn_alignbyte(r[i + 1], r[i], sh);\n"
	"  }\n"
	"  if (cap >= 18u && (w[3] & 0xFFFFu) == 0x0008u) {\n"
	"    lip = 14u + be16(w[4]);\n"
	"    if (lip > cap) lip = 0;\n"
	"  }\n"
	"  u32 match = 0;\n";

/* bounds test "(u64)off + size > L" for a constant offset: 1 = always out of range.
 * In a program's fast copy (`lp` "F") L covers every constant offset: only the
 * offsets past any length (2^32) remain. */
static void gen_abs_check(struct sbuf *s, unsigned j, uint32_t k, uint32_t size, const char *lp)
{
	if ((uint64_t)k + size > 0xFFFFFFFFull)
		sb_printf(s, "goto P%u_R0; ", j);
	else if (!*lp)
		sb_printf(s, "if (%uu > L) goto P%u_R0; ", (unsigned)(k + size), j);
}

/* How the generated program code reads frame bytes. */
struct genopt {
	int fused;          /* 0: standalone kernel (staged bytes); 1: classify header wave (its window) */
	uint32_t stage_w;   /* standalone: realigned staged dwords in w[] */
	uint32_t wend;      /* fused: the header window the tiles load for the set ends at frame byte wend */
	int pred;           /* 1: if-converted programs (gen_pred, MOSRX_BPF_PRED=1); 0: branchy */
	int lds;            /* fused: the hook stages the window in LDS for loads at X + k with X not 4 * ihl */
};

/* Per-instruction flags of a program: a jump target; X holds 4 * ihl (only
 * `ldxb 4*([k]&0xf)` defines the X that reaches here). */
enum { TG_TARGET = 1, TG_XMSH = 2 };

/* Which definitions of X reach each instruction (forward over the DAG):
 * sets TG_XMSH where every one is an MSH load.  Returns 1 if some indexed
 * load sees any other X. */
static int x_provenance(const mosrx_bpf_insn *f, uint32_t len, uint8_t *tg)
{
	enum { XI = 1, XM = 2, XO = 4 };   /* X still 0, from MSH, from anything else */
	uint8_t *in = calloc((size_t)len + 1, 1);
	uint32_t i;
	int other = 0;
	if (!in)
		return 1;
	in[0] = XI;
	for (i = 0; i < len; i++) {
		const uint16_t c = f[i].code;
		uint8_t out = in[i];
		if (c == (LDX | MSH | B))
			out = XM;
		else if ((c & 7) == LDX || c == (MISC | TAX))
			out = XO;
		if ((c & 7) == LD && (c & 0xe0) == IND) {
			if (in[i] == XM)
				tg[i] |= TG_XMSH;
			else
				other = 1;
		}
		if (c == (JMP | JA)) {
			in[i + 1 + f[i].k] |= out;
		} else if ((c & 7) == JMP) {
			in[i + 1 + f[i].jt] |= out;
			in[i + 1 + f[i].jf] |= out;
		} else if ((c & 7) != RET && i + 1 < len) {
			in[i + 1] |= out;
		}
	}
	free(in);
	return other;
}

/* The program shape: branchy by default (the 64 B fused ring measured 123.5 us
 * branchy, 125.3 if-converted; IMIX 139.1 / 138.6: profiles/r04/fused_cost/);
 * MOSRX_BPF_PRED=1 selects the if-converted form. */
static int pred_mode(void)
{
	const char *e = getenv("MOSRX_BPF_PRED");
	return e && e[0] == '1';
}

/* Constant-offset load expression.  Standalone: registers when frame bytes
 * [k, k + 8) are in w[], else the LDS stage / memory (fr_le32).  Fused: the
 * header window's realigned registers (frame bytes [2, 94)), else memory. */
static void gen_ld(struct sbuf *s, uint32_t k, uint32_t size, const struct genopt *g)
{
	if (g->fused) {
		if (k >= 2 && (uint64_t)k + 8 <= g->wend)
			sb_printf(s, "RW32(%uu)", k);
		else
			sb_printf(s, "hk_ld_le32(rs, o + %uu)", k);
	} else if ((uint64_t)k + 8 <= 4ull * g->stage_w) {
		sb_printf(s, "W32(%uu)", k);
	} else {
		sb_printf(s, "fr_le32(win, sh, rs, o, %uu, %uu)", k, size);
	}
}

/* Load at the run-time offset kk = X + k (size bytes).  Standalone: the LDS
 * stage / memory.  Fused: where X is 4 * ihl (`ldxb 4*([14]&0xf)`, every
 * header filter mOS compiles) ihl is 5 in nearly every frame, so kk = k + 20
 * is speculated: a constant offset, read from the window's registers, any
 * other X reads memory.  Any other X (payload offsets such as
 * `tcp[((tcp[12:1] & 0xf0) >> 2):4]`) reads the hook's LDS copy of the window
 * (hk_ind_le32), memory past it: a dependent memory read in every wave cost
 * the 64 B ring 19 us per such program. */
static void gen_ind(struct sbuf *s, uint32_t k, uint32_t size, int msh, const struct genopt *g)
{
	if (!g->fused) {   /* the same speculation from the realigned staged registers */
		if (msh && (uint64_t)k + 20 + 8 <= 4ull * g->stage_w)
			sb_printf(s, "(X == 20u ? W32(%uu) : fr_le32(win, sh, rs, o, kk, %uu))", k + 20, size);
		else
			sb_printf(s, "fr_le32(win, sh, rs, o, kk, %uu)", size);
		return;
	}
	if (msh && (uint64_t)k + 20 + 8 <= g->wend) {
		sb_printf(s, "(X == 20u ? ");
		gen_ld(s, k + 20, size, g);
		sb_printf(s, " : hk_ld_le32(rs, o + kk))");
	} else if (!msh && g->lds) {
		sb_printf(s, "hk_ind_le32<HL>(bw, kk, rs, o)");
	} else {
		sb_printf(s, "hk_ld_le32(rs, o + kk)");
	}
}

/* One copy of program j's instructions, labels P<j>_<lp><i>: lp "" checks
 * every constant-offset load against L as sfbpf_filter does; lp "F" is the
 * copy for lanes whose L covers all of them (frames long enough for every
 * header field the program reads -- nearly all), with those checks left out:
 * half the branches of a typical filter. */
static int gen_body(struct sbuf *s, unsigned j, const mosrx_bpf_insn *f, uint32_t len, const uint8_t *tgt,
                    const char *lp, const struct genopt *g)
{
	uint32_t i;
	for (i = 0; i < len; i++) {
		const uint16_t c = f[i].code;
		const uint32_t k = f[i].k;
		const unsigned jt = i + 1 + f[i].jt, jf = i + 1 + f[i].jf;
		if (tgt[i] & TG_TARGET)
			sb_printf(s, "  P%u_%s%u: ", j, lp, (unsigned)i);
		else
			sb_printf(s, "    ");
		switch (c) {
		case RET | K: sb_printf(s, "ret = %uu; goto P%u_E;", k, j); break;
		case RET | A: sb_printf(s, "ret = A; goto P%u_E;", j); break;
		case LD | W | ABS:
			gen_abs_check(s, j, k, 4, lp); sb_printf(s, "A = be32("); gen_ld(s, k, 4, g); sb_printf(s, ");");
			break;
		case LD | H | ABS:
			gen_abs_check(s, j, k, 2, lp); sb_printf(s, "A = be16("); gen_ld(s, k, 2, g); sb_printf(s, ");");
			break;
		case LD | B | ABS:
			gen_abs_check(s, j, k, 1, lp); sb_printf(s, "A = "); gen_ld(s, k, 1, g); sb_printf(s, " & 0xFFu;");
			break;
		case LD | W | LEN: sb_printf(s, "A = L;"); break;
		case LDX | W | LEN: sb_printf(s, "X = L;"); break;
		case LD | W | IND:
			sb_printf(s, "{ const u32 kk = X + %uu; if ((u64)kk + 4u > L) goto P%u_R0; A = be32(", k, j);
			gen_ind(s, k, 4, tgt[i] & TG_XMSH, g);
			sb_printf(s, "); }");
			break;
		case LD | H | IND:
			sb_printf(s, "{ const u32 kk = X + %uu; if ((u64)kk + 2u > L) goto P%u_R0; A = be16(", k, j);
			gen_ind(s, k, 2, tgt[i] & TG_XMSH, g);
			sb_printf(s, "); }");
			break;
		case LD | B | IND:
			sb_printf(s, "{ const u32 kk = X + %uu; if (kk >= L) goto P%u_R0; A = ", k, j);
			gen_ind(s, k, 1, tgt[i] & TG_XMSH, g);
			sb_printf(s, " & 0xFFu; }");
			break;
		case LDX | MSH | B:
			gen_abs_check(s, j, k, 1, lp);
			sb_printf(s, "X = ("); gen_ld(s, k, 1, g); sb_printf(s, " & 0xFu) << 2;");
			break;
		case LD | IMM: sb_printf(s, "A = %uu;", k); break;
		case LDX | IMM: sb_printf(s, "X = %uu;", k); break;
		case LD | MEM: sb_printf(s, "A = M%u;", k & 15); break;
		case LDX | MEM: sb_printf(s, "X = M%u;", k & 15); break;
		case ST: sb_printf(s, "M%u = A;", k & 15); break;
		case STX: sb_printf(s, "M%u = X;", k & 15); break;
		case JMP | JA: sb_printf(s, "goto P%u_%s%u;", j, lp, (unsigned)(i + 1 + k)); break;
		case JMP | JGT | K: sb_printf(s, "if (A > %uu) goto P%u_%s%u; goto P%u_%s%u;", k, j, lp, jt, j, lp, jf); break;
		case JMP | JGE | K: sb_printf(s, "if (A >= %uu) goto P%u_%s%u; goto P%u_%s%u;", k, j, lp, jt, j, lp, jf); break;
		case JMP | JEQ | K: sb_printf(s, "if (A == %uu) goto P%u_%s%u; goto P%u_%s%u;", k, j, lp, jt, j, lp, jf); break;
		case JMP | JSET | K: sb_printf(s, "if (A & %uu) goto P%u_%s%u; goto P%u_%s%u;", k, j, lp, jt, j, lp, jf); break;
		case JMP | JGT | X: sb_printf(s, "if (A > X) goto P%u_%s%u; goto P%u_%s%u;", j, lp, jt, j, lp, jf); break;
		case JMP | JGE | X: sb_printf(s, "if (A >= X) goto P%u_%s%u; goto P%u_%s%u;", j, lp, jt, j, lp, jf); break;
		case JMP | JEQ | X: sb_printf(s, "if (A == X) goto P%u_%s%u; goto P%u_%s%u;", j, lp, jt, j, lp, jf); break;
		case JMP | JSET | X: sb_printf(s, "if (A & X) goto P%u_%s%u; goto P%u_%s%u;", j, lp, jt, j, lp, jf); break;
		case ALU | ADD | X: sb_printf(s, "A += X;"); break;
		case ALU | SUB | X: sb_printf(s, "A -= X;"); break;
		case ALU | MUL | X: sb_printf(s, "A *= X;"); break;
		case ALU | DIV | X: sb_printf(s, "if (X == 0u) goto P%u_R0; A /= X;", j); break;
		case ALU | AND | X: sb_printf(s, "A &= X;"); break;
		case ALU | OR | X: sb_printf(s, "A |= X;"); break;
		case ALU | LSH | X: sb_printf(s, "A <<= (X & 31u);"); break;
		case ALU | RSH | X: sb_printf(s, "A >>= (X & 31u);"); break;
		case ALU | ADD | K: sb_printf(s, "A += %uu;", k); break;
		case ALU | SUB | K: sb_printf(s, "A -= %uu;", k); break;
		case ALU | MUL | K: sb_printf(s, "A *= %uu;", k); break;
		case ALU | DIV | K: sb_printf(s, "A /= %uu;", k); break;        /* k != 0 (mosrx_bpf_check) */
		case ALU | AND | K: sb_printf(s, "A &= %uu;", k); break;
		case ALU | OR | K: sb_printf(s, "A |= %uu;", k); break;
		case ALU | LSH | K: sb_printf(s, "A <<= %uu;", k & 31u); break;
		case ALU | RSH | K: sb_printf(s, "A >>= %uu;", k & 31u); break;
		case ALU | NEG: sb_printf(s, "A = 0u - A;"); break;
		case MISC | TAX: sb_printf(s, "X = A;"); break;
		case MISC | TXA: sb_printf(s, "A = X;"); break;
		default:   /* rejected by mosrx_bpf_check */
			return -EINVAL;
		}
		sb_printf(s, "\n");
	}
	return 0;
}

/* Registers of the BPF machine as bits: A, X, the 16 scratch slots. */
#define RB_A 1u
#define RB_X 2u
#define RB_M(k) (4u << ((k) & 15u))

static void insn_use_def(const mosrx_bpf_insn *f, uint32_t *use, uint32_t *def)
{
	const uint16_t c = f->code;
	*use = *def = 0;
	switch (c & 7) {
	case LD:
		*def = RB_A;
		if ((c & 0xe0) == IND) *use = RB_X;
		else if ((c & 0xe0) == MEM) *use = RB_M(f->k);
		break;
	case LDX:
		*def = RB_X;
		if ((c & 0xe0) == MEM) *use = RB_M(f->k);
		break;
	case ST: *use = RB_A; *def = RB_M(f->k); break;
	case STX: *use = RB_X; *def = RB_M(f->k); break;
	case ALU: *use = RB_A | ((c & 8) && (c & 0xf0) != NEG ? RB_X : 0); *def = RB_A; break;
	case JMP: if (c != (JMP | JA)) *use = RB_A | ((c & 8) ? RB_X : 0); break;
	case RET: if ((c & 0x18) == A) *use = RB_A; break;
	case MISC: if (c == (MISC | TAX)) { *use = RB_A; *def = RB_X; } else { *use = RB_X; *def = RB_A; } break;
	}
}

/* Program j if-converted, for the lanes whose L covers every constant-offset
 * load: no branches.  Each lane's position is a predicate -- `c` for the
 * instruction being emitted, b<i> for the jump targets not yet reached -- a
 * jump moves `c` into its targets' predicates, a return sets the lane's hit
 * flag `h`.  A write to A / X / a scratch slot is a select on `c` only when a
 * lane waiting at a pending jump target still needs the old value (liveness
 * over the program's DAG); mOS filters reload A after nearly every jump, so
 * most writes are plain, and the same load in several programs of the set
 * becomes one value (one compare) for all of them.  The branchy form pays the
 * structurizer's exec-mask bookkeeping at every join instead.  Blocks of 4 or
 * more instructions no lane reaches are skipped with a uniform branch. */
static int gen_pred(struct sbuf *s, const mosrx_bpf_insn *f, uint32_t len, const uint8_t *tgt,
                    const struct genopt *g)
{
	uint32_t i, t, e = 0, *live, *need;
	int open = 0;
	live = calloc((size_t)len + 1, sizeof(*live));   /* registers live on entry to instruction i */
	need = calloc((size_t)len + 1, sizeof(*need));   /* of them, those a lane waiting at target i needs */
	if (!live || !need) {
		free(live);
		free(need);
		return -ENOMEM;
	}
	for (i = len; i-- > 0;) {
		const uint16_t c = f[i].code;
		uint32_t use, def, out = 0;
		insn_use_def(&f[i], &use, &def);
		if (c == (JMP | JA))
			out = live[i + 1 + f[i].k];
		else if ((c & 7) == JMP)
			out = live[i + 1 + f[i].jt] | live[i + 1 + f[i].jf];
		else if ((c & 7) != RET)
			out = live[i + 1];
		live[i] = use | (out & ~def);
	}
	for (i = 1; i < len; i++)
		if (tgt[i] & TG_TARGET)
			sb_printf(s, "    bool b%u = false;\n", (unsigned)i);
	for (i = 0; i < len; i++) {
		const uint16_t c = f[i].code;
		const uint32_t k = f[i].k;
		const unsigned jt = i + 1 + f[i].jt, jf = i + 1 + f[i].jf;
		uint32_t use, def, wait = 0;
		const char *r;
		insn_use_def(&f[i], &use, &def);
		for (t = i + 1; t < len; t++)   /* what the lanes parked at targets past i still read */
			wait |= need[t];
		if (i == 0 || (tgt[i] & TG_TARGET)) {
			if (i > 0)
				sb_printf(s, "    c = c || b%u;\n", (unsigned)i);
			/* the block: up to its jump / return, or up to the next jump target */
			for (e = i; e + 1 < len && (f[e].code & 7) != JMP && (f[e].code & 7) != RET && !(tgt[e + 1] & TG_TARGET); e++)
				;
			if (e - i + 1 >= 4) {
				sb_printf(s, "    if (__any(c)) {\n");
				open = 1;
			}
		}
		sb_printf(s, "      ");
		if ((c == (LD | W | ABS) && (uint64_t)k + 4 > 0xFFFFFFFFull) ||
		    (c == (LD | H | ABS) && (uint64_t)k + 2 > 0xFFFFFFFFull) ||
		    ((c == (LD | B | ABS) || c == (LDX | MSH | B)) && (uint64_t)k + 1 > 0xFFFFFFFFull)) {
			sb_printf(s, "c = false;\n");   /* past any length: the lane returns 0 */
			goto next;
		}
		/* "R = (value);" or "R = c ? (value) : R;" */
		r = def == RB_A ? "A" : def == RB_X ? "X" : NULL;
#define SET_OPEN(name) do { if (def & wait) sb_printf(s, "%s = c ? (", name); else sb_printf(s, "%s = (", name); } while (0)
#define SET_CLOSE(name) do { if (def & wait) sb_printf(s, ") : %s;", name); else sb_printf(s, ");"); } while (0)
		switch (c) {
		case RET | K: sb_printf(s, k ? "h = h || c; c = false;" : "c = false;"); break;
		case RET | A: sb_printf(s, "h = h || (c && A != 0u); c = false;"); break;
		case LD | W | ABS: SET_OPEN(r); sb_printf(s, "be32("); gen_ld(s, k, 4, g); sb_printf(s, ")"); SET_CLOSE(r); break;
		case LD | H | ABS: SET_OPEN(r); sb_printf(s, "be16("); gen_ld(s, k, 2, g); sb_printf(s, ")"); SET_CLOSE(r); break;
		case LD | B | ABS: SET_OPEN(r); gen_ld(s, k, 1, g); sb_printf(s, " & 0xFFu"); SET_CLOSE(r); break;
		case LD | W | LEN: case LDX | W | LEN: SET_OPEN(r); sb_printf(s, "L"); SET_CLOSE(r); break;
		case LD | W | IND: case LD | H | IND: case LD | B | IND: {
			const uint32_t size = (c & 0x18) == W ? 4 : (c & 0x18) == H ? 2 : 1;
			sb_printf(s, "{ const u32 kk = X + %uu; c = c && (u64)kk + %uu <= L; u32 v; ", k, size);
			if (g->fused && (tgt[i] & TG_XMSH) && (uint64_t)k + 20 + 8 <= g->wend) {
				/* the speculated window read; a wave with any other live X also reads memory */
				sb_printf(s, "v = ");
				gen_ld(s, k + 20, size, g);
				sb_printf(s, "; if (__any(c && X != 20u)) v = X == 20u ? v : hk_ld_le32(rs, o + kk); ");
			} else if (g->fused && !(tgt[i] & TG_XMSH) && g->lds) {
				sb_printf(s, "v = hk_ind_le32<HL>(bw, c ? kk : 2u, rs, o); ");
			} else if (g->fused) {
				sb_printf(s, "v = hk_ld_le32(rs, o + kk); ");   /* a buffer load: out-of-range offsets read 0 */
			} else if ((tgt[i] & TG_XMSH) && (uint64_t)k + 20 + 8 <= 4ull * g->stage_w) {
				sb_printf(s, "v = W32(%uu); if (__any(c && X != 20u)) v = X == 20u ? v : fr_le32(win, sh, rs, o, kk, %uu); ",
				          k + 20, size);
			} else {   /* lanes off the path read the stage at offset 0, not at their X + k */
				sb_printf(s, "v = fr_le32(win, sh, rs, o, c ? kk : 0u, %uu); ", size);
			}
			SET_OPEN(r);
			sb_printf(s, size == 4 ? "be32(v)" : size == 2 ? "be16(v)" : "v & 0xFFu");
			SET_CLOSE(r);
			sb_printf(s, " }");
			break;
		}
		case LDX | MSH | B: SET_OPEN(r); sb_printf(s, "("); gen_ld(s, k, 1, g); sb_printf(s, " & 0xFu) << 2"); SET_CLOSE(r); break;
		case LD | IMM: case LDX | IMM: SET_OPEN(r); sb_printf(s, "%uu", k); SET_CLOSE(r); break;
		case LD | MEM: case LDX | MEM: SET_OPEN(r); sb_printf(s, "M%u", k & 15); SET_CLOSE(r); break;
		case ST: case STX: {
			char m[8];
			snprintf(m, sizeof(m), "M%u", k & 15);
			SET_OPEN(m); sb_printf(s, c == ST ? "A" : "X"); SET_CLOSE(m);
			break;
		}
		case JMP | JA: sb_printf(s, "b%u = b%u || c; c = false;", (unsigned)(i + 1 + k), (unsigned)(i + 1 + k)); break;
		case JMP | JGT | K: case JMP | JGE | K: case JMP | JEQ | K: case JMP | JSET | K:
		case JMP | JGT | X: case JMP | JGE | X: case JMP | JEQ | X: case JMP | JSET | X: {
			const char *rhs = (c & 8) ? "X" : NULL;
			char kb[16];
			const char *op = (c & 0xf0) == JGT ? ">" : (c & 0xf0) == JGE ? ">=" : (c & 0xf0) == JEQ ? "==" : "&";
			if (!rhs) {
				snprintf(kb, sizeof(kb), "%uu", k);
				rhs = kb;
			}
			if (jt == jf) {
				sb_printf(s, "b%u = b%u || c; c = false;", jt, jt);
				break;
			}
			sb_printf(s, (c & 0xf0) == JSET ? "{ const bool t_ = (A & %s) != 0u; " : "{ const bool t_ = A %s %s; ",
			          (c & 0xf0) == JSET ? rhs : op, rhs);
			sb_printf(s, "b%u = b%u || (c && t_); b%u = b%u || (c && !t_); c = false; }", jt, jt, jf, jf);
			break;
		}
		case ALU | DIV | X:
			sb_printf(s, "c = c && X != 0u; ");
			SET_OPEN(r); sb_printf(s, "A / (X ? X : 1u)"); SET_CLOSE(r);
			break;
		case ALU | NEG: SET_OPEN(r); sb_printf(s, "0u - A"); SET_CLOSE(r); break;
		case MISC | TAX: SET_OPEN(r); sb_printf(s, "A"); SET_CLOSE(r); break;
		case MISC | TXA: SET_OPEN(r); sb_printf(s, "X"); SET_CLOSE(r); break;
		default:
			if ((c & 7) == ALU) {
				static const char *const ops[] = {"+", "-", "*", "/", "|", "&", "<<", ">>"};
				const unsigned o = (c & 0xf0) >> 4;
				if (o > 7)
					goto bad;
				SET_OPEN(r);
				if (c & 8)
					sb_printf(s, o >= 6 ? "A %s (X & 31u)" : "A %s X", ops[o]);
				else
					sb_printf(s, "A %s %uu", ops[o], o >= 6 ? k & 31u : k);   /* DIV K: k != 0 (mosrx_bpf_check) */
				SET_CLOSE(r);
				break;
			}
		bad:
			free(live);
			free(need);
			return -EINVAL;
		}
#undef SET_OPEN
#undef SET_CLOSE
		sb_printf(s, "\n");
	next:
		/* a jump parks its lanes at its targets: they need what is live there */
		if (c == (JMP | JA))
			need[i + 1 + k] |= live[i + 1 + k];
		else if ((c & 7) == JMP) {
			need[jt] |= live[jt];
			need[jf] |= live[jf];
		}
		if (open && i == e) {
			sb_printf(s, "    }\n");
			open = 0;
		}
	}
	free(live);
	free(need);
	return 0;
}

static int gen_program(struct sbuf *s, unsigned j, const mosrx_bpf_insn *f, uint32_t len, int ipm,
                       const struct genopt *g)
{
	uint8_t *tgt, mem_used[16];
	uint32_t i, q;
	uint64_t maxk = 0;   /* every constant-offset load lies below it */
	int rc;

	sb_printf(s, "  { /* program %u, %u insns, %s length */\n", j, (unsigned)len, ipm ? "datagram" : "frame");
	if (len == 0) {
		sb_printf(s, "    if (live%s) match |= %uu;\n  }\n", ipm ? " && lip != 0u" : "", 1u << j);
		return 0;
	}
	tgt = calloc(len + 1, 1);
	if (!tgt)
		return -ENOMEM;
	x_provenance(f, len, tgt);
	memset(mem_used, 0, sizeof(mem_used));
	for (i = 0; i < len; i++) {
		const uint16_t c = f[i].code;
		if ((c & 7) == JMP) {
			if (c == (JMP | JA)) {
				tgt[i + 1 + f[i].k] |= TG_TARGET;
			} else {
				tgt[i + 1 + f[i].jt] |= TG_TARGET;
				tgt[i + 1 + f[i].jf] |= TG_TARGET;
			}
		}
		if (c == (LD | MEM) || c == (LDX | MEM) || c == ST || c == STX)
			mem_used[f[i].k & 15] = 1;
		{
			const uint64_t end = c == (LD | W | ABS) ? (uint64_t)f[i].k + 4 : c == (LD | H | ABS) ? (uint64_t)f[i].k + 2
			                   : c == (LD | B | ABS) || c == (LDX | MSH | B) ? (uint64_t)f[i].k + 1 : 0;
			if (end <= 0xFFFFFFFFull && end > maxk)
				maxk = end;
		}
	}
	sb_printf(s, "    u32 A = 0, X = 0, ret = 0;\n");
	for (q = 0; q < 16; q++)
		if (mem_used[q])
			sb_printf(s, "    u32 M%u = 0;\n", q);
	sb_printf(s, "    const u32 L = %s;\n", ipm ? "lip" : "cap");
	if (g->pred && maxk <= 65535) {   /* lengths are 16-bit: a larger bound never holds */
		const char *lv = ipm ? "live && lip != 0u" : "live";
		sb_printf(s, "    bool h = false;\n");
		if (maxk)
			sb_printf(s, "    bool c = %s && L >= %uu;\n", lv, (unsigned)maxk);
		else
			sb_printf(s, "    bool c = %s;\n", lv);
		if ((rc = gen_pred(s, f, len, tgt, g))) {
			free(tgt);
			return rc;
		}
		if (!maxk) {
			sb_printf(s, "    if (h) match |= %uu;\n  }\n", 1u << j);
			free(tgt);
			return 0;
		}
		/* frames shorter than the program's furthest constant load: the checked copy */
		sb_printf(s, "    if (__any(%s && L < %uu)) {\n    if (%s && L < %uu) {\n", lv, (unsigned)maxk, lv,
		          (unsigned)maxk);
		/* the if-converted code wrote registers of lanes off its path: start afresh */
		sb_printf(s, "    A = 0u; X = 0u;");
		for (q = 0; q < 16; q++)
			if (mem_used[q])
				sb_printf(s, " M%u = 0u;", q);
		sb_printf(s, "\n");
		if ((rc = gen_body(s, j, f, len, tgt, "", g))) {
			free(tgt);
			return rc;
		}
		sb_printf(s, "  P%u_R0: ret = 0;\n    }}\n", j);
		sb_printf(s, "  P%u_E: if (h || ret) match |= %uu;\n  }\n", j, 1u << j);
		free(tgt);
		return 0;
	}
	sb_printf(s, "    if (!live%s) goto P%u_E;\n", ipm ? " || lip == 0u" : "", j);
	if (maxk && maxk <= 65535) {
		tgt[0] |= TG_TARGET;
		sb_printf(s, "    if (L >= %uu) goto P%u_F0;\n", (unsigned)maxk, j);
		if ((rc = gen_body(s, j, f, len, tgt, "", g)) || (rc = gen_body(s, j, f, len, tgt, "F", g))) {
			free(tgt);
			return rc;
		}
	} else if ((rc = gen_body(s, j, f, len, tgt, "", g))) {
		free(tgt);
		return rc;
	}
	/* P<j>_R0 is always emitted (the fast copy's indexed loads and divisions jump there too) */
	sb_printf(s, "  P%u_R0: ret = 0;\n", j);
	sb_printf(s, "  P%u_E: if (ret) match |= %uu;\n  }\n", j, 1u << j);
	free(tgt);
	return 0;
}

/* FNV-1a over the set (instructions + table): the module cache key. */
static uint64_t set_hash(const mosrx_bpf_insn *insns, const mosrx_bparams *t)
{
	uint64_t h = 1469598103934665603ull;
	uint32_t j, total = 0;
	const uint8_t *q;
	size_t i;
#define MIX(ptr, nbytes) for (q = (const uint8_t *)(ptr), i = 0; i < (size_t)(nbytes); i++) h = (h ^ q[i]) * 1099511628211ull
	MIX(&t->nprog, sizeof(t->nprog));
	MIX(&t->ip_mode, sizeof(t->ip_mode));
	for (j = 0; j < t->nprog; j++) {
		MIX(&t->prog_len[j], sizeof(t->prog_len[j]));
		total += t->prog_len[j];
	}
	MIX(insns, (size_t)total * sizeof(*insns));
#undef MIX
	return h;
}

/* 16-byte pieces of each frame to stage in LDS: enough for every constant
 * offset the set loads, and for loads at X + k the offset X most frames give:
 * 4 * ihl with ihl 5 where only `ldxb 4*([k]&0xf)` defines X (x_provenance),
 * else IPv4 + a TCP header with timestamps (52); loads past the stage read
 * memory.  A window read costs the HBM sectors it touches (the IMIX launch
 * moved 2x its algorithmic bytes staging 96 bytes per frame), so it is no
 * longer than the set needs. */
static uint32_t stage_pieces(const mosrx_bpf_insn *insns, const mosrx_bparams *t)
{
	uint64_t need = 18;   /* the datagram-length probe reads frame bytes 12..17 */
	uint32_t j, i;
	for (j = 0; j < t->nprog; j++) {
		const mosrx_bpf_insn *f = &insns[t->prog_off[j]];
		uint8_t *tg = calloc((size_t)t->prog_len[j] + 1, 1);
		if (!tg)
			return 9;
		x_provenance(f, t->prog_len[j], tg);
		for (i = 0; i < t->prog_len[j]; i++) {
			const uint16_t c = f[i].code;
			const uint64_t size = (c & 0x18) == W ? 4 : (c & 0x18) == H ? 2 : 1;
			uint64_t end = 0;
			if (c == (LD | W | ABS) || c == (LD | H | ABS) || c == (LD | B | ABS) || c == (LDX | MSH | B))
				end = (uint64_t)f[i].k + size;
			else if (c == (LD | W | IND) || c == (LD | H | IND) || c == (LD | B | IND))
				end = (uint64_t)f[i].k + size + ((tg[i] & TG_XMSH) ? 20 : 52);
			if (end > need)
				need = end;
		}
		free(tg);
	}
	if (getenv("MOSRX_BPF_STAGE96") && need < 96)   /* diagnostic: round 3's 96 bytes for any indexed load */
		need = 96;
	/* frame bytes [0, 16 V - 3) are staged whatever the start alignment */
	need = (need + 3 + 15) / 16;
	return need > 9 ? 9 : (uint32_t)need;
}

int mosrx__bpf_jit_source(const mosrx_bpf_insn *insns, const mosrx_bparams *t, char **out)
{
	struct sbuf s = {0};
	const uint32_t v = stage_pieces(insns, t);
	const struct genopt g = {0, 4 * v - 1, 0, pred_mode(), 0};
	uint32_t j;
	int rc, lds = 0;
	*out = NULL;
	for (j = 0; j < t->nprog && !lds; j++) {
		uint8_t *tg = calloc((size_t)t->prog_len[j] + 1, 1);
		lds = !tg || x_provenance(insns + t->prog_off[j], t->prog_len[j], tg);
		free(tg);
	}
	sb_printf(&s, "#define STAGE_V %uu\n#define STAGE_LD %uu\n#define STAGE_B %uu\n#define STAGE_LDS %d\n", v, 4 * v + 1,
	          16 * v - 3, lds);
	sb_printf(&s, "%s", k_preamble);
	for (j = 0; j < t->nprog; j++)
		if ((rc = gen_program(&s, j, insns + t->prog_off[j], t->prog_len[j], (t->ip_mode >> j) & 1u, &g))) {
			free(s.p);
			return rc;
		}
	sb_printf(&s, "  if (live) match_out[p] = match;\n}\n");
	if (s.err) {
		free(s.p);
		return -ENOMEM;
	}
	*out = s.p;
	return 0;
}

/* The fused hook: the program set as a device function the classify header
 * wave calls with its 96-byte window (mosrx_kernels.hip, VAR_BPF), plus the
 * kernel entry points that instantiate the S13 and SMALL tiles with it. */
static const char k_hook_pre[] =
	"typedef unsigned int u32;\n"
	"typedef unsigned long long u64;\n"
	"static __device__ __attribute__((always_inline)) inline u32 be32(u32 v) { return __builtin_bswap32(v); }\n"
	"static __device__ __attribute__((always_inline)) inline u32 be16(u32 v) { return ((v & 0xFFu) << 8) | ((v >> 8) & 0xFFu); }\n"
	"static __device__ __attribute__((always_inline)) inline u32 hk_ld_le32(__amdgpu_buffer_rsrc_t rs, u32 a) {\n"
	"  const u32 a4 = a & ~3u;\n"
	"  const u32 lo = __builtin_amdgcn_raw_buffer_load_b32(rs, a4, 0, 0);\n"
	"  const u32 hi = __builtin_amdgcn_raw_buffer_load_b32(rs, a4 + 4u, 0, 0);\n"
	"  return __builtin_amdgcn_alignbyte(hi, lo, a & 3u);\n"
	"}\n"
	"/* frame bytes [kk, kk+4) at a run-time offset: the hook's LDS copy of the window (dword j of the lane at\n"
	"   bw[HL j], HL header lanes per workgroup), memory past it */\n"
	"template <u32 HL>\n"
	"static __device__ __attribute__((always_inline)) inline u32 hk_ind_le32(const u32 *bw, u32 kk,\n"
	"    __amdgpu_buffer_rsrc_t rs, u32 o) {\n"
	"  if (kk >= 2u && kk + 8u <= MOSRX_BPF_WEND) {\n"
	"    const u32 a = kk - 2u;\n"
	"    return __builtin_amdgcn_alignbyte(bw[HL * ((a >> 2) + 1u)], bw[HL * (a >> 2)], a & 3u);\n"
	"  }\n"
	"  return hk_ld_le32(rs, o + kk);\n"
	"}\n"
	"/* frame bytes [k, k+4), k constant in [2, 86]: the realigned window registers */\n"
	"#define RW32(k) (((k) - 2u) % 4u == 0u ? w[((k) - 2u) / 4u] \\\n"
	"                 : __builtin_amdgcn_alignbyte(w[((k) - 2u) / 4u + 1u], w[((k) - 2u) / 4u], ((k) - 2u) % 4u))\n"
	"/* w: the header wave's realigned window, frame bytes [4j + 2, 4j + 6) in w[j], valid up to MOSRX_BPF_WEND;\n"
	"   HL: the workgroup's header lanes (the SMALL tile 256, the stream tile's one header wave 64) */\n"
	"template <u32 HL>\n"
	"static __device__ __attribute__((always_inline)) inline u32 mosrx_bpf_hook(const u32 *w, u32 o, u32 cap,\n"
	"    bool live, __amdgpu_buffer_rsrc_t rs) {\n"
	"  u32 lip = 0;\n"
	"  if (cap >= 18u && be16hi(w[2]) == 0x0800u) {\n"
	"    lip = 14u + be16hi(w[3]);\n"
	"    if (lip > cap) lip = 0;\n"
	"  }\n"
	"  u32 match = 0;\n";

/* Entry points of the fused module: one batch (kp), and the batch queue (a
 * descriptor table of resident batches, one launch; gpu_module_func's groups),
 * each as the stream tile with non-temporal tails, the stream tile with cached
 * tails (batches of small frames) and the SMALL tile. */
static const char k_fused_main[] =
	"#define MOSRX_RTC_BPF 1\n"
	"#include \"mosrx_kernels.hip\"\n"
	"#define WGS __launch_bounds__(WG_THREADS(MOSRX_KIND_S13)) __attribute__((amdgpu_waves_per_eu(MIN_WAVES(MOSRX_KIND_S13))))\n"
	"#define WGM __launch_bounds__(WG_THREADS(MOSRX_KIND_SMALL))\n"
	"extern \"C\" __global__ WGS void mosrx_classify_bpf_stream(mosrx_kparams kp)\n"
	"{ classify_tile<MOSRX_KIND_S13, 2 | VAR_BPF>(kp, blockIdx.x); }\n"
	"extern \"C\" __global__ WGS void mosrx_classify_bpf_stream_rt(mosrx_kparams kp)\n"
	"{ classify_tile<MOSRX_KIND_S13, VAR_BPF>(kp, blockIdx.x); }\n"
	"extern \"C\" __global__ WGM void mosrx_classify_bpf_small(mosrx_kparams kp)\n"
	"{ classify_tile<MOSRX_KIND_SMALL, 2 | VAR_BPF>(kp, blockIdx.x); }\n"
	"extern \"C\" __global__ WGS void mosrx_classify_bpf_queue_stream(const mosrx_qdesc *desc, uint32_t tpb, uint32_t nb,\n"
	"    mosrx_qparams qp)\n"
	"{ queue_tile<MOSRX_KIND_S13, 2 | VAR_BPF>(desc, tpb, nb, qp); }\n"
	"extern \"C\" __global__ WGS void mosrx_classify_bpf_queue_stream_rt(const mosrx_qdesc *desc, uint32_t tpb,\n"
	"    uint32_t nb, mosrx_qparams qp)\n"
	"{ queue_tile<MOSRX_KIND_S13, VAR_BPF>(desc, tpb, nb, qp); }\n"
	"extern \"C\" __global__ WGM void mosrx_classify_bpf_queue_small(const mosrx_qdesc *desc, uint32_t tpb, uint32_t nb,\n"
	"    mosrx_qparams qp)\n"
	"{ queue_tile<MOSRX_KIND_SMALL, 2 | VAR_BPF>(desc, tpb, nb, qp); }\n"
	/* the same three queue forms with 8-byte records (gpu_module_func cfg.compact with filters) */
	"extern \"C\" __global__ WGS void mosrx_classify_bpf_queue_stream_c8(const mosrx_qdesc *desc, uint32_t tpb,\n"
	"    uint32_t nb, mosrx_qparams qp)\n"
	"{ queue_tile<MOSRX_KIND_S13, 2 | VAR_BPF | VAR_C8>(desc, tpb, nb, qp); }\n"
	"extern \"C\" __global__ WGS void mosrx_classify_bpf_queue_stream_rt_c8(const mosrx_qdesc *desc, uint32_t tpb,\n"
	"    uint32_t nb, mosrx_qparams qp)\n"
	"{ queue_tile<MOSRX_KIND_S13, VAR_BPF | VAR_C8>(desc, tpb, nb, qp); }\n"
	"extern \"C\" __global__ WGM void mosrx_classify_bpf_queue_small_c8(const mosrx_qdesc *desc, uint32_t tpb,\n"
	"    uint32_t nb, mosrx_qparams qp)\n"
	"{ queue_tile<MOSRX_KIND_SMALL, 2 | VAR_BPF | VAR_C8>(desc, tpb, nb, qp); }\n";

static const char *const k_fused_names[MOSRX_BPF_NFUSED] = {
	"mosrx_classify_bpf_stream", "mosrx_classify_bpf_stream_rt", "mosrx_classify_bpf_small",
	"mosrx_classify_bpf_queue_stream", "mosrx_classify_bpf_queue_stream_rt", "mosrx_classify_bpf_queue_small",
	"mosrx_classify_bpf_queue_stream_c8", "mosrx_classify_bpf_queue_stream_rt_c8", "mosrx_classify_bpf_queue_small_c8"};

/* The header window a fused set needs: every constant-offset load at frame
 * bytes [k, k + 8) with k >= 2 -- and every indexed load at its speculated
 * offset k + 20 -- inside it is read from the window's registers, anything
 * else from memory.  The smallest of the tiles' windows (62 / 78 / 94 bytes:
 * 4 / 5 / 6 chunks) that holds them, so the fused tiles load no more than the
 * classify tiles for the filters mOS compiles (they read Ethernet, IP and
 * TCP header fields). */
static uint32_t hook_wend(const mosrx_bpf_insn *insns, const mosrx_bparams *t, int *lds)
{
	uint64_t need = 18;   /* the datagram-length probe reads frame bytes 12..17 */
	uint32_t j, i;
	*lds = 0;
	for (j = 0; j < t->nprog; j++) {
		const mosrx_bpf_insn *f = &insns[t->prog_off[j]];
		uint8_t *tg = calloc((size_t)t->prog_len[j] + 1, 1);
		if (!tg)
			return MOSRX_WINDOW_END_FULL;
		*lds |= x_provenance(f, t->prog_len[j], tg);
		for (i = 0; i < t->prog_len[j]; i++) {
			const uint16_t c = f[i].code;
			uint64_t end = 0;
			if (c == (LD | W | ABS) || c == (LD | H | ABS) || c == (LD | B | ABS) || c == (LDX | MSH | B))
				end = f[i].k >= 2 ? (uint64_t)f[i].k + 8 : 0;
			else if (c == (LD | W | IND) || c == (LD | H | IND) || c == (LD | B | IND))
				/* X = 4 * ihl: ihl 5; any other X: a payload offset past IPv4 + a TCP header with
				 * timestamps (20 + 32: 42 % of the IMIX trace's segments, most of a real trace's) */
				end = (uint64_t)f[i].k + ((tg[i] & TG_XMSH) ? 20 : 52) + 8;
			if (end > need && end <= MOSRX_WINDOW_END_FULL)
				need = end;
		}
		free(tg);
	}
	return need <= MOSRX_WINDOW_END_STREAM ? MOSRX_WINDOW_END_STREAM
	     : need <= MOSRX_WINDOW_END_SMALL ? MOSRX_WINDOW_END_SMALL : MOSRX_WINDOW_END_FULL;
}

int mosrx__bpf_jit_hook_source(const mosrx_bpf_insn *insns, const mosrx_bparams *t, char **out)
{
	struct sbuf s = {0};
	struct genopt g = {1, 0, 0, pred_mode(), 0};
	uint32_t j;
	int rc;
	*out = NULL;
	g.wend = hook_wend(insns, t, &g.lds);
	sb_printf(&s, "/* generated by bpf_jit.c */\n#define MOSRX_BPF_WEND %u\n%s", g.wend, k_hook_pre);
	if (g.lds)   /* the window, column per lane (conflict-free): loads at X + k index it */
		sb_printf(&s, "  __shared__ u32 s_bw[(MOSRX_BPF_WEND - 2u) / 4u * HL];\n"
		              "  u32 *const bw = s_bw + threadIdx.x % HL;\n"
		              "#pragma unroll\n"
		              "  for (u32 j = 0; j < (MOSRX_BPF_WEND - 2u) / 4u; j++) bw[HL * j] = w[j];\n");
	for (j = 0; j < t->nprog; j++)
		if ((rc = gen_program(&s, j, insns + t->prog_off[j], t->prog_len[j], (t->ip_mode >> j) & 1u, &g))) {
			free(s.p);
			return rc;
		}
	sb_printf(&s, "  return match;\n}\n#undef RW32\n");
	if (s.err) {
		free(s.p);
		return -ENOMEM;
	}
	*out = s.p;
	return 0;
}

/* hipRTC compiles are serialised process-wide: every mTCP thread's context has
 * its own compile thread, and the compiles are rare (a filter set change). */
static pthread_mutex_t g_rtc_lock = PTHREAD_MUTEX_INITIALIZER;

/* Code objects already built in this process, by source text: every mTCP
 * thread's context compiles the same set when mOS installs its filters, and
 * after the first one the others only load it (hipRTC through comgr's disk
 * cache still takes ~50 ms a time, serialised by g_rtc_lock). */
#define RTC_CACHE 8
static struct rtc_cached {
	char *src, *hook;   /* the program text and its last header (the generated hook), exact keys */
	int nh;
	char *code;
	size_t size;
	uint64_t used;
} g_rtc_cache[RTC_CACHE];
static uint64_t g_rtc_tick;

static int rtc_cache_get(const char *src, int nh, const char *hook, char **code, size_t *size)
{
	int i;
	for (i = 0; i < RTC_CACHE; i++) {
		struct rtc_cached *e = &g_rtc_cache[i];
		if (e->code && e->nh == nh && !strcmp(e->src, src) && !strcmp(e->hook, hook)) {
			if (!(*code = malloc(e->size)))
				return 0;
			memcpy(*code, e->code, e->size);
			*size = e->size;
			e->used = ++g_rtc_tick;
			return 1;
		}
	}
	return 0;
}

static void rtc_cache_put(const char *src, int nh, const char *hook, const char *code, size_t size)
{
	struct rtc_cached *e = NULL;
	char *s2, *h2, *c2;
	int i;
	for (i = 0; i < RTC_CACHE && !e; i++)   /* an empty slot, else the least recently used */
		if (!g_rtc_cache[i].code)
			e = &g_rtc_cache[i];
	if (!e)
		for (e = &g_rtc_cache[0], i = 1; i < RTC_CACHE; i++)
			if (g_rtc_cache[i].used < e->used)
				e = &g_rtc_cache[i];
	s2 = strdup(src);
	h2 = strdup(hook);
	c2 = malloc(size);
	if (!s2 || !h2 || !c2) {
		free(s2);
		free(h2);
		free(c2);
		return;
	}
	memcpy(c2, code, size);
	free(e->src);
	free(e->hook);
	free(e->code);
	e->src = s2;
	e->hook = h2;
	e->nh = nh;
	e->code = c2;
	e->size = size;
	e->used = ++g_rtc_tick;
}

/* hipRTC: source -> gfx950 code object (malloc'd into *code). */
static int compile_code_h(const char *src, int nh, const char *const *htexts, const char *const *hnames,
                          char **code, size_t *size, char *log, size_t logsz)
{
	hiprtcProgram prog;
	/* the library's kernarg preloading (Makefile KFLAGS): the kernels' leading
	 * scalar arguments arrive in SGPRs at dispatch */
	const char *opts[] = {"--offload-arch=gfx950", "-O3", "-mllvm", "-amdgpu-kernarg-preload-count=7"};
	size_t sz = 0;
	int rc = 0;
	const char *hook = nh ? htexts[nh - 1] : "";
	*code = NULL;
	pthread_mutex_lock(&g_rtc_lock);
	if (rtc_cache_get(src, nh, hook, code, size)) {
		pthread_mutex_unlock(&g_rtc_lock);
		return 0;
	}
	if (hiprtcCreateProgram(&prog, src, "mosrx_bpf_jit.hip", nh, (const char **)htexts, (const char **)hnames) !=
	    HIPRTC_SUCCESS) {
		pthread_mutex_unlock(&g_rtc_lock);
		return -EIO;
	}
	if (hiprtcCompileProgram(prog, (int)(sizeof(opts) / sizeof(opts[0])), opts) != HIPRTC_SUCCESS) {
		size_t ls = 0;
		if (log && logsz && hiprtcGetProgramLogSize(prog, &ls) == HIPRTC_SUCCESS && ls) {
			char *l = malloc(ls + 1);
			if (l && hiprtcGetProgramLog(prog, l) == HIPRTC_SUCCESS) {
				l[ls] = 0;
				snprintf(log, logsz, "%s", l);
			}
			free(l);
		}
		hiprtcDestroyProgram(&prog);
		pthread_mutex_unlock(&g_rtc_lock);
		return -EIO;
	}
	if (hiprtcGetCodeSize(prog, &sz) != HIPRTC_SUCCESS || !sz || !(*code = malloc(sz)))
		rc = -EIO;
	else if (hiprtcGetCode(prog, *code) != HIPRTC_SUCCESS)
		rc = -EIO;
	hiprtcDestroyProgram(&prog);
	if (!rc)
		rtc_cache_put(src, nh, hook, *code, sz);
	pthread_mutex_unlock(&g_rtc_lock);
	if (!rc && getenv("MOSRX_BPF_DUMP")) {   /* diagnostics: the code object, for llvm-readelf --notes */
		char path[512];
		FILE *f;
		snprintf(path, sizeof(path), "%s.%s.co", getenv("MOSRX_BPF_DUMP"), nh ? "fused" : "set");
		if ((f = fopen(path, "wb"))) {
			fwrite(*code, 1, sz, f);
			fclose(f);
		}
	}
	if (rc) {
		free(*code);
		*code = NULL;
	}
	*size = sz;
	return rc;
}

static int compile_code(const char *src, char **code, size_t *size, char *log, size_t logsz)
{
	return compile_code_h(src, 0, NULL, NULL, code, size, log, logsz);
}

extern const int mosrx__src_count;
extern const char *const mosrx__src_names[];
extern const char *const mosrx__src_texts[];

/* The fused classify + BPF module: the embedded kernel sources + the hook. */
static int compile_fused(const char *hook, hipModule_t *mod, hipFunction_t *fu, char *log, size_t logsz,
                         size_t *code_size)
{
	const char *names[8], *texts[8];
	char *code;
	size_t sz = 0;
	int i, n = mosrx__src_count, rc;
	for (i = 0; i < n && i < 7; i++) {
		names[i] = mosrx__src_names[i];
		texts[i] = mosrx__src_texts[i];
	}
	names[n] = "mosrx_bpf_hook.h";
	texts[n] = hook;
	rc = compile_code_h(k_fused_main, n + 1, texts, names, &code, &sz, log, logsz);
	if (code_size)
		*code_size = rc ? 0 : sz;
	if (rc || !mod) {
		free(code);
		return rc;
	}
	if (hipModuleLoadData(mod, code) != hipSuccess) {
		rc = -EIO;
	} else {
		for (i = 0; i < MOSRX_BPF_NFUSED && !rc; i++)
			if (hipModuleGetFunction(&fu[i], *mod, k_fused_names[i]) != hipSuccess)
				rc = -EIO;
		if (rc) {
			hipModuleUnload(*mod);
			*mod = NULL;
		}
	}
	free(code);
	return rc;
}

static int compile_module(const char *src, hipModule_t *mod, hipFunction_t *fn, char *log, size_t logsz)
{
	char *code;
	size_t sz;
	int rc = compile_code(src, &code, &sz, log, logsz);
	if (rc)
		return rc;
	if (hipModuleLoadData(mod, code) != hipSuccess || hipModuleGetFunction(fn, *mod, "mosrx_bpf_jit") != hipSuccess)
		rc = -EIO;
	free(code);
	return rc;
}

int mosrx__bpf_jit_compile_fused(const mosrx_bpf_insn *insns, const mosrx_bparams *t, char *log, size_t logsz,
                                 size_t *code_size)
{
	char *hook = NULL;
	int rc = mosrx__bpf_jit_hook_source(insns, t, &hook);
	if (!rc)
		rc = compile_fused(hook, NULL, NULL, log, logsz, code_size);
	free(hook);
	return rc;
}

int mosrx__bpf_jit_compile(const char *src, char *log, size_t logsz, size_t *code_size)
{
	char *code;
	size_t sz = 0;
	int rc = compile_code(src, &code, &sz, log, logsz);
	free(code);
	if (code_size)
		*code_size = rc ? 0 : sz;
	return rc;
}

/* Build both modules of a set (on the compile thread): e->fn NULL when the
 * standalone kernel failed (the interpreter keeps the set), e->fu[] NULL when
 * only the fused one did (two launches then). */
static void build_entry(const mosrx_bpf_insn *insns, const mosrx_bparams *t, struct mosrx_jit_entry *e, char *log,
                        size_t logsz)
{
	char *src = NULL, *hook = NULL;
	memset(e, 0, sizeof(*e));
	e->key = set_hash(insns, t);
	if (mosrx__bpf_jit_source(insns, t, &src) || compile_module(src, &e->mod, &e->fn, log, logsz)) {
		e->mod = NULL;
		e->fn = NULL;
		free(src);
		return;
	}
	free(src);
	if (mosrx__bpf_jit_hook_source(insns, t, &hook) || compile_fused(hook, &e->fmod, e->fu, log, logsz, NULL)) {
		e->fmod = NULL;
		memset(e->fu, 0, sizeof(e->fu));
	}
	free(hook);
}

static void entry_unload(struct mosrx_jit_entry *e)
{
	if (e->mod)
		hipModuleUnload(e->mod);
	if (e->fmod)
		hipModuleUnload(e->fmod);
	memset(e, 0, sizeof(*e));
}

/* ---- the context's compile thread ------------------------------------------
 * mosrx_bpf_set_async hands the set to it and returns; the thread compiles
 * (hipRTC) and loads (hipModuleLoadData) the set's kernels and leaves the
 * entry in `done`; the context's own thread takes finished entries into its
 * cache at its next launch or call (mosrx__bpf_poll) -- so the kernels in use
 * only ever change on the thread that launches them, between launches. */
#define WORKER_DONE 8
struct mosrx_bpf_worker {
	pthread_t th;
	pthread_mutex_t mu;
	pthread_cond_t cv;          /* work for the thread, or stop */
	pthread_cond_t done_cv;     /* a compile finished */
	int device, stop, started;
	int have_want;              /* `want` holds a set to compile */
	mosrx_bparams want_t;
	mosrx_bpf_insn *want_insns; /* MOSRX_BPF_MAX_INSNS */
	uint64_t want_key;
	int busy;                   /* compiling busy_key */
	uint64_t busy_key;
	struct mosrx_jit_entry done[WORKER_DONE];
	char done_log[WORKER_DONE][512];
	uint32_t ndone;
};

static void *worker_main(void *arg)
{
	struct mosrx_bpf_worker *w = arg;
	mosrx_bpf_insn *insns = malloc(MOSRX_BPF_MAX_INSNS * sizeof(*insns));
	hipSetDevice(w->device);
	pthread_mutex_lock(&w->mu);
	if (!insns)
		w->stop = 1;   /* no buffer to compile from: the thread is gone, its sets stay on the interpreter */
	for (;;) {
		struct mosrx_jit_entry e;
		mosrx_bparams t;
		char log[512];
		uint32_t total = 0, j;
		while (!w->stop && !w->have_want)
			pthread_cond_wait(&w->cv, &w->mu);
		if (w->stop || !insns)
			break;
		t = w->want_t;
		for (j = 0; j < t.nprog; j++)
			total += t.prog_len[j];
		memcpy(insns, w->want_insns, (size_t)total * sizeof(*insns));
		w->have_want = 0;
		w->busy = 1;
		w->busy_key = w->want_key;
		pthread_mutex_unlock(&w->mu);
		log[0] = 0;
		build_entry(insns, &t, &e, log, sizeof(log));
		pthread_mutex_lock(&w->mu);
		if (w->ndone == WORKER_DONE) {   /* nobody collected them: drop the oldest */
			entry_unload(&w->done[0]);
			memmove(&w->done[0], &w->done[1], sizeof(w->done[0]) * (WORKER_DONE - 1));
			memmove(&w->done_log[0], &w->done_log[1], sizeof(w->done_log[0]) * (WORKER_DONE - 1));
			w->ndone--;
		}
		w->done[w->ndone] = e;
		memcpy(w->done_log[w->ndone], log, sizeof(log));
		w->ndone++;
		w->busy = 0;
		pthread_cond_broadcast(&w->done_cv);
	}
	w->busy = 0;
	pthread_cond_broadcast(&w->done_cv);
	pthread_mutex_unlock(&w->mu);
	free(insns);
	return NULL;
}

static struct mosrx_bpf_worker *worker_get(mosrx_ctx *c)
{
	struct mosrx_bpf_worker *w = c->bw;
	if (w)
		return w;
	w = calloc(1, sizeof(*w));
	if (!w)
		return NULL;
	w->want_insns = malloc(MOSRX_BPF_MAX_INSNS * sizeof(*w->want_insns));
	w->device = c->device;
	pthread_mutex_init(&w->mu, NULL);
	pthread_cond_init(&w->cv, NULL);
	pthread_cond_init(&w->done_cv, NULL);
	if (!w->want_insns || pthread_create(&w->th, NULL, worker_main, w)) {
		free(w->want_insns);
		free(w);
		return NULL;
	}
	w->started = 1;
	c->bw = w;
	return w;
}


static void install(mosrx_ctx *c, const struct mosrx_jit_entry *e)
{
	c->bpf_fn = e ? e->fn : NULL;
	if (e && e->fn)
		memcpy(c->bpf_fu, e->fu, sizeof(c->bpf_fu));
	else
		memset(c->bpf_fu, 0, sizeof(c->bpf_fu));
}

/* Into the cache, evicting the oldest entry that is not the installed set's
 * (its kernels may be in use; launches still in flight -- on the context's
 * streams or a caller's -- are drained before a module goes, mosrx__drain). */
static void cache_put(mosrx_ctx *c, const struct mosrx_jit_entry *e)
{
	uint32_t i;
	for (i = 0; i < c->njit; i++)
		if (c->jit[i].key == e->key) {   /* compiled twice (a set re-requested while compiling) */
			struct mosrx_jit_entry dup = *e;
			entry_unload(&dup);
			return;
		}
	if (c->njit == MOSRX_BPF_JIT_CACHE) {
		uint32_t v = 0;
		while (v < c->njit && c->jit[v].key == c->bpf_key)
			v++;
		if (v == c->njit)
			v = 0;
		mosrx__drain(c);
		entry_unload(&c->jit[v]);
		memmove(&c->jit[v], &c->jit[v + 1], sizeof(c->jit[0]) * (MOSRX_BPF_JIT_CACHE - 1 - v));
		c->njit--;
	}
	c->jit[c->njit++] = *e;
}

static const struct mosrx_jit_entry *cache_find(const mosrx_ctx *c, uint64_t key)
{
	uint32_t i;
	for (i = 0; i < c->njit; i++)
		if (c->jit[i].key == key)
			return &c->jit[i];
	return NULL;
}

/* Take the compiles the thread finished into the cache.  On the context's own
 * thread only. */
static void collect(mosrx_ctx *c)
{
	struct mosrx_bpf_worker *w = c->bw;
	struct mosrx_jit_entry got[WORKER_DONE];
	char logs[WORKER_DONE][512];
	uint32_t i, n;
	if (!w)
		return;
	pthread_mutex_lock(&w->mu);
	n = w->ndone;
	memcpy(got, w->done, sizeof(got[0]) * n);
	memcpy(logs, w->done_log, sizeof(logs[0]) * n);
	w->ndone = 0;
	pthread_mutex_unlock(&w->mu);
	for (i = 0; i < n; i++) {
		cache_put(c, &got[i]);
		if (got[i].key == c->bpf_key) {
			memcpy(c->bpf_jit_log, logs[i], sizeof(c->bpf_jit_log));
			c->bpf_jit_log[sizeof(c->bpf_jit_log) - 1] = 0;
		}
	}
}

/* Install the installed set's compiled form once its compile is in (called
 * before every launch that runs the set). */
void mosrx__bpf_poll(mosrx_ctx *c)
{
	const struct mosrx_jit_entry *e;
	if (!c->bw || !c->bpf_pending)
		return;
	collect(c);
	if ((e = cache_find(c, c->bpf_key))) {
		install(c, e);
		c->bpf_pending = 0;
	}
}

/* The installed set (c->bpf, staged `insns`) gets its compiled form: from the
 * cache at once, else asynchronously (c->bpf_pending until mosrx__bpf_poll
 * installs it); the interpreter runs the set meanwhile.  0, or -errno when no
 * compile thread could be started (the interpreter keeps the set). */
int mosrx__bpf_jit_request(mosrx_ctx *c, const mosrx_bpf_insn *insns)
{
	const mosrx_bparams *t = &c->bpf;
	const struct mosrx_jit_entry *e;
	struct mosrx_bpf_worker *w;
	uint32_t j, total = 0;
	c->bpf_key = set_hash(insns, t);
	c->bpf_pending = 0;
	c->bpf_jit_log[0] = 0;
	install(c, NULL);
	collect(c);   /* compiles the thread finished (this set's among them, perhaps) */
	if ((e = cache_find(c, c->bpf_key))) {
		install(c, e);
		return 0;
	}
	if (!(w = worker_get(c)))
		return -EAGAIN;
	for (j = 0; j < t->nprog; j++)
		total += t->prog_len[j];
	pthread_mutex_lock(&w->mu);
	if (w->stop) {                                  /* the thread is gone: the interpreter keeps the set */
		pthread_mutex_unlock(&w->mu);
		return -EAGAIN;
	}
	if (!(w->busy && w->busy_key == c->bpf_key)) {   /* (being compiled already: wait for that one) */
		w->want_t = *t;
		w->want_key = c->bpf_key;
		memcpy(w->want_insns, insns, (size_t)total * sizeof(*insns));
		w->have_want = 1;
		pthread_cond_signal(&w->cv);
	}
	pthread_mutex_unlock(&w->mu);
	c->bpf_pending = 1;
	return 0;
}

/* Block until the installed set's compile is collected (or the thread has
 * nothing left for it: the interpreter stays). */
int mosrx__bpf_jit_wait(mosrx_ctx *c)
{
	struct mosrx_bpf_worker *w = c->bw;
	if (!w || !c->bpf_pending)
		return 0;
	for (;;) {
		uint32_t i;
		int found = 0, idle;
		pthread_mutex_lock(&w->mu);
		for (;;) {
			for (i = 0; i < w->ndone; i++)
				found |= w->done[i].key == c->bpf_key;
			idle = !w->busy && !w->have_want;
			if (found || idle || w->stop)
				break;
			pthread_cond_wait(&w->done_cv, &w->mu);
		}
		pthread_mutex_unlock(&w->mu);
		mosrx__bpf_poll(c);
		if (!c->bpf_pending)
			return 0;
		if (idle || w->stop) {   /* nothing for this set in flight: stay on the interpreter */
			c->bpf_pending = 0;
			return 0;
		}
	}
}

/* One launch of a hipRTC-built kernel, dispatch-stamped when the timing asks. */
static int module_launch(hipFunction_t f, unsigned grid, unsigned threads, hipStream_t s, void **args)
{
	void *e0, *e1;
	hipError_t rc;
	if (mosrx__stamp_take(&e0, &e1))
		rc = hipExtModuleLaunchKernel(f, grid * threads, 1, 1, threads, 1, 1, 0, s, args, NULL, (hipEvent_t)e0,
		                              (hipEvent_t)e1, 0);
	else
		rc = hipModuleLaunchKernel(f, grid, 1, 1, threads, 1, 1, 0, s, args, NULL);
	return rc == hipSuccess ? 0 : -EIO;
}

/* Fused classify + BPF launch (kp carries bmatch). */
int mosrx__bpf_fused_launch(mosrx_ctx *c, const mosrx_kparams *kp, int small, hipStream_t s)
{
	/* the library's tail policy: cached tail loads for batches of small frames */
	const int cached = !(mosrx__tail_variant(c, kp->frames_bytes, kp->n) & 2);
	hipFunction_t f = small ? c->bpf_fu[FU_M] : cached && c->bpf_fu[FU_SR] ? c->bpf_fu[FU_SR] : c->bpf_fu[FU_S];
	const unsigned tile = small ? MOSRX_KIND_FRAMES(MOSRX_KIND_SMALL) : MOSRX_KIND_FRAMES(MOSRX_KIND_S13);
	const unsigned threads = small ? 256u : 64u * (1u + MOSRX_STREAMERS);
	mosrx_kparams k = *kp;
	void *args[] = {&k};
	int rc;
	if (!f)
		return -EINVAL;
	rc = module_launch(f, (kp->n + tile - 1) / tile, threads, s, args);
	mosrx__note_stream(c, s);   /* (after the launch: its event covers it) */
	return rc;
}

/* The fused kernel over a batch queue (qp's descriptors carry the masks). */
int mosrx__bpf_fused_queue_launch(mosrx_ctx *c, const mosrx_qparams *qp, uint32_t total_tiles, int small,
                                  int variant, hipStream_t s)
{
	const int c8 = qp->tinfo == 2 ? FU_QS8 - FU_QS : 0;   /* 8-byte records: the _c8 forms */
	hipFunction_t f = small ? c->bpf_fu[FU_QM + c8]
	                        : !(variant & 2) && c->bpf_fu[FU_QSR + c8] ? c->bpf_fu[FU_QSR + c8] : c->bpf_fu[FU_QS + c8];
	const unsigned threads = small ? 256u : 64u * (1u + MOSRX_STREAMERS);
	const mosrx_qdesc *desc = qp->desc;
	uint32_t tpb = qp->tpb, nb = qp->nb;
	mosrx_qparams q = *qp;
	void *args[] = {&desc, &tpb, &nb, &q};
	if (!f)
		return -EINVAL;
	int rc;
	if (!total_tiles)
		return 0;
	rc = module_launch(f, total_tiles, threads, s, args);
	mosrx__note_stream(c, s);   /* (after the launch: its event covers it) */
	return rc;
}

int mosrx__bpf_jit_launch(mosrx_ctx *c, const mosrx_bparams *bp, hipStream_t s)
{
	const uint8_t *frames = bp->frames;
	const uint32_t *off = bp->off;
	const uint16_t *len = bp->len;
	uint32_t *match = bp->match;
	uint32_t nbytes = bp->frames_bytes, n = bp->n;
	void *args[] = {&frames, &off, &len, &match, &nbytes, &n};
	const unsigned grid = (n + 255u) / 256u;
	if (!c->bpf_fn)
		return -EINVAL;
	return module_launch(c->bpf_fn, grid, 256, s, args);
}

void mosrx__bpf_jit_free(mosrx_ctx *c)
{
	uint32_t i;
	struct mosrx_bpf_worker *w = c->bw;
	if (w) {
		pthread_mutex_lock(&w->mu);
		w->stop = 1;
		pthread_cond_broadcast(&w->cv);
		pthread_mutex_unlock(&w->mu);
		if (w->started)
			pthread_join(w->th, NULL);
		for (i = 0; i < w->ndone; i++)
			entry_unload(&w->done[i]);
		pthread_mutex_destroy(&w->mu);
		pthread_cond_destroy(&w->cv);
		pthread_cond_destroy(&w->done_cv);
		free(w->want_insns);
		free(w);
		c->bw = NULL;
	}
	for (i = 0; i < c->njit; i++)
		entry_unload(&c->jit[i]);
	c->njit = 0;
	c->bpf_pending = 0;
	install(c, NULL);
}
