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
 */
#include <errno.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "mosrx_ctx.h"
#include <hip/hiprtc.h>

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
	"static __device__ __attribute__((always_inline)) inline u32 fr_le32(const u32 *win, u32 sh, __amdgpu_buffer_rsrc_t rs, u32 o,\n"
	"                                              u32 k, u32 size) {\n"
	"  if (k + size <= STAGE_B) {\n"
	"    const u32 a = sh + k;\n"
	"    return __builtin_amdgcn_alignbyte(win[(a >> 2) + 1u], win[a >> 2], a & 3u);\n"
	"  }\n"
	"  return ld_le32(rs, o + k);\n"
	"}\n"
	"#define STAGE_W (4u * STAGE_V - 1u)\n"
	"/* little-endian dword of frame bytes [k, k+4), k constant, from the registers */\n"
	"#define W32(k) ((k) % 4u == 0u ? w[(k) / 4u] : __builtin_amdgcn_alignbyte(w[(k) / 4u + 1u], w[(k) / 4u], (k) % 4u))\n"
	"static __device__ __attribute__((always_inline)) inline u32 be32(u32 v) { return __builtin_bswap32(v); }\n"
	"static __device__ __attribute__((always_inline)) inline u32 be16(u32 v) { return ((v & 0xFFu) << 8) | ((v >> 8) & 0xFFu); }\n"
	"extern \"C\" __global__ __launch_bounds__(256) void mosrx_bpf_jit(const u8 *frames, const u32 *offs,\n"
	"    const u16 *lens, u32 *match_out, u32 nbytes, u32 n) {\n"
	"  __shared__ u32 s_win[STAGE_LD * 256];\n"
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
	"  u32 *win = s_win + STAGE_LD * t;\n"
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
	"      win[4 * m + 0] = v[m].x; win[4 * m + 1] = v[m].y; win[4 * m + 2] = v[m].z; win[4 * m + 3] = v[m].w;\n"
	"    }\n"
	"#pragma unroll\n"
	"    for (u32 i = 0; i < STAGE_W; i++) w[i] = __builtin_amdgcn_alignbyte(r[i + 1], r[i], sh);\n"
	"  }\n"
	"  if (cap >= 18u && (w[3] & 0xFFFFu) == 0x0008u) {\n"
	"    lip = 14u + be16(w[4]);\n"
	"    if (lip > cap) lip = 0;\n"
	"  }\n"
	"  u32 match = 0;\n";

/* bounds test "(u64)off + size > L" for a constant offset: 1 = always out of range */
static void gen_abs_check(struct sbuf *s, unsigned j, uint32_t k, uint32_t size)
{
	if ((uint64_t)k + size > 0xFFFFFFFFull)
		sb_printf(s, "goto P%u_R0; ", j);
	else
		sb_printf(s, "if (%uu > L) goto P%u_R0; ", (unsigned)(k + size), j);
}

/* How the generated program code reads frame bytes. */
struct genopt {
	int fused;          /* 0: standalone kernel (staged bytes); 1: classify header wave (its window) */
	uint32_t stage_w;   /* standalone: realigned staged dwords in w[] */
};

/* Constant-offset load expression.  Standalone: registers when frame bytes
 * [k, k + 8) are in w[], else the LDS stage / memory (fr_le32).  Fused: the
 * header window's realigned registers (frame bytes [2, 94)), else memory. */
static void gen_ld(struct sbuf *s, uint32_t k, uint32_t size, const struct genopt *g)
{
	if (g->fused) {
		if (k >= 2 && (uint64_t)k + 8 <= 94)
			sb_printf(s, "RW32(%uu)", k);
		else
			sb_printf(s, "hk_ld_le32(rs, o + %uu)", k);
	} else if ((uint64_t)k + 8 <= 4ull * g->stage_w) {
		sb_printf(s, "W32(%uu)", k);
	} else {
		sb_printf(s, "fr_le32(win, sh, rs, o, %uu, %uu)", k, size);
	}
}

/* Load at the run-time offset kk (X + k). */
static const char *ind_ld(const struct genopt *g, uint32_t size)
{
	if (g->fused)
		return size == 4 ? "hk_ind(kk, 4u)" : size == 2 ? "hk_ind(kk, 2u)" : "hk_ind(kk, 1u)";
	return size == 4 ? "fr_le32(win, sh, rs, o, kk, 4u)" : size == 2 ? "fr_le32(win, sh, rs, o, kk, 2u)"
	                                                          : "fr_le32(win, sh, rs, o, kk, 1u)";
}

static int gen_program(struct sbuf *s, unsigned j, const mosrx_bpf_insn *f, uint32_t len, int ipm,
                       const struct genopt *g)
{
	uint8_t *tgt, mem_used[16];
	uint32_t i, q;
	int need_r0 = 0;

	sb_printf(s, "  { /* program %u, %u insns, %s length */\n", j, (unsigned)len, ipm ? "datagram" : "frame");
	if (len == 0) {
		sb_printf(s, "    if (live%s) match |= %uu;\n  }\n", ipm ? " && lip != 0u" : "", 1u << j);
		return 0;
	}
	tgt = calloc(len + 1, 1);
	if (!tgt)
		return -ENOMEM;
	memset(mem_used, 0, sizeof(mem_used));
	for (i = 0; i < len; i++) {
		const uint16_t c = f[i].code;
		if ((c & 7) == JMP) {
			if (c == (JMP | JA)) {
				tgt[i + 1 + f[i].k] = 1;
			} else {
				tgt[i + 1 + f[i].jt] = 1;
				tgt[i + 1 + f[i].jf] = 1;
			}
		}
		if (c == (LD | MEM) || c == (LDX | MEM) || c == ST || c == STX)
			mem_used[f[i].k & 15] = 1;
		if (c == (LD | W | ABS) || c == (LD | H | ABS) || c == (LD | B | ABS) || c == (LD | W | IND) ||
		    c == (LD | H | IND) || c == (LD | B | IND) || c == (LDX | MSH | B) || c == (ALU | DIV | X))
			need_r0 = 1;
	}
	sb_printf(s, "    u32 A = 0, X = 0, ret = 0;\n");
	for (q = 0; q < 16; q++)
		if (mem_used[q])
			sb_printf(s, "    u32 M%u = 0;\n", q);
	sb_printf(s, "    const u32 L = %s;\n", ipm ? "lip" : "cap");
	sb_printf(s, "    if (!live%s) goto P%u_E;\n", ipm ? " || lip == 0u" : "", j);
	for (i = 0; i < len; i++) {
		const uint16_t c = f[i].code;
		const uint32_t k = f[i].k;
		const unsigned jt = i + 1 + f[i].jt, jf = i + 1 + f[i].jf;
		if (tgt[i])
			sb_printf(s, "  P%u_%u: ", j, (unsigned)i);
		else
			sb_printf(s, "    ");
		switch (c) {
		case RET | K: sb_printf(s, "ret = %uu; goto P%u_E;", k, j); break;
		case RET | A: sb_printf(s, "ret = A; goto P%u_E;", j); break;
		case LD | W | ABS:
			gen_abs_check(s, j, k, 4); sb_printf(s, "A = be32("); gen_ld(s, k, 4, g); sb_printf(s, ");");
			break;
		case LD | H | ABS:
			gen_abs_check(s, j, k, 2); sb_printf(s, "A = be16("); gen_ld(s, k, 2, g); sb_printf(s, ");");
			break;
		case LD | B | ABS:
			gen_abs_check(s, j, k, 1); sb_printf(s, "A = "); gen_ld(s, k, 1, g); sb_printf(s, " & 0xFFu;");
			break;
		case LD | W | LEN: sb_printf(s, "A = L;"); break;
		case LDX | W | LEN: sb_printf(s, "X = L;"); break;
		case LD | W | IND:
			sb_printf(s, "{ const u32 kk = X + %uu; if ((u64)kk + 4u > L) goto P%u_R0; A = be32(%s); }",
			          k, j, ind_ld(g, 4));
			break;
		case LD | H | IND:
			sb_printf(s, "{ const u32 kk = X + %uu; if ((u64)kk + 2u > L) goto P%u_R0; A = be16(%s); }",
			          k, j, ind_ld(g, 2));
			break;
		case LD | B | IND:
			sb_printf(s, "{ const u32 kk = X + %uu; if (kk >= L) goto P%u_R0; A = %s & 0xFFu; }",
			          k, j, ind_ld(g, 1));
			break;
		case LDX | MSH | B:
			gen_abs_check(s, j, k, 1);
			sb_printf(s, "X = ("); gen_ld(s, k, 1, g); sb_printf(s, " & 0xFu) << 2;");
			break;
		case LD | IMM: sb_printf(s, "A = %uu;", k); break;
		case LDX | IMM: sb_printf(s, "X = %uu;", k); break;
		case LD | MEM: sb_printf(s, "A = M%u;", k & 15); break;
		case LDX | MEM: sb_printf(s, "X = M%u;", k & 15); break;
		case ST: sb_printf(s, "M%u = A;", k & 15); break;
		case STX: sb_printf(s, "M%u = X;", k & 15); break;
		case JMP | JA: sb_printf(s, "goto P%u_%u;", j, (unsigned)(i + 1 + k)); break;
		case JMP | JGT | K: sb_printf(s, "if (A > %uu) goto P%u_%u; goto P%u_%u;", k, j, jt, j, jf); break;
		case JMP | JGE | K: sb_printf(s, "if (A >= %uu) goto P%u_%u; goto P%u_%u;", k, j, jt, j, jf); break;
		case JMP | JEQ | K: sb_printf(s, "if (A == %uu) goto P%u_%u; goto P%u_%u;", k, j, jt, j, jf); break;
		case JMP | JSET | K: sb_printf(s, "if (A & %uu) goto P%u_%u; goto P%u_%u;", k, j, jt, j, jf); break;
		case JMP | JGT | X: sb_printf(s, "if (A > X) goto P%u_%u; goto P%u_%u;", j, jt, j, jf); break;
		case JMP | JGE | X: sb_printf(s, "if (A >= X) goto P%u_%u; goto P%u_%u;", j, jt, j, jf); break;
		case JMP | JEQ | X: sb_printf(s, "if (A == X) goto P%u_%u; goto P%u_%u;", j, jt, j, jf); break;
		case JMP | JSET | X: sb_printf(s, "if (A & X) goto P%u_%u; goto P%u_%u;", j, jt, j, jf); break;
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
			free(tgt);
			return -EINVAL;
		}
		sb_printf(s, "\n");
	}
	if (need_r0)
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
 * offset the set loads, and 96 bytes (Ethernet + IP + TCP headers with
 * options) when a program loads at X + k; loads past the stage read memory. */
static uint32_t stage_pieces(const mosrx_bpf_insn *insns, const mosrx_bparams *t)
{
	uint64_t need = 18;   /* the datagram-length probe reads frame bytes 12..17 */
	uint32_t j, i;
	for (j = 0; j < t->nprog; j++)
		for (i = 0; i < t->prog_len[j]; i++) {
			const mosrx_bpf_insn *f = &insns[t->prog_off[j] + i];
			const uint16_t c = f->code;
			uint64_t end = 0;
			if (c == (LD | W | ABS)) end = (uint64_t)f->k + 4;
			else if (c == (LD | H | ABS)) end = (uint64_t)f->k + 2;
			else if (c == (LD | B | ABS) || c == (LDX | MSH | B)) end = (uint64_t)f->k + 1;
			else if (c == (LD | W | IND) || c == (LD | H | IND) || c == (LD | B | IND)) end = 96;
			if (end > need)
				need = end;
		}
	/* frame bytes [0, 16 V - 3) are staged whatever the start alignment */
	need = (need + 3 + 15) / 16;
	return need > 9 ? 9 : (uint32_t)need;
}

int mosrx__bpf_jit_source(const mosrx_bpf_insn *insns, const mosrx_bparams *t, char **out)
{
	struct sbuf s = {0};
	const uint32_t v = stage_pieces(insns, t);
	const struct genopt g = {0, 4 * v - 1};
	uint32_t j;
	int rc;
	*out = NULL;
	sb_printf(&s, "#define STAGE_V %uu\n#define STAGE_LD %uu\n#define STAGE_B %uu\n", v, 4 * v + 1, 16 * v - 3);
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
	"/* frame bytes [k, k+4), k constant in [2, 86]: the realigned window registers */\n"
	"#define RW32(k) (((k) - 2u) % 4u == 0u ? w[((k) - 2u) / 4u] \\\n"
	"                 : __builtin_amdgcn_alignbyte(w[((k) - 2u) / 4u + 1u], w[((k) - 2u) / 4u], ((k) - 2u) % 4u))\n"
	"/* frame bytes [kk, kk+4) at a run-time offset: the lane's LDS copy of the window, else memory */\n"
	"#define hk_ind(kk, size) (((kk) >= 2u && (kk) + (size) <= 94u) \\\n"
	"  ? __builtin_amdgcn_alignbyte(lw[(((kk) - 2u) >> 2) + 1u], lw[((kk) - 2u) >> 2], ((kk) - 2u) & 3u) \\\n"
	"  : hk_ld_le32(rs, o + (kk)))\n"
	"static __device__ __attribute__((always_inline)) inline u32 mosrx_bpf_hook(const hdr_win_t &win, u32 o, u32 cap,\n"
	"    bool live, __amdgpu_buffer_rsrc_t rs, u32 *lw) {\n"
	"  u32 w[WIN_DW];\n"
	"  const u32 rsh = (o + 2u) & 3u;\n"
	"#pragma unroll\n"
	"  for (int j = 0; j < WIN_DW; j++) w[j] = __builtin_amdgcn_alignbyte(win.raw[j + 1], win.raw[j], rsh);\n"
	"#pragma unroll\n"
	"  for (int j = 0; j < WIN_DW; j++) lw[j] = w[j];\n"
	"  lw[WIN_DW] = 0u;\n"
	"  u32 lip = 0;\n"
	"  if (cap >= 18u && be16hi(w[2]) == 0x0800u) {\n"
	"    lip = 14u + be16hi(w[3]);\n"
	"    if (lip > cap) lip = 0;\n"
	"  }\n"
	"  u32 match = 0;\n";

static const char k_fused_main[] =
	"#define MOSRX_RTC_BPF 1\n"
	"#include \"mosrx_kernels.hip\"\n"
	"extern \"C\" __global__ __launch_bounds__(WG_THREADS(MOSRX_KIND_S13)) void mosrx_classify_bpf_stream(mosrx_kparams kp)\n"
	"{ classify_tile<MOSRX_KIND_S13, 2 | VAR_BPF>(kp, blockIdx.x); }\n"
	"extern \"C\" __global__ __launch_bounds__(WG_THREADS(MOSRX_KIND_S13)) void mosrx_classify_bpf_stream_rt(mosrx_kparams kp)\n"
	"{ classify_tile<MOSRX_KIND_S13, VAR_BPF>(kp, blockIdx.x); }\n"
	"extern \"C\" __global__ __launch_bounds__(WG_THREADS(MOSRX_KIND_SMALL)) void mosrx_classify_bpf_small(mosrx_kparams kp)\n"
	"{ classify_tile<MOSRX_KIND_SMALL, 2 | VAR_BPF>(kp, blockIdx.x); }\n";

int mosrx__bpf_jit_hook_source(const mosrx_bpf_insn *insns, const mosrx_bparams *t, char **out)
{
	struct sbuf s = {0};
	const struct genopt g = {1, 0};
	uint32_t j;
	int rc;
	*out = NULL;
	sb_printf(&s, "/* generated by bpf_jit.c */\n%s", k_hook_pre);
	for (j = 0; j < t->nprog; j++)
		if ((rc = gen_program(&s, j, insns + t->prog_off[j], t->prog_len[j], (t->ip_mode >> j) & 1u, &g))) {
			free(s.p);
			return rc;
		}
	sb_printf(&s, "  return match;\n}\n#undef RW32\n#undef hk_ind\n");
	if (s.err) {
		free(s.p);
		return -ENOMEM;
	}
	*out = s.p;
	return 0;
}

/* hipRTC: source -> gfx950 code object (malloc'd into *code). */
static int compile_code_h(const char *src, int nh, const char *const *htexts, const char *const *hnames,
                          char **code, size_t *size, char *log, size_t logsz)
{
	hiprtcProgram prog;
	const char *opts[] = {"--offload-arch=gfx950", "-O3"};
	size_t sz = 0;
	int rc = 0;
	*code = NULL;
	if (hiprtcCreateProgram(&prog, src, "mosrx_bpf_jit.hip", nh, (const char **)htexts, (const char **)hnames) !=
	    HIPRTC_SUCCESS)
		return -EIO;
	if (hiprtcCompileProgram(prog, 2, opts) != HIPRTC_SUCCESS) {
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
		return -EIO;
	}
	if (hiprtcGetCodeSize(prog, &sz) != HIPRTC_SUCCESS || !sz || !(*code = malloc(sz)))
		rc = -EIO;
	else if (hiprtcGetCode(prog, *code) != HIPRTC_SUCCESS)
		rc = -EIO;
	hiprtcDestroyProgram(&prog);
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
static int compile_fused(const char *hook, hipModule_t *mod, hipFunction_t *fs, hipFunction_t *fm,
                         hipFunction_t *fr, char *log, size_t logsz, size_t *code_size)
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
	if (hipModuleLoadData(mod, code) != hipSuccess ||
	    hipModuleGetFunction(fs, *mod, "mosrx_classify_bpf_stream") != hipSuccess ||
	    hipModuleGetFunction(fr, *mod, "mosrx_classify_bpf_stream_rt") != hipSuccess ||
	    hipModuleGetFunction(fm, *mod, "mosrx_classify_bpf_small") != hipSuccess)
		rc = -EIO;
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
		rc = compile_fused(hook, NULL, NULL, NULL, NULL, log, logsz, code_size);
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

/* Install the compiled form of the set (c->bpf must already hold its table):
 * 0 with c->bpf_fn set, or -errno with the interpreter left in charge. */
int mosrx__bpf_jit_build(mosrx_ctx *c, const mosrx_bpf_insn *insns)
{
	const mosrx_bparams *t = &c->bpf;
	const uint64_t key = set_hash(insns, t);
	char *src = NULL;
	uint32_t i;
	int rc;
	c->bpf_fn = NULL;
	c->bpf_fs = NULL;
	c->bpf_fm = NULL;
	c->bpf_fr = NULL;
	c->bpf_jit_log[0] = 0;
	for (i = 0; i < c->njit; i++)
		if (c->jit[i].key == key) {
			c->bpf_fn = c->jit[i].fn;
			c->bpf_fs = c->jit[i].fs;
			c->bpf_fm = c->jit[i].fm;
			c->bpf_fr = c->jit[i].fr;
			return 0;
		}
	if ((rc = mosrx__bpf_jit_source(insns, t, &src)))
		return rc;
	{
		hipModule_t mod;
		hipFunction_t fn;
		rc = compile_module(src, &mod, &fn, c->bpf_jit_log, sizeof(c->bpf_jit_log));
		free(src);
		if (rc)
			return rc;
		hipModule_t fmod = NULL;
		hipFunction_t fs = NULL, fm = NULL, fr = NULL;
		char *hook = NULL;
		if (mosrx__bpf_jit_hook_source(insns, t, &hook) ||
		    compile_fused(hook, &fmod, &fs, &fm, &fr, c->bpf_jit_log, sizeof(c->bpf_jit_log), NULL)) {
			fmod = NULL;   /* no fused kernel: mosrx_classify_bpf_dev runs two launches */
			fs = fm = fr = NULL;
		}
		free(hook);
		if (c->njit == MOSRX_BPF_JIT_CACHE) {   /* evict the oldest */
			hipModuleUnload(c->jit[0].mod);
			if (c->jit[0].fmod)
				hipModuleUnload(c->jit[0].fmod);
			memmove(&c->jit[0], &c->jit[1], sizeof(c->jit[0]) * (MOSRX_BPF_JIT_CACHE - 1));
			c->njit--;
		}
		c->jit[c->njit].key = key;
		c->jit[c->njit].mod = mod;
		c->jit[c->njit].fn = fn;
		c->jit[c->njit].fmod = fmod;
		c->jit[c->njit].fs = fs;
		c->jit[c->njit].fm = fm;
		c->jit[c->njit].fr = fr;
		c->njit++;
		c->bpf_fn = fn;
		c->bpf_fs = fs;
		c->bpf_fm = fm;
		c->bpf_fr = fr;
	}
	return 0;
}

/* Fused classify + BPF launch (kp carries bmatch). */
int mosrx__bpf_fused_launch(mosrx_ctx *c, const mosrx_kparams *kp, int small, hipStream_t s)
{
	/* the library's tail policy: cached tail loads for batches of small frames */
	const int cached = !(mosrx__tail_variant(c, kp->frames_bytes, kp->n) & 2);
	hipFunction_t f = small ? c->bpf_fm : cached && c->bpf_fr ? c->bpf_fr : c->bpf_fs;
	const unsigned tile = small ? MOSRX_KIND_FRAMES(MOSRX_KIND_SMALL) : MOSRX_KIND_FRAMES(MOSRX_KIND_S13);
	const unsigned threads = small ? 256u : 64u * (1u + MOSRX_STREAMERS);
	mosrx_kparams k = *kp;
	void *args[] = {&k};
	if (!f)
		return -EINVAL;
	if (hipModuleLaunchKernel(f, (kp->n + tile - 1) / tile, 1, 1, threads, 1, 1, 0, s, args, NULL) != hipSuccess)
		return -EIO;
	return 0;
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
	if (hipModuleLaunchKernel(c->bpf_fn, grid, 1, 1, 256, 1, 1, 0, s, args, NULL) != hipSuccess)
		return -EIO;
	return 0;
}

void mosrx__bpf_jit_free(mosrx_ctx *c)
{
	uint32_t i;
	for (i = 0; i < c->njit; i++) {
		hipModuleUnload(c->jit[i].mod);
		if (c->jit[i].fmod)
			hipModuleUnload(c->jit[i].fmod);
	}
	c->njit = 0;
	c->bpf_fn = NULL;
	c->bpf_fs = NULL;
	c->bpf_fm = NULL;
	c->bpf_fr = NULL;
}
