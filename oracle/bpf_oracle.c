/*
 * bpf_oracle.c — TEST INFRASTRUCTURE ONLY (part of libmosrx_oracle.so).
 *
 * CPU restatement of mOS's classic-BPF interpreter and validator, the checker
 * for the batched BPF kernel.  Pinned against mOS's own
 * compiled core/src/bpf sources through oracle/_ref/mosbpf (tests/golden/bpf.npz).
 */
#include <string.h>

#include "mosrx_oracle.h"

/* BPF opcode fields (include/bpf/sfbpf.h) */
#define CLS(c)  ((c) & 0x07)
#define SIZE(c) ((c) & 0x18)
#define MODE(c) ((c) & 0xe0)
#define OP(c)   ((c) & 0xf0)
enum { LD = 0, LDX = 1, ST = 2, STX = 3, ALU = 4, JMP = 5, RET = 6, MISC = 7 };
enum { W = 0, H = 8, B = 0x10 };
enum { IMM = 0, ABS = 0x20, IND = 0x40, MEM = 0x60, LEN = 0x80, MSH = 0xa0 };
enum { ADD = 0, SUB = 0x10, MUL = 0x20, DIV = 0x30, OR = 0x40, AND = 0x50, LSH = 0x60, RSH = 0x70,
       NEG = 0x80 };
enum { JA = 0, JEQ = 0x10, JGT = 0x20, JGE = 0x30, JSET = 0x40 };
enum { K = 0, X_ = 8, A_ = 0x10 };
enum { TAX = 0, TXA = 0x80 };
#define MEMWORDS 16

static uint32_t be32(const uint8_t *p) { return (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3]; }
static uint32_t be16(const uint8_t *p) { return (uint32_t)p[0] << 8 | p[1]; }

/* sfbpf_filter, bpf/sf_bpf_filter.c:214-536 (user-space build).  `k` is an
 * int there: word/half bounds compare k + sizeof(..) as size_t (a negative k
 * is huge), byte bounds compare (u_int)k; both equal the u64 checks below.
 * Shift counts are masked to 5 bits as x86 does.  mem[] starts zeroed (the
 * reference leaves it uninitialised; compiled programs store before loading).
 * Returns 0 for an opcode the reference would abort() on (rejected at set). */
uint32_t mo_bpf_filter(const mosrx_bpf_insn *pc, const uint8_t *p, uint32_t wirelen, uint32_t buflen)
{
	uint32_t A = 0, X = 0, k;
	uint32_t mem[MEMWORDS];
	if (!pc)
		return ~0u;
	memset(mem, 0, sizeof(mem));
	for (;; pc++) {
		switch (pc->code) {
		case RET | K: return pc->k;
		case RET | A_: return A;
		case LD | W | ABS: k = pc->k; if ((uint64_t)k + 4 > buflen) return 0; A = be32(p + k); break;
		case LD | H | ABS: k = pc->k; if ((uint64_t)k + 2 > buflen) return 0; A = be16(p + k); break;
		case LD | B | ABS: k = pc->k; if (k >= buflen) return 0; A = p[k]; break;
		case LD | W | LEN: A = wirelen; break;
		case LDX | W | LEN: X = wirelen; break;
		case LD | W | IND: k = X + pc->k; if ((uint64_t)k + 4 > buflen) return 0; A = be32(p + k); break;
		case LD | H | IND: k = X + pc->k; if ((uint64_t)k + 2 > buflen) return 0; A = be16(p + k); break;
		case LD | B | IND: k = X + pc->k; if (k >= buflen) return 0; A = p[k]; break;
		case LDX | MSH | B: k = pc->k; if (k >= buflen) return 0; X = (uint32_t)(p[k] & 0xf) << 2; break;
		case LD | IMM: A = pc->k; break;
		case LDX | IMM: X = pc->k; break;
		case LD | MEM: A = mem[pc->k]; break;
		case LDX | MEM: X = mem[pc->k]; break;
		case ST: mem[pc->k] = A; break;
		case STX: mem[pc->k] = X; break;
		case JMP | JA: pc += pc->k; break;
		case JMP | JGT | K: pc += (A > pc->k) ? pc->jt : pc->jf; break;
		case JMP | JGE | K: pc += (A >= pc->k) ? pc->jt : pc->jf; break;
		case JMP | JEQ | K: pc += (A == pc->k) ? pc->jt : pc->jf; break;
		case JMP | JSET | K: pc += (A & pc->k) ? pc->jt : pc->jf; break;
		case JMP | JGT | X_: pc += (A > X) ? pc->jt : pc->jf; break;
		case JMP | JGE | X_: pc += (A >= X) ? pc->jt : pc->jf; break;
		case JMP | JEQ | X_: pc += (A == X) ? pc->jt : pc->jf; break;
		case JMP | JSET | X_: pc += (A & X) ? pc->jt : pc->jf; break;
		case ALU | ADD | X_: A += X; break;
		case ALU | SUB | X_: A -= X; break;
		case ALU | MUL | X_: A *= X; break;
		case ALU | DIV | X_: if (X == 0) return 0; A /= X; break;
		case ALU | AND | X_: A &= X; break;
		case ALU | OR | X_: A |= X; break;
		case ALU | LSH | X_: A <<= (X & 31); break;
		case ALU | RSH | X_: A >>= (X & 31); break;
		case ALU | ADD | K: A += pc->k; break;
		case ALU | SUB | K: A -= pc->k; break;
		case ALU | MUL | K: A *= pc->k; break;
		case ALU | DIV | K: A /= pc->k; break;
		case ALU | AND | K: A &= pc->k; break;
		case ALU | OR | K: A |= pc->k; break;
		case ALU | LSH | K: A <<= (pc->k & 31); break;
		case ALU | RSH | K: A >>= (pc->k & 31); break;
		case ALU | NEG: A = -A; break;
		case MISC | TAX: X = A; break;
		case MISC | TXA: A = X; break;
		default: return 0;
		}
	}
}

/* sfbpf_validate, bpf/sf_bpf_filter.c:548-691 (user-space build: no program
 * or packet-offset limits, jump targets checked in u_int arithmetic). */
int mo_bpf_validate(const mosrx_bpf_insn *f, int len)
{
	unsigned i, from;
	if (len < 1)
		return 0;
	for (i = 0; i < (unsigned)len; i++) {
		const mosrx_bpf_insn *p = &f[i];
		switch (CLS(p->code)) {
		case LD:
		case LDX:
			switch (MODE(p->code)) {
			case IMM: case ABS: case IND: case MSH: case LEN: break;
			case MEM: if (p->k >= MEMWORDS) return 0; break;
			default: return 0;
			}
			break;
		case ST:
		case STX:
			if (p->k >= MEMWORDS)
				return 0;
			break;
		case ALU:
			switch (OP(p->code)) {
			case ADD: case SUB: case MUL: case OR: case AND: case LSH: case RSH: case NEG: break;
			/* the reference tests BPF_RVAL (code & 0x18), which is never 0 for
			 * DIV, so a constant division by zero passes (and SIGFPEs at run) */
			case DIV: if ((p->code & 0x18) == K && p->k == 0) return 0; break;
			default: return 0;
			}
			break;
		case JMP:
			from = i + 1;
			switch (OP(p->code)) {
			case JA: if (from + p->k >= (unsigned)len) return 0; break;
			case JEQ: case JGT: case JGE: case JSET:
				if (from + p->jt >= (unsigned)len || from + p->jf >= (unsigned)len)
					return 0;
				break;
			default: return 0;
			}
			break;
		case RET:
		case MISC:
			break;
		default:
			return 0;
		}
	}
	return CLS(f[len - 1].code) == RET;
}

/* Length of frame i at a call site (MOSRX_BPF_LEN_*); 0 = not evaluated there. */
static uint32_t site_len(const uint8_t *frames, uint64_t frames_bytes, uint32_t off, uint16_t len, int mode,
                         int *eval)
{
	const uint8_t *f = frames + off;
	uint32_t cap = (off >= frames_bytes) ? 0 : (uint32_t)(frames_bytes - off < len ? frames_bytes - off : len);
	uint32_t lip = 0;
	if (cap >= 18 && f[12] == 0x08 && f[13] == 0x00) {
		lip = 14u + be16(f + 16);
		if (lip > cap)
			lip = 0;
	}
	*eval = mode != MOSRX_BPF_LEN_IP || lip != 0;
	return mode == MOSRX_BPF_LEN_IP ? lip : cap;
}

/* sfbpf_filter return value of one program on every frame (0 where not evaluated). */
int mo_bpf_returns(const mosrx_bpf_insn *insns, uint32_t ninsn, int len_mode, const uint8_t *frames,
                   uint64_t frames_bytes, const uint32_t *off, const uint16_t *len, uint32_t n, uint32_t *ret)
{
	uint32_t i;
	for (i = 0; i < n; i++) {
		int ev;
		uint32_t l = site_len(frames, frames_bytes, off[i], len[i], len_mode, &ev);
		ret[i] = ev ? mo_bpf_filter(ninsn ? insns : NULL, frames + off[i], l, l) : 0;
	}
	return 0;
}

/* Batch form: out[i] bit j = filter j matched frame i, with the lengths of
 * EVAL_BPFFILTER at each call site (see MOSRX_BPF_LEN_* in include/mosrx.h). */
int mo_bpf_eval(const mosrx_bpf_prog *progs, uint32_t nprog, const uint8_t *frames, uint64_t frames_bytes,
                const uint32_t *off, const uint16_t *len, uint32_t n, uint32_t *out)
{
	uint32_t i, j;
	if (nprog > MOSRX_BPF_MAX_PROGS)
		return -22;
	for (i = 0; i < n; i++) {
		uint32_t m = 0;
		for (j = 0; j < nprog; j++) {
			int ev;
			uint32_t l = site_len(frames, frames_bytes, off[i], len[i], progs[j].len_mode, &ev);
			if (ev && mo_bpf_filter(progs[j].len ? progs[j].insns : NULL, frames + off[i], l, l))
				m |= 1u << j;
		}
		out[i] = m;
	}
	return 0;
}
