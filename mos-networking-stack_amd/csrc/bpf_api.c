/*
 * bpf_api.c — host side of the batched BPF row (include/mosrx.h).
 *
 * mosrx_bpf_set is the GPU-side counterpart of SET_BPFFILTER (sfbpf.h:83):
 * mOS keeps compiling filter expressions with sfbpf_compile and hands the
 * resulting struct sfbpf_program here; the check below admits exactly the
 * programs sfbpf_filter (bpf/sf_bpf_filter.c:214-536) runs to a defined result.
 */
#include <errno.h>
#include <stdlib.h>
#include <string.h>

#include "mosrx_ctx.h"

enum {
	LD = 0, LDX = 1, ST = 2, STX = 3, ALU = 4, JMP = 5, RET = 6, MISC = 7,
	W = 0, H = 8, B = 0x10, IMM = 0, ABS = 0x20, IND = 0x40, MEM = 0x60, LEN = 0x80, MSH = 0xa0,
	ADD = 0, SUB = 0x10, MUL = 0x20, DIV = 0x30, OR = 0x40, AND = 0x50, LSH = 0x60, RSH = 0x70, NEG = 0x80,
	JA = 0, JEQ = 0x10, JGT = 0x20, JGE = 0x30, JSET = 0x40, K = 0, X = 8, A = 0x10, TAX = 0, TXA = 0x80,
	MEMWORDS = 16
};

/* sfbpf_validate (sf_bpf_filter.c:548-691) tightened to what sfbpf_filter can
 * execute on x86-64: only the opcodes of its switch (any other abort()s),
 * memory slots < 16, no constant division by zero (validate misses it: it
 * tests BPF_RVAL, :628, and the division traps), jump targets inside the
 * program in 64-bit arithmetic (pc += k moves a pointer forward), and a
 * return as the last instruction. */
int mosrx_bpf_check(const mosrx_bpf_insn *f, uint32_t len)
{
	uint32_t i;
	if (!f || len == 0 || len > MOSRX_BPF_MAX_INSNS)
		return -EINVAL;
	for (i = 0; i < len; i++) {
		const uint32_t k = f[i].k;
		const uint64_t from = (uint64_t)i + 1;
		switch (f[i].code) {
		case LD | W | ABS:
			/* sfbpf_filter keeps k in an int: k + sizeof(int32) wraps in size_t for
			 * k in [-4, -1] and the bounds check passes, reading before the frame
			 * (undefined); every other k >= 2^31 fails the check and returns 0 there
			 * as on the GPU (sf_bpf_filter.c:265-281) */
			if (k >= 0xFFFFFFFCu)
				return -EINVAL;
			break;
		case LD | H | ABS:   /* the same for k + sizeof(short), k in [-2, -1] (:283-299) */
			if (k >= 0xFFFFFFFEu)
				return -EINVAL;
			break;
		case RET | K: case RET | A:
		case LD | B | ABS: case LD | W | LEN: case LDX | W | LEN:
		case LD | W | IND: case LD | H | IND: case LD | B | IND: case LDX | MSH | B:
		case LD | IMM: case LDX | IMM:
		case ALU | ADD | X: case ALU | SUB | X: case ALU | MUL | X: case ALU | DIV | X: case ALU | AND | X:
		case ALU | OR | X: case ALU | LSH | X: case ALU | RSH | X:
		case ALU | ADD | K: case ALU | SUB | K: case ALU | MUL | K: case ALU | AND | K: case ALU | OR | K:
		case ALU | LSH | K: case ALU | RSH | K: case ALU | NEG:
		case MISC | TAX: case MISC | TXA:
			break;
		case ALU | DIV | K:
			if (k == 0)
				return -EINVAL;
			break;
		case LD | MEM: case LDX | MEM: case ST: case STX:
			if (k >= MEMWORDS)
				return -EINVAL;
			break;
		case JMP | JA:
			if (from + k >= len)
				return -EINVAL;
			break;
		case JMP | JGT | K: case JMP | JGE | K: case JMP | JEQ | K: case JMP | JSET | K:
		case JMP | JGT | X: case JMP | JGE | X: case JMP | JEQ | X: case JMP | JSET | X:
			if (from + f[i].jt >= len || from + f[i].jf >= len)
				return -EINVAL;
			break;
		default:
			return -EINVAL;
		}
	}
	return (f[len - 1].code & 7) == RET ? 0 : -EINVAL;
}

/* Program table + staged instructions of an admitted set. */
static int stage_set(const mosrx_bpf_prog *progs, uint32_t nprog, mosrx_bparams *tp, mosrx_bpf_insn *staged,
                     uint32_t *totalp)
{
	mosrx_bparams t;
	uint32_t j, total = 0;
	int rc;
	if (nprog > MOSRX_BPF_MAX_PROGS || (nprog && !progs))
		return -EINVAL;
	memset(&t, 0, sizeof(t));
	for (j = 0; j < nprog; j++) {
		const uint32_t len = progs[j].insns ? progs[j].len : 0;
		if (progs[j].len_mode != MOSRX_BPF_LEN_FRAME && progs[j].len_mode != MOSRX_BPF_LEN_IP)
			return -EINVAL;
		if (len && (rc = mosrx_bpf_check(progs[j].insns, len)))
			return rc;
		if (total + len > MOSRX_BPF_MAX_INSNS)
			return -E2BIG;
		if (len)
			memcpy(staged + total, progs[j].insns, (size_t)len * sizeof(mosrx_bpf_insn));
		t.prog_off[j] = (uint16_t)total;
		t.prog_len[j] = (uint16_t)len;
		if (progs[j].len_mode == MOSRX_BPF_LEN_IP)
			t.ip_mode |= 1u << j;
		total += len;
	}
	t.nprog = nprog;
	*tp = t;
	*totalp = total;
	return 0;
}

int mosrx_bpf_jit_source(const mosrx_bpf_prog *progs, uint32_t nprog, char **src)
{
	mosrx_bpf_insn *staged;
	mosrx_bparams t;
	uint32_t total;
	int rc;
	if (!src)
		return -EINVAL;
	*src = NULL;
	if (!(staged = malloc(MOSRX_BPF_MAX_INSNS * sizeof(*staged))))
		return -ENOMEM;
	if (!(rc = stage_set(progs, nprog, &t, staged, &total)))
		rc = mosrx__bpf_jit_source(staged, &t, src);
	free(staged);
	return rc;
}

int mosrx_bpf_jit_hook_source(const mosrx_bpf_prog *progs, uint32_t nprog, char **src)
{
	mosrx_bpf_insn *staged;
	mosrx_bparams t;
	uint32_t total;
	int rc;
	if (!src)
		return -EINVAL;
	*src = NULL;
	if (!(staged = malloc(MOSRX_BPF_MAX_INSNS * sizeof(*staged))))
		return -ENOMEM;
	if (!(rc = stage_set(progs, nprog, &t, staged, &total)))
		rc = mosrx__bpf_jit_hook_source(staged, &t, src);
	free(staged);
	return rc;
}

int mosrx_bpf_jit_compile(const mosrx_bpf_prog *progs, uint32_t nprog, char *log, size_t logsz,
                          size_t *code_size)
{
	char *src = NULL;
	int rc = mosrx_bpf_jit_source(progs, nprog, &src);
	if (!rc)
		rc = mosrx__bpf_jit_compile(src, log, logsz, code_size);
	free(src);
	return rc;
}

int mosrx_bpf_jit_compile_fused(const mosrx_bpf_prog *progs, uint32_t nprog, char *log, size_t logsz,
                                size_t *code_size)
{
	mosrx_bpf_insn *staged;
	mosrx_bparams t;
	uint32_t total;
	int rc;
	if (!(staged = malloc(MOSRX_BPF_MAX_INSNS * sizeof(*staged))))
		return -ENOMEM;
	if (!(rc = stage_set(progs, nprog, &t, staged, &total)))
		rc = mosrx__bpf_jit_compile_fused(staged, &t, log, logsz, code_size);
	free(staged);
	return rc;
}

int mosrx_bpf_fused(const mosrx_ctx *c)
{
	return c && c->bpf_fu[FU_S] && c->bpf_fu[FU_M] ? 1 : 0;
}

int mosrx_bpf_set_engine(mosrx_ctx *c, int engine)
{
	if (!c || (engine != MOSRX_BPF_ENGINE_INTERP && engine != MOSRX_BPF_ENGINE_JIT))
		return -EINVAL;
	c->bpf_engine_req = engine;
	return 0;
}

int mosrx_bpf_engine(const mosrx_ctx *c)
{
	if (!c)
		return -EINVAL;
	return c->bpf_fn ? MOSRX_BPF_ENGINE_JIT : MOSRX_BPF_ENGINE_INTERP;
}

const char *mosrx_bpf_jit_log(const mosrx_ctx *c)
{
	return c ? c->bpf_jit_log : "";
}

void mosrx__note_stream(mosrx_ctx *c, hipStream_t s)
{
	uint32_t k;
	if (s && s == c->stream)
		return;
	for (k = 0; k < NSLOT; k++)
		if (s && s == c->slot[k].stream)
			return;
	for (k = 0; k < c->nxs; k++)
		if (s && s == c->xs[k])
			return;
	/* a caller's stream (or the null stream): an event after the launch just made */
	for (k = 0; k < c->nfs && c->fstream[k] != s; k++)
		;
	if (k == c->nfs) {
		if (k == MOSRX_FOREIGN ||
		    (!c->fev[k] && hipEventCreateWithFlags(&c->fev[k], hipEventDisableTiming) != hipSuccess)) {
			c->foreign_streams = 1;   /* no room: the drain syncs the device */
			return;
		}
		c->fstream[k] = s;
		c->nfs++;
	}
	if (hipEventRecord(c->fev[k], s) != hipSuccess)
		c->foreign_streams = 1;
}

int mosrx__drain(mosrx_ctx *c)
{
	uint32_t k;
	HIPCHK(hipSetDevice(c->device));
	if (c->foreign_streams) {
		HIPCHK(hipDeviceSynchronize());
		c->foreign_streams = 0;
		c->nfs = 0;
		return 0;
	}
	for (k = 0; k < c->nfs; k++)
		HIPCHK(hipEventSynchronize(c->fev[k]));
	c->nfs = 0;
	HIPCHK(hipStreamSynchronize(c->stream));
	for (k = 0; k < NSLOT; k++)
		HIPCHK(hipStreamSynchronize(c->slot[k].stream));
	for (k = 0; k < c->nxs; k++)
		HIPCHK(hipStreamSynchronize(c->xs[k]));
	return 0;
}

/* The interpreter reads the installed instructions from device memory while
 * earlier launches may still be in flight (a group classified behind the rx
 * loop on the context's streams, or a caller's mosrx_bpf_dev /
 * mosrx_queue_run on its own stream), so each set goes to the next buffer of a
 * pool: a buffer is written again only after those launches drained
 * (mosrx__drain), and only if a launch may have read it since its last
 * write.  The compiled kernels carry their programs in their code. */
static int stage_insns(mosrx_ctx *c, const mosrx_bpf_insn *staged, uint32_t total)
{
	const uint32_t i = c->bpf_pool_next;
	int rc;
	if (!c->d_bpf_pool[i] &&
	    hipMalloc((void **)&c->d_bpf_pool[i], MOSRX_BPF_MAX_INSNS * sizeof(mosrx_bpf_insn)) != hipSuccess)
		return -ENOMEM;
	if (c->bpf_pool_used[i]) {
		if ((rc = mosrx__drain(c)))
			return rc;
		memset(c->bpf_pool_used, 0, sizeof(c->bpf_pool_used));
	}
	if (total)
		HIPCHK(hipMemcpy(c->d_bpf_pool[i], staged, (size_t)total * sizeof(mosrx_bpf_insn), hipMemcpyHostToDevice));
	c->d_bpf = c->d_bpf_pool[i];
	c->bpf_pool_next = (i + 1) % MOSRX_BPF_POOL;
	return 0;
}

int mosrx_bpf_set_async(mosrx_ctx *c, const mosrx_bpf_prog *progs, uint32_t nprog)
{
	mosrx_bparams t;
	mosrx_bpf_insn *staged;
	uint32_t total = 0;
	int rc;
	if (!c)
		return -EINVAL;
	if (!(staged = malloc(MOSRX_BPF_MAX_INSNS * sizeof(*staged))))
		return -ENOMEM;
	if ((rc = stage_set(progs, nprog, &t, staged, &total))) {
		free(staged);
		return rc;
	}
	if (hipSetDevice(c->device) != hipSuccess || (rc = stage_insns(c, staged, total))) {
		free(staged);
		return rc ? rc : -EIO;
	}
	c->bpf = t;
	c->bpf_fn = NULL;   /* the compiled kernels of the previous set no longer apply */
	memset(c->bpf_fu, 0, sizeof(c->bpf_fu));
	c->bpf_pending = 0;
	if (c->bpf_engine_req == MOSRX_BPF_ENGINE_JIT && nprog)
		mosrx__bpf_jit_request(c, staged);   /* cached: installed now; else compiled behind, interpreter meanwhile */
	free(staged);
	return 0;
}

int mosrx_bpf_wait(mosrx_ctx *c)
{
	if (!c)
		return -EINVAL;
	return mosrx__bpf_jit_wait(c);
}

int mosrx_bpf_pending(mosrx_ctx *c)
{
	if (!c)
		return -EINVAL;
	mosrx__bpf_poll(c);
	return c->bpf_pending;
}

int mosrx_bpf_set(mosrx_ctx *c, const mosrx_bpf_prog *progs, uint32_t nprog)
{
	int rc = mosrx_bpf_set_async(c, progs, nprog);
	return rc ? rc : mosrx_bpf_wait(c);
}

int mosrx__bpf_launch_dev(mosrx_ctx *c, const uint8_t *frames, uint64_t frames_bytes, const uint32_t *off,
                          const uint16_t *len, uint32_t n, uint32_t *match, hipStream_t s)
{
	mosrx_bparams bp = c->bpf;
	int rc;
	if (!n)
		return 0;
	mosrx__bpf_poll(c);
	bp.frames = frames;
	bp.off = off;
	bp.len = len;
	bp.match = match;
	bp.insns = c->d_bpf;
	bp.frames_bytes = (uint32_t)frames_bytes;
	bp.n = n;
	if (c->bpf_fn)
		rc = mosrx__bpf_jit_launch(c, &bp, s);
	else if (!c->d_bpf && bp.nprog)
		return -EINVAL;
	else {
		if (c->d_bpf)
			c->bpf_pool_used[(c->bpf_pool_next + MOSRX_BPF_POOL - 1) % MOSRX_BPF_POOL] = 1;
		rc = mosrx_launch_bpf(&bp, (void *)s);
	}
	mosrx__note_stream(c, s);   /* (after the launch: its event covers it) */
	return rc;
}

static int bpf_launch(mosrx_ctx *c, const mosrx_batch *b, const uint8_t *frames, const uint32_t *off,
                      const uint16_t *len, uint32_t *match, hipStream_t s)
{
	return mosrx__bpf_launch_dev(c, frames, b->frames_bytes, off, len, b->n, match, s);
}

int mosrx_bpf_dev(mosrx_ctx *c, const mosrx_batch *b, uint32_t *d_match, void *stream)
{
	int rc;
	if (!c || (rc = mosrx__check_batch(b, 1)))
		return c ? rc : -EINVAL;
	if (b->n == 0)
		return 0;
	if (!d_match || ((uintptr_t)d_match & 3))
		return -EINVAL;
	return bpf_launch(c, b, b->frames, b->off, b->len, d_match, stream ? (hipStream_t)stream : c->stream);
}

int mosrx_bpf_host(mosrx_ctx *c, const mosrx_batch *b, uint32_t *h_match)
{
	struct slot *s;
	int rc;
	if (!c || (rc = mosrx__check_batch(b, 0)))
		return c ? rc : -EINVAL;
	if (b->n == 0)
		return 0;
	if (!h_match)
		return -EINVAL;
	s = &c->slot[0];
	if (s->busy)
		return -EBUSY;
	HIPCHK(hipSetDevice(c->device));
	if ((rc = mosrx__slot_reserve(c, s, b->frames_bytes, b->n)))
		return rc;
	HIPCHK(hipMemcpyAsync(s->d_frames, b->frames, b->frames_bytes, hipMemcpyHostToDevice, s->stream));
	HIPCHK(hipMemcpyAsync(s->d_off, b->off, (size_t)b->n * 4, hipMemcpyHostToDevice, s->stream));
	HIPCHK(hipMemcpyAsync(s->d_len, b->len, (size_t)b->n * 2, hipMemcpyHostToDevice, s->stream));
	if ((rc = bpf_launch(c, b, s->d_frames, s->d_off, s->d_len, s->d_fh, s->stream)))
		return rc;
	HIPCHK(hipMemcpyAsync(h_match, s->d_fh, (size_t)b->n * 4, hipMemcpyDeviceToHost, s->stream));
	HIPCHK(hipStreamSynchronize(s->stream));
	return 0;
}
