/*
 * gpu_emul.c — TEST INFRASTRUCTURE ONLY (tests/test_mos_consumer.py, CPU leg).
 *
 * Stands in for the GPU under gpu_module_func in a container with no GPU:
 * linked into oracle/_ref/mos_app_emul with -Wl,--wrap for each libmosrx call
 * the module makes, it produces the records (and BPF match masks) with the
 * oracle's C restatement (mosrx_oracle.c, bpf_oracle.c) at submit time.  It
 * lets the CPU suite check the host logic above the kernels -- the backend's
 * grouping / reclassification and the mOS-side consumer (csrc/mos_rx.c)
 * against mOS's own ProcessPacket -- while the -m gpu test runs the same
 * program with the real kernels.  Never part of a product build.
 */
#include <errno.h>
#include <stdlib.h>
#include <string.h>

#include "mosrx_oracle.h"

struct emul_ctx {
	mosrx_params p;
	mosrx_bpf_prog progs[MOSRX_BPF_MAX_PROGS];
	mosrx_bpf_insn *insns[MOSRX_BPF_MAX_PROGS];
	uint32_t nprog;
};

static int emul_gpus(void)
{
	const char *e = getenv("MOSRX_EMUL_NDEV");
	return e ? atoi(e) : 1;
}

int __wrap_mosrx_device_count(void) { return emul_gpus(); }

int __wrap_mosrx_open(int device, const mosrx_params *p, mosrx_ctx **out)
{
	struct emul_ctx *c;
	if (device < 0 || device >= emul_gpus() || !p)
		return -ENODEV;
	c = calloc(1, sizeof(*c));
	if (!c)
		return -ENOMEM;
	c->p = *p;
	*out = (mosrx_ctx *)c;
	return 0;
}

static void drop_progs(struct emul_ctx *c)
{
	uint32_t i;
	for (i = 0; i < c->nprog; i++)
		free(c->insns[i]);
	c->nprog = 0;
}

void __wrap_mosrx_close(mosrx_ctx *mc)
{
	struct emul_ctx *c = (struct emul_ctx *)mc;
	if (c)
		drop_progs(c);
	free(c);
}

int __wrap_mosrx_set_params(mosrx_ctx *mc, const mosrx_params *p)
{
	((struct emul_ctx *)mc)->p = *p;
	return 0;
}

int __wrap_mosrx_set_timing(mosrx_ctx *mc, int on) { (void)mc; (void)on; return 0; }
int __wrap_mosrx_last_kernel_ms(mosrx_ctx *mc, float *ms) { (void)mc; (void)ms; return -ENODATA; }
int __wrap_mosrx_host_alloc(mosrx_ctx *mc, size_t bytes, void **p)
{
	(void)mc;
	*p = calloc(1, bytes ? bytes : 1);
	return *p ? 0 : -ENOMEM;
}
int __wrap_mosrx_host_free(mosrx_ctx *mc, void *p) { (void)mc; free(p); return 0; }
int __wrap_mosrx_classify_host_wait(mosrx_ctx *mc, int slot) { (void)mc; (void)slot; return 0; }
int __wrap_mosrx_classify_host_ready(mosrx_ctx *mc, int slot) { (void)mc; (void)slot; return 1; }
int __wrap_mosrx_set_counters(mosrx_ctx *mc, int on) { (void)mc; (void)on; return 0; }
int __wrap_mosrx_classify_host_reserve(mosrx_ctx *mc, uint64_t fb, uint32_t n) { (void)mc; (void)fb; (void)n; return 0; }
int __wrap_mosrx_set_direct(mosrx_ctx *mc, uint64_t max_bytes, uint32_t max_frames)
{
	(void)mc; (void)max_bytes; (void)max_frames;
	return 0;
}
int __wrap_mosrx_slot_direct(mosrx_ctx *mc, int slot) { (void)mc; (void)slot; return 0; }

int __wrap_mosrx_bpf_set(mosrx_ctx *mc, const mosrx_bpf_prog *progs, uint32_t nprog)
{
	struct emul_ctx *c = (struct emul_ctx *)mc;
	uint32_t i;
	if (nprog > MOSRX_BPF_MAX_PROGS)
		return -EINVAL;
	for (i = 0; i < nprog; i++)
		if (progs[i].len && mo_bpf_validate(progs[i].insns, (int)progs[i].len) != 1)
			return -EINVAL;
	drop_progs(c);
	for (i = 0; i < nprog; i++) {
		c->progs[i] = progs[i];
		c->insns[i] = NULL;
		if (progs[i].len) {
			c->insns[i] = malloc(progs[i].len * sizeof(mosrx_bpf_insn));
			if (!c->insns[i])
				return -ENOMEM;
			memcpy(c->insns[i], progs[i].insns, progs[i].len * sizeof(mosrx_bpf_insn));
			c->progs[i].insns = c->insns[i];
		}
	}
	c->nprog = nprog;
	return 0;
}

/* The set is in effect at once (the interpreter's results = the compiled ones). */
int __wrap_mosrx_bpf_set_async(mosrx_ctx *mc, const mosrx_bpf_prog *progs, uint32_t nprog)
{
	return __wrap_mosrx_bpf_set(mc, progs, nprog);
}

int __wrap_mosrx_classify_host_submit_ex(mosrx_ctx *mc, int slot, const mosrx_batch *b, mosrx_result *out,
                                         mosrx_tcpinfo *ti)
{
	struct emul_ctx *c = (struct emul_ctx *)mc;
	(void)slot;
	return mo_classify_ex(&c->p, b->frames, b->frames_bytes, b->off, b->len, b->n, out, NULL, ti);
}

int __wrap_mosrx_classify_host_group_submit(mosrx_ctx *mc, int slot, const mosrx_batch *b, uint32_t nb,
                                            mosrx_result *const *out, mosrx_tcpinfo *const *ti)
{
	uint32_t i;
	int rc;
	for (i = 0; i < nb; i++)
		if ((rc = __wrap_mosrx_classify_host_submit_ex(mc, slot, &b[i], out[i], ti ? ti[i] : NULL)))
			return rc;
	return 0;
}

int __wrap_mosrx_classify_host_group_submit_ex(mosrx_ctx *mc, int slot, const mosrx_batch *b, uint32_t nb,
                                               mosrx_result *const *out, mosrx_tcpinfo *const *ti,
                                               uint32_t *const *fh)
{
	struct emul_ctx *c = (struct emul_ctx *)mc;
	uint32_t i;
	int rc;
	(void)slot;
	for (i = 0; i < nb; i++)
		if ((rc = mo_classify_ex(&c->p, b[i].frames, b[i].frames_bytes, b[i].off, b[i].len, b[i].n, out[i],
		                         fh ? fh[i] : NULL, ti ? ti[i] : NULL)))
			return rc;
	return 0;
}

/* 8-byte records (gpu_module_func cfg.compact): the oracle's 16-byte record projected
 * onto mosrx_result8's fields, and the flow hashes when asked for */
int __wrap_mosrx_classify_host_group_submit_c8(mosrx_ctx *mc, int slot, const mosrx_batch *b, uint32_t nb,
                                               mosrx_result8 *const *out8, uint32_t *const *fh)
{
	struct emul_ctx *c = (struct emul_ctx *)mc;
	uint32_t i, k;
	int rc = 0;
	(void)slot;
	for (i = 0; i < nb && !rc; i++) {
		mosrx_result *r = malloc((size_t)(b[i].n ? b[i].n : 1) * sizeof(*r));
		if (!r)
			return -ENOMEM;
		rc = mo_classify_ex(&c->p, b[i].frames, b[i].frames_bytes, b[i].off, b[i].len, b[i].n, r,
		                    fh ? fh[i] : NULL, NULL);
		for (k = 0; !rc && k < b[i].n; k++) {
			out8[i][k].rss = r[k].rss;
			out8[i][k].reason = r[k].reason;
			out8[i][k].queue = r[k].queue;
			out8[i][k].verdict = r[k].verdict;
			out8[i][k].tcp_flags = r[k].tcp_flags;
		}
		free(r);
	}
	return rc;
}

int __wrap_mosrx_classify_host_group_submit_bpf_c8(mosrx_ctx *mc, int slot, const mosrx_batch *b, uint32_t nb,
                                                   mosrx_result8 *const *out8, uint32_t *const *fh,
                                                   uint32_t *const *match)
{
	struct emul_ctx *c = (struct emul_ctx *)mc;
	uint32_t i;
	int rc = __wrap_mosrx_classify_host_group_submit_c8(mc, slot, b, nb, out8, fh);
	for (i = 0; i < nb && !rc; i++)
		rc = mo_bpf_eval(c->progs, c->nprog, b[i].frames, b[i].frames_bytes, b[i].off, b[i].len, b[i].n, match[i]);
	return rc;
}

int __wrap_mosrx_classify_bpf_host_submit(mosrx_ctx *mc, int slot, const mosrx_batch *b, mosrx_result *out,
                                          uint32_t *match)
{
	struct emul_ctx *c = (struct emul_ctx *)mc;
	int rc = __wrap_mosrx_classify_host_submit_ex(mc, slot, b, out, NULL);
	if (rc)
		return rc;
	return mo_bpf_eval(c->progs, c->nprog, b->frames, b->frames_bytes, b->off, b->len, b->n, match);
}

int __wrap_mosrx_classify_host_group_submit_bpf(mosrx_ctx *mc, int slot, const mosrx_batch *b, uint32_t nb,
                                                mosrx_result *const *out, uint32_t *const *fh,
                                                uint32_t *const *match)
{
	struct emul_ctx *c = (struct emul_ctx *)mc;
	uint32_t i;
	int rc;
	(void)slot;
	for (i = 0; i < nb; i++)
		if ((rc = mo_classify_ex(&c->p, b[i].frames, b[i].frames_bytes, b[i].off, b[i].len, b[i].n, out[i],
		                         fh ? fh[i] : NULL, NULL)) ||
		    (rc = mo_bpf_eval(c->progs, c->nprog, b[i].frames, b[i].frames_bytes, b[i].off, b[i].len, b[i].n,
		                      match[i])))
			return rc;
	return 0;
}

/* The TX rewrite (mosrx_tx_csum_host): the oracle's restatement, in place. */
int __wrap_mosrx_tx_csum_host(mosrx_ctx *mc, const mosrx_batch *b, int flags)
{
	(void)mc;
	return mo_tx_csum((uint8_t *)b->frames, b->frames_bytes, b->off, b->len, b->n, flags);
}
