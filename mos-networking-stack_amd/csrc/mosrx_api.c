/*
 * mosrx_api.c — C host side of the MI355X rx classifier (include/mosrx.h).
 *
 * Plain C over the HIP runtime API.  It owns the per-context device state
 * (lookup tables, staging for the end-to-end path, the stream) and enqueues the
 * kernels in mosrx_kernels.hip.  There is no CPU fallback: without a usable GPU
 * mosrx_open() fails with -ENODEV.
 */
#include <errno.h>
#include <stdlib.h>
#include <string.h>

#include "mosrx_ctx.h"
#include "mosrx_source.h"

#include <pthread.h>

/* Default cache policy per access class (bit 0: header windows non-temporal,
 * bit 1: tail stream non-temporal), chosen from measurements on MI355X. */
#define MOSRX_DEFAULT_VARIANT 2   /* tails nt, windows default: scripts/tune.py, profiles/r01_tune_variants.log */

int mosrx_set_variant(mosrx_ctx *c, int variant)
{
	if (!c || variant < 0 || variant > 127)
		return -EINVAL;
	c->variant = variant;
	return 0;
}

int mosrx_abi_version(void) { return MOSRX_ABI_VERSION; }

const char *mosrx_strerror(int err)
{
	switch (err) {
	case 0: return "success";
	case -EINVAL: return "invalid argument";
	case -ENODEV: return "no usable gfx950 device / HIP runtime";
	case -ENOMEM: return "out of memory";
	case -EIO: return "HIP runtime error";
	case -E2BIG: return "batch too large";
	default: return "unknown error";
	}
}

void mosrx_params_default(mosrx_params *p)
{
	memset(p, 0, sizeof(*p));
	p->num_msp = 1;           /* simple_firewall opens one MONITOR_STREAM socket (socket.c:77-78) */
	p->num_esp = 0;
	p->forward = 1;           /* setup.sh:135 */
	p->num_queues = 1;        /* pcap_module.c:159 */
	p->queue_mode = MOSRX_QMAP_I40E;   /* FetchEndianType() without DPDK, config.c:1277 */
	p->skip_tcp_csum = 0;
	p->rss_key_len = 40;      /* util.c:36-42 */
	memset(p->rss_key, 0x05, 40);
}

void mosrx_params_set_ms_key(mosrx_params *p)
{
	static const uint8_t ms[40] = {
		0x6d, 0x5a, 0x56, 0xda, 0x25, 0x5b, 0x0e, 0xc2, 0x41, 0x67, 0x25, 0x3d, 0x43, 0xa3,
		0x8f, 0xb0, 0xd0, 0xca, 0x2b, 0xcb, 0xae, 0x7b, 0x30, 0xb4, 0x77, 0xcb, 0x2d, 0xa3,
		0x80, 0x30, 0xf2, 0x0c, 0x6a, 0x42, 0xb7, 0x3b, 0xbe, 0xac, 0x01, 0xfa};
	memset(p->rss_key, 0, sizeof(p->rss_key));
	memcpy(p->rss_key, ms, sizeof(ms));
	p->rss_key_len = sizeof(ms);
}

/* Key cache of BuildKeyCache (util.c:27-58): cache[i] = the 32 key bits starting
 * at bit i.  The 96-bit input bit i (MSB-first over saddr|daddr|sport|dport)
 * contributes cache[i]; grouping input bits by nibble gives 24 tables of 16. */
int mosrx_rss_tables(const uint8_t *key, uint32_t key_len, uint32_t tables[24 * 16])
{
	uint32_t cache[96];
	uint32_t result, idx = 32;
	int i, k, v, b;

	if (!key || !tables || key_len < 16)
		return -EINVAL;
	result = ((uint32_t)key[0] << 24) | ((uint32_t)key[1] << 16) | ((uint32_t)key[2] << 8) | key[3];
	for (i = 0; i < 96; i++, idx++) {
		cache[i] = result;
		result = (result << 1) | (((key[idx / 8] << (idx % 8)) & 0x80) ? 1u : 0u);
	}
	for (k = 0; k < 24; k++)
		for (v = 0; v < 16; v++) {
			uint32_t h = 0;
			for (b = 0; b < 4; b++)
				if (v & (8 >> b))
					h ^= cache[4 * k + b];
			tables[k * 16 + v] = h;
		}
	return 0;
}

static int check_params(const mosrx_params *p)
{
	if (!p || p->rss_key_len < 16 || p->rss_key_len > MOSRX_RSS_KEY_MAX)
		return -EINVAL;
	if (p->num_queues < 1 || p->num_queues > 256)
		return -EINVAL;
	if (p->queue_mode != MOSRX_QMAP_I40E && p->queue_mode != MOSRX_QMAP_IXGBE)
		return -EINVAL;
	if (p->num_local > MOSRX_MAX_LOCAL)
		return -EINVAL;
	return 0;
}

/* GetRSSCPUCore (util.c:114-131) evaluated for every (hash & 0x1FF). */
static void build_qlut(const mosrx_params *p, uint8_t lut[512])
{
	static const uint32_t offs[4] = {3, 1, (uint32_t)-1, (uint32_t)-3};
	uint32_t x;
	for (x = 0; x < 512; x++) {
		uint32_t m;
		if (p->queue_mode == MOSRX_QMAP_I40E) {
			m = x & 0x1FF;
			m += offs[m & 3];
		} else {
			m = x & 0x7F;
		}
		lut[x] = (uint8_t)(m % (uint32_t)p->num_queues);
	}
}

int mosrx_set_params(mosrx_ctx *c, const mosrx_params *p)
{
	uint32_t tab[MOSRX_TAB_ALLOC_WORDS];
	int rc;

	if (!c)
		return -EINVAL;
	if ((rc = check_params(p)))
		return rc;
	memset(tab, 0, sizeof(tab));
	if ((rc = mosrx_rss_tables(p->rss_key, p->rss_key_len, tab)))
		return rc;
	build_qlut(p, (uint8_t *)(tab + MOSRX_TAB_RSS_WORDS));
	tab[MOSRX_TAB_LOCAL] = p->num_local;
	memcpy(tab + MOSRX_TAB_LOCAL + 1, p->local_ip, sizeof(p->local_ip));
	HIPCHK(hipSetDevice(c->device));
	HIPCHK(hipMemcpyAsync(c->d_tables, tab, sizeof(tab), hipMemcpyHostToDevice, c->stream));
	HIPCHK(hipStreamSynchronize(c->stream));
	c->params = *p;
	c->kflags = ((p->num_msp || p->num_esp) ? MOSRX_KF_VERIFY : 0) |
	            ((p->num_msp && p->forward) ? MOSRX_KF_FWD_NONIP : 0) |
	            (p->skip_tcp_csum ? MOSRX_KF_SKIP_TCP : 0);
	return 0;
}

int mosrx__ensure_streams(mosrx_ctx *c, uint32_t n);

int mosrx_device_count(void)
{
	int n = 0;
	return hipGetDeviceCount(&n) == hipSuccess ? n : 0;
}

int mosrx_open(int device, const mosrx_params *p, mosrx_ctx **out)
{
	mosrx_ctx *c;
	int ndev = 0, rc, i;
	hipDeviceProp_t prop;

	if (!out)
		return -EINVAL;
	*out = NULL;
	if ((rc = check_params(p)))
		return rc;
	if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev)
		return -ENODEV;
	if (hipGetDeviceProperties(&prop, device) != hipSuccess || strncmp(prop.gcnArchName, "gfx950", 6))
		return -ENODEV;
	c = calloc(1, sizeof(*c));
	if (!c)
		return -ENOMEM;
	c->device = device;
	c->variant = MOSRX_DEFAULT_VARIANT;
	c->last_kernel_ms = -1.0f;
	if (getenv("MOSRX_KVARIANT"))
		c->variant = atoi(getenv("MOSRX_KVARIANT")) & 127;
	c->bpf_engine_req = MOSRX_BPF_ENGINE_JIT;
	if (getenv("MOSRX_BPF_ENGINE") && atoi(getenv("MOSRX_BPF_ENGINE")) == 0)
		c->bpf_engine_req = MOSRX_BPF_ENGINE_INTERP;
	/* the timing streams are created right after the context stream: HIP maps
	 * streams to hardware queues round robin (GPU_MAX_HW_QUEUES, 4 by default),
	 * so the first three land on queues of their own */
	if (hipSetDevice(device) != hipSuccess ||
	    hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
	    mosrx__ensure_streams(c, 3) != 0 ||
	    hipMalloc((void **)&c->d_tables, MOSRX_TAB_ALLOC_WORDS * 4) != hipSuccess ||
	    hipEventCreate(&c->ev0) != hipSuccess || hipEventCreate(&c->ev1) != hipSuccess) {
		mosrx_close(c);
		return -ENODEV;
	}
	for (i = 0; i < NSLOT; i++) {
		if (hipStreamCreateWithFlags(&c->slot[i].stream, hipStreamNonBlocking) != hipSuccess ||
		    hipEventCreateWithFlags(&c->slot[i].done, hipEventDisableTiming) != hipSuccess ||
		    hipEventCreate(&c->slot[i].kev0) != hipSuccess || hipEventCreate(&c->slot[i].kev1) != hipSuccess ||
		    hipMalloc((void **)&c->slot[i].d_qdesc, MOSRX_MAX_GROUP * sizeof(mosrx_qdesc)) != hipSuccess ||
		    hipHostMalloc((void **)&c->slot[i].h_qdesc, MOSRX_MAX_GROUP * sizeof(mosrx_qdesc),
		                  hipHostMallocDefault) != hipSuccess ||
		    hipMalloc((void **)&c->slot[i].d_cnt, MOSRX_CNT_WORDS * 4) != hipSuccess ||
		    hipHostMalloc((void **)&c->slot[i].h_cnt, MOSRX_CNT_WORDS * 4, hipHostMallocDefault) != hipSuccess ||
		    !(c->slot[i].h_prev = calloc(MOSRX_CNT_WORDS, 4))) {
			mosrx_close(c);
			return -ENODEV;
		}
		c->slot[i].cnt_dirty = 1;   /* the first launch on the slot zeroes its counters */
		{
			void *d = NULL;
			if (hipHostGetDevicePointer(&d, c->slot[i].h_qdesc, 0) == hipSuccess)
				c->slot[i].hq_dev = (const mosrx_qdesc *)d;
		}
	}
	if ((rc = mosrx_set_params(c, p))) {
		mosrx_close(c);
		return rc;
	}
	*out = c;
	return 0;
}

static void slot_free(struct slot *s)
{
	if (s->d_frames) hipFree(s->d_frames);
	if (s->d_off) hipFree(s->d_off);
	if (s->d_len) hipFree(s->d_len);
	if (s->d_res) hipFree(s->d_res);
	if (s->d_fh) hipFree(s->d_fh);
	if (s->d_ti) hipFree(s->d_ti);
	if (s->d_match) hipFree(s->d_match);
	s->d_frames = NULL; s->d_off = NULL; s->d_len = NULL; s->d_res = NULL; s->d_fh = NULL; s->d_ti = NULL;
	s->d_match = NULL;
	s->cap_frames = 0; s->cap_n = 0;
}

void mosrx_close(mosrx_ctx *c)
{
	int i;
	if (!c)
		return;
	hipSetDevice(c->device);
	if (c->foreign_streams)   /* a caller's stream may still run the set's kernels: they go below */
		hipDeviceSynchronize();
	for (i = 0; i < (int)c->nfs; i++)
		hipEventSynchronize(c->fev[i]);
	for (i = 0; i < MOSRX_FOREIGN; i++)
		if (c->fev[i])
			hipEventDestroy(c->fev[i]);
	if (c->stream)
		hipStreamSynchronize(c->stream);
	for (i = 0; i < NSLOT; i++) {
		if (c->slot[i].stream) {
			hipStreamSynchronize(c->slot[i].stream);
			hipStreamDestroy(c->slot[i].stream);
		}
		if (c->slot[i].done) hipEventDestroy(c->slot[i].done);
		if (c->slot[i].kev0) hipEventDestroy(c->slot[i].kev0);
		if (c->slot[i].kev1) hipEventDestroy(c->slot[i].kev1);
		if (c->slot[i].d_qdesc) hipFree(c->slot[i].d_qdesc);
		if (c->slot[i].h_qdesc) hipHostFree(c->slot[i].h_qdesc);
		if (c->slot[i].d_cnt) hipFree(c->slot[i].d_cnt);
		if (c->slot[i].h_cnt) hipHostFree(c->slot[i].h_cnt);
		free(c->slot[i].h_prev);
		if (c->slot[i].h_txc) hipHostFree(c->slot[i].h_txc);
		slot_free(&c->slot[i]);
	}
	mosrx__bpf_jit_free(c);   /* (joins the compile thread; launches drained above) */
	if (c->d_tables) hipFree(c->d_tables);
	for (i = 0; i < MOSRX_BPF_POOL; i++)
		if (c->d_bpf_pool[i])
			hipFree(c->d_bpf_pool[i]);
	for (i = 0; i < (int)c->nxs; i++) {
		hipStreamSynchronize(c->xs[i]);
		hipStreamDestroy(c->xs[i]);
		hipEventDestroy(c->xdone[i]);
	}
	if (c->ev0) hipEventDestroy(c->ev0);
	if (c->ev1) hipEventDestroy(c->ev1);
	if (c->stream) hipStreamDestroy(c->stream);
	free(c);
}

int mosrx__check_batch(const mosrx_batch *b, int dev)
{
	if (!b)
		return -EINVAL;
	if (b->n == 0)
		return 0;
	if (!b->frames || !b->off || !b->len || (dev && ((uintptr_t)b->frames & 15)))
		return -EINVAL;
	if (b->frames_bytes > MOSRX_MAX_FRAMES_BYTES)
		return -E2BIG;
	return 0;
}

/* Kernel shape: SMALL when every frame fits the SMALL header window (max_len
 * known and <= MOSRX_WINDOW_END_SMALL, 78); otherwise S13 (one header wave + three span streamers, 50 VGPRs,
 * 8 waves per SIMD).  Measured on MI355X (profiles/r01_probe_w8.log,
 * back-to-back launches): 1500 B config S13 18.75 us, S14 18.73, S12 18.73,
 * LARGE 20.84; IMIX S13 20.5 us, S14 21.6, S12 21.7, LARGE 41.8; IMIX with
 * descriptors in reverse buffer order (unsorted tiles) S13 43.5, LARGE 41.6.
 * The tuning shapes are built by scripts/probe_classify.hip only; variant
 * bits 2-6 force one of the library's two (value - 1, MOSRX_KIND_*). */
static int kind_of(const mosrx_ctx *c, uint32_t max_len, uint64_t bytes, uint64_t n)
{
	(void)bytes;
	(void)n;
	const int force = (c->variant >> 2) & 31;
	if (force && force <= MOSRX_KIND_COUNT)
		return force - 1;
	if (max_len && max_len <= MOSRX_WINDOW_END_SMALL)
		return MOSRX_KIND_SMALL;
	return MOSRX_KIND_S13;
}

/* Cache policy of the tail streams (variant bit 1): non-temporal for batches
 * of large frames (the stream is read once), default for batches of small ones,
 * where the header windows and the tails share lines and the windows find them
 * in L2 behind the streamers (IMIX 256K: 22.1 -> 21.0 us; 1500 B: 17.7 us
 * non-temporal against 20.1 us cached; profiles/r02_probe/).  Only when the
 * context runs the library's default variant. */
#ifndef MOSRX_NT_TAIL_MIN_FRAME
#define MOSRX_NT_TAIL_MIN_FRAME 768   /* mean bytes per frame */
#endif
int mosrx__tail_variant(const mosrx_ctx *c, uint64_t bytes, uint64_t n)
{
	if (c->variant != MOSRX_DEFAULT_VARIANT || n == 0 || bytes / n >= MOSRX_NT_TAIL_MIN_FRAME)
		return c->variant;
	return c->variant & ~2;
}

static int tile_for(const mosrx_ctx *c, const mosrx_batch *b)
{
	return kind_of(c, b->max_len, b->frames_bytes, b->n);
}

static int launch_flags(mosrx_ctx *c, const mosrx_batch *b, const uint8_t *frames, const uint32_t *off,
                        const uint16_t *len, mosrx_result *out, uint32_t *cnt, uint32_t *fhash,
                        mosrx_tcpinfo *tinfo, uint32_t kflags, hipStream_t s)
{
	mosrx_kparams kp;
	kp.frames = frames;
	kp.off = off;
	kp.len = len;
	kp.out = out;
	kp.tables = c->d_tables;
	kp.counters = cnt;
	kp.fhash = fhash;
	kp.bmatch = NULL;
	kp.tinfo = tinfo;
	kp.frames_bytes = (uint32_t)b->frames_bytes;
	kp.n = b->n;
	kp.flags = kflags;
	kp.uni = mosrx_uni_pack(b);
	return mosrx_launch_classify(&kp, tile_for(c, b), mosrx__tail_variant(c, b->frames_bytes, b->n), (void *)s);
}

static int launch(mosrx_ctx *c, const mosrx_batch *b, const uint8_t *frames, const uint32_t *off,
                  const uint16_t *len, mosrx_result *out, uint32_t *cnt, uint32_t *fhash, mosrx_tcpinfo *tinfo,
                  hipStream_t s)
{
	return launch_flags(c, b, frames, off, len, out, cnt, fhash, tinfo, c->kflags, s);
}

static uint32_t tx_kflags(int flags)
{
	return ((flags & MOSRX_TX_IP_CSUM) ? MOSRX_KF_TX_IP : 0u) | ((flags & MOSRX_TX_TCP_CSUM) ? MOSRX_KF_TX_TCP : 0u);
}

int mosrx_tx_csum_dev(mosrx_ctx *c, const mosrx_batch *b, int flags, void *stream)
{
	int rc;
	if (!c || (rc = mosrx__check_batch(b, 1)))
		return c ? rc : -EINVAL;
	if (flags & ~(MOSRX_TX_IP_CSUM | MOSRX_TX_TCP_CSUM))
		return -EINVAL;
	if (b->n == 0 || !flags)
		return 0;
	return launch_flags(c, b, b->frames, b->off, b->len, NULL, NULL, NULL, NULL, tx_kflags(flags),
	                    stream ? (hipStream_t)stream : c->stream);
}

int mosrx_tx_csum_dev_checks(mosrx_ctx *c, const mosrx_batch *b, int flags, mosrx_tx_check *d_checks, void *stream)
{
	int rc;
	if (!c || (rc = mosrx__check_batch(b, 1)))
		return c ? rc : -EINVAL;
	if ((flags & ~(MOSRX_TX_IP_CSUM | MOSRX_TX_TCP_CSUM)) || !d_checks || ((uintptr_t)d_checks & 7))
		return -EINVAL;
	if (b->n == 0)
		return 0;
	if (!flags) {   /* no check requested: every record says `what` = 0 */
		HIPCHK(hipMemsetAsync(d_checks, 0, (size_t)b->n * sizeof(*d_checks),
		                      stream ? (hipStream_t)stream : c->stream));
		return 0;
	}
	return launch_flags(c, b, b->frames, b->off, b->len, (mosrx_result *)d_checks, NULL, NULL, NULL,
	                    tx_kflags(flags), stream ? (hipStream_t)stream : c->stream);
}

/* The host side of the TX pass: each frame's checks into the caller's frames,
 * the bytes the in-place rewrite would have stored (little-endian u16). */
static void tx_patch(uint8_t *frames, const uint32_t *off, uint32_t n, const mosrx_tx_check *r)
{
	uint32_t i;
	for (i = 0; i < n; i++) {
		uint8_t *f = frames + off[i];
		if (r[i].what & 1u) {
			f[24] = (uint8_t)r[i].ip_check;
			f[25] = (uint8_t)(r[i].ip_check >> 8);
		}
		if (r[i].what & 2u) {
			uint8_t *t = f + 30u + 4u * r[i].ihl;
			t[0] = (uint8_t)r[i].tcp_check;
			t[1] = (uint8_t)(r[i].tcp_check >> 8);
		}
	}
}

int mosrx_tx_csum_host(mosrx_ctx *c, const mosrx_batch *b, int flags)
{
	struct slot *s;
	int rc;
	if (!c || (rc = mosrx__check_batch(b, 0)))
		return c ? rc : -EINVAL;
	if (flags & ~(MOSRX_TX_IP_CSUM | MOSRX_TX_TCP_CSUM))
		return -EINVAL;
	if (b->n == 0 || !flags)
		return 0;
	s = &c->slot[0];
	if (s->busy)
		return -EBUSY;
	HIPCHK(hipSetDevice(c->device));
	if ((rc = mosrx__slot_reserve(c, s, b->frames_bytes, b->n)))
		return rc;
	static int inplace = -1;                 /* diagnostic: round 3's pass, the frames rewritten and copied back */
	if (inplace < 0)
		inplace = getenv("MOSRX_TX_HOST_INPLACE") != NULL;
	if (inplace) {
		HIPCHK(hipMemcpyAsync(s->d_frames, b->frames, b->frames_bytes, hipMemcpyHostToDevice, s->stream));
		HIPCHK(hipMemcpyAsync(s->d_off, b->off, (size_t)b->n * 4, hipMemcpyHostToDevice, s->stream));
		HIPCHK(hipMemcpyAsync(s->d_len, b->len, (size_t)b->n * 2, hipMemcpyHostToDevice, s->stream));
		if ((rc = launch_flags(c, b, s->d_frames, s->d_off, s->d_len, NULL, NULL, NULL, NULL, tx_kflags(flags),
		                       s->stream)))
			return rc;
		HIPCHK(hipMemcpyAsync((void *)b->frames, s->d_frames, b->frames_bytes, hipMemcpyDeviceToHost, s->stream));
		HIPCHK(hipStreamSynchronize(s->stream));
		return 0;
	}
	if (s->h_txc_n < b->n) {          /* the check records come back into pinned memory */
		if (s->h_txc)
			hipHostFree(s->h_txc);
		s->h_txc = NULL;
		s->h_txc_n = 0;
		if (hipHostMalloc((void **)&s->h_txc, (size_t)s->cap_n * sizeof(mosrx_tx_check), hipHostMallocDefault) !=
		    hipSuccess)
			return -ENOMEM;
		s->h_txc_n = s->cap_n;
	}
	HIPCHK(hipMemcpyAsync(s->d_frames, b->frames, b->frames_bytes, hipMemcpyHostToDevice, s->stream));
	HIPCHK(hipMemcpyAsync(s->d_off, b->off, (size_t)b->n * 4, hipMemcpyHostToDevice, s->stream));
	HIPCHK(hipMemcpyAsync(s->d_len, b->len, (size_t)b->n * 2, hipMemcpyHostToDevice, s->stream));
	/* the kernel writes 8-byte check records (into the records' buffer, 16 B per frame), not the frames */
	if ((rc = launch_flags(c, b, s->d_frames, s->d_off, s->d_len, s->d_res, NULL, NULL, NULL, tx_kflags(flags),
	                       s->stream)))
		return rc;
	HIPCHK(hipMemcpyAsync(s->h_txc, s->d_res, (size_t)b->n * sizeof(mosrx_tx_check), hipMemcpyDeviceToHost,
	                      s->stream));
	HIPCHK(hipStreamSynchronize(s->stream));
	tx_patch((uint8_t *)b->frames, b->off, b->n, s->h_txc);
	return 0;
}

int mosrx_classify_dev_ex(mosrx_ctx *c, const mosrx_batch *b, mosrx_result *d_out, uint32_t *d_fhash,
                          mosrx_tcpinfo *d_tcpinfo, void *stream)
{
	int rc;
	if (!c || (rc = mosrx__check_batch(b, 1)))
		return c ? rc : -EINVAL;
	if (b->n == 0)
		return 0;
	if (!d_out || ((uintptr_t)d_out & 15) || ((uintptr_t)d_fhash & 3) || ((uintptr_t)d_tcpinfo & 3))
		return -EINVAL;
	return launch(c, b, b->frames, b->off, b->len, d_out, NULL, d_fhash, d_tcpinfo,
	              stream ? (hipStream_t)stream : c->stream);
}

int mosrx_classify_dev_compact(mosrx_ctx *c, const mosrx_batch *b, mosrx_result8 *d_out8, void *stream)
{
	int rc;
	if (!c || (rc = mosrx__check_batch(b, 1)))
		return c ? rc : -EINVAL;
	if (b->n == 0)
		return 0;
	if (!d_out8 || ((uintptr_t)d_out8 & 7))
		return -EINVAL;
	return launch_flags(c, b, b->frames, b->off, b->len, (mosrx_result *)d_out8, NULL, NULL, NULL,
	                    c->kflags | MOSRX_KF_COMPACT, stream ? (hipStream_t)stream : c->stream);
}

int mosrx_classify_dev_fh(mosrx_ctx *c, const mosrx_batch *b, mosrx_result *d_out, uint32_t *d_fhash,
                          void *stream)
{
	return mosrx_classify_dev_ex(c, b, d_out, d_fhash, NULL, stream);
}

int mosrx_classify_dev(mosrx_ctx *c, const mosrx_batch *b, mosrx_result *d_out, void *stream)
{
	return mosrx_classify_dev_fh(c, b, d_out, NULL, stream);
}

/* Classification + the installed BPF set over a device-resident batch: the
 * fused kernel when the set has one and the shape is a stream or SMALL tile,
 * else the two kernels back to back on the same stream. */
static int cls_bpf_launch(mosrx_ctx *c, const mosrx_batch *db, mosrx_result *out, uint32_t *cnt, uint32_t *match,
                          hipStream_t s)
{
	mosrx_kparams kp;
	int rc;
	const int kind = tile_for(c, db);
	mosrx__bpf_poll(c);   /* the set's compiled kernels, once its compile is in */
	if (!mosrx_bpf_fused(c) || (kind != MOSRX_KIND_SMALL && kind != MOSRX_KIND_S13)) {
		if ((rc = launch(c, db, db->frames, db->off, db->len, out, cnt, NULL, NULL, s)))
			return rc;
		return mosrx_bpf_dev(c, db, match, (void *)s);
	}
	kp.frames = db->frames;
	kp.off = db->off;
	kp.len = db->len;
	kp.out = out;
	kp.tables = c->d_tables;
	kp.counters = cnt;
	kp.fhash = NULL;
	kp.bmatch = match;
	kp.tinfo = NULL;
	kp.frames_bytes = (uint32_t)db->frames_bytes;
	kp.n = db->n;
	kp.flags = c->kflags;
	kp.uni = 0;   /* the fused kernels take no layout hint */
	return mosrx__bpf_fused_launch(c, &kp, kind == MOSRX_KIND_SMALL, s);
}

int mosrx_classify_bpf_dev(mosrx_ctx *c, const mosrx_batch *b, mosrx_result *d_out, uint32_t *d_match,
                           void *stream)
{
	int rc;
	if (!c || (rc = mosrx__check_batch(b, 1)))
		return c ? rc : -EINVAL;
	if (b->n == 0)
		return 0;
	if (!d_out || !d_match || ((uintptr_t)d_out & 15) || ((uintptr_t)d_match & 3))
		return -EINVAL;
	HIPCHK(hipSetDevice(c->device));
	return cls_bpf_launch(c, b, d_out, NULL, d_match, stream ? (hipStream_t)stream : c->stream);
}

int mosrx_classify_dev_many(mosrx_ctx *c, const mosrx_batch *b, uint32_t nb,
                            mosrx_result *const *d_out, void *stream)
{
	uint32_t i;
	int rc;
	if (!c || !b || !d_out)
		return -EINVAL;
	for (i = 0; i < nb; i++)
		if ((rc = mosrx_classify_dev(c, &b[i], d_out[i], stream)))
			return rc;
	return 0;
}

/* Host batches whose frames and descriptors share one block (a staging area
 * laid out frames | off | len, or descriptors first) cross PCIe in ONE copy:
 * per-copy setup costs ~8 us on MI355X, three copies per 2 MB batch of 64 B
 * frames cost a third of its end-to-end time.  The block may hold gaps up to
 * an eighth of the payload + 4 KiB (a partially filled staging area); the
 * slot's frame buffer is sized for that (span_cap). */
static uint64_t span_limit(uint64_t frames_bytes, uint32_t n)
{
	const uint64_t used = frames_bytes + (uint64_t)n * 6;
	return used + (used >> 3) + 4096;
}

static uint64_t span_cap(uint64_t cap_frames, uint32_t cap_n)
{
	return span_limit(cap_frames, cap_n) + 256;
}

/* One-copy layout of b: the block's lowest address and length, or 0. */
static uint64_t batch_span(const mosrx_batch *b, const uint8_t **lo_out)
{
	const uint8_t *f = b->frames, *o = (const uint8_t *)b->off, *l = (const uint8_t *)b->len;
	const uint8_t *lo = f, *hi = f + b->frames_bytes;
	const uint8_t *oe = o + (size_t)b->n * 4, *le = l + (size_t)b->n * 2;
	if (o < lo) lo = o;
	if (l < lo) lo = l;
	if (oe > hi) hi = oe;
	if (le > hi) hi = le;
	/* disjoint regions (descriptors never inside the frames), alignments kept */
	if ((o < f + b->frames_bytes && oe > f) || (l < f + b->frames_bytes && le > f) || (l < oe && le > o))
		return 0;
	if (((uintptr_t)(f - lo) & 15) || ((uintptr_t)(o - lo) & 3) || ((uintptr_t)(l - lo) & 1))
		return 0;
	if ((uint64_t)(hi - lo) > span_limit(b->frames_bytes, b->n))
		return 0;
	if (!mosrx__host_range_of(lo, (uint64_t)(hi - lo)))   /* the span must lie in one pinned allocation */
		return 0;
	*lo_out = lo;
	return (uint64_t)(hi - lo);
}

int mosrx__slot_reserve(mosrx_ctx *c, struct slot *s, uint64_t frames_bytes, uint32_t n)
{
	if (frames_bytes > s->cap_frames || n > s->cap_n) {
		uint64_t fb = frames_bytes > s->cap_frames ? frames_bytes + (frames_bytes >> 2) : s->cap_frames;
		uint32_t nn = n > s->cap_n ? n + (n >> 2) : s->cap_n;
		hipStreamSynchronize(s->stream);
		slot_free(s);
		fb = (fb + 255) & ~(uint64_t)255;
		if (hipMalloc((void **)&s->d_frames, span_cap(fb, nn)) != hipSuccess ||
		    hipMalloc((void **)&s->d_off, (size_t)nn * 4) != hipSuccess ||
		    hipMalloc((void **)&s->d_len, (size_t)nn * 2) != hipSuccess ||
		    hipMalloc((void **)&s->d_res, (size_t)nn * sizeof(mosrx_result)) != hipSuccess ||
		    hipMalloc((void **)&s->d_fh, (size_t)nn * 4) != hipSuccess ||
		    hipMalloc((void **)&s->d_ti, (size_t)nn * sizeof(mosrx_tcpinfo)) != hipSuccess ||
		    hipMalloc((void **)&s->d_match, (size_t)nn * 4) != hipSuccess) {
			slot_free(s);
			return -ENOMEM;
		}
		s->cap_frames = fb;
		s->cap_n = nn;
	}
	(void)c;
	return 0;
}

/* Before a launch that adds to the slot's reason counters: zero them only when
 * their device value is not known to equal h_prev (mosrx_ctx.h); the launch
 * leaves them unknown until its wait has taken its counts. */
static hipError_t counters_arm(struct slot *s)
{
	if (s->cnt_dirty) {
		hipError_t e = hipMemsetAsync(s->d_cnt, 0, MOSRX_CNT_WORDS * 4, s->stream);
		if (e != hipSuccess)
			return e;
		memset(s->h_prev, 0, MOSRX_CNT_WORDS * 4);
	}
	s->cnt_dirty = 1;
	return hipSuccess;
}

/* Enqueue one end-to-end batch on slot s: H2D frames+descriptors, kernel, D2H results. */
/* h_fhash: flow hashes; h_match: the installed BPF set's match masks (one of
 * the two at most; both use the slot's per-frame u32 buffer); h_ti: pkt_info
 * TCP fields (not with h_match). */
static int host_enqueue(mosrx_ctx *c, struct slot *s, const mosrx_batch *b, mosrx_result *h_out,
                        uint32_t *h_fhash, uint32_t *h_match, mosrx_tcpinfo *h_ti)
{
	int rc;
	if ((rc = mosrx__slot_reserve(c, s, b->frames_bytes, b->n)))
		return rc;
	const uint8_t *lo = NULL;
	const uint64_t span = batch_span(b, &lo);
	const uint8_t *dframes = s->d_frames;
	const uint32_t *doff = s->d_off;
	const uint16_t *dlen = s->d_len;
	if (span) {
		HIPCHK(hipMemcpyAsync(s->d_frames, lo, span, hipMemcpyHostToDevice, s->stream));
		dframes = s->d_frames + (b->frames - lo);
		doff = (const uint32_t *)(s->d_frames + ((const uint8_t *)b->off - lo));
		dlen = (const uint16_t *)(s->d_frames + ((const uint8_t *)b->len - lo));
	} else {
		HIPCHK(hipMemcpyAsync(s->d_frames, b->frames, b->frames_bytes, hipMemcpyHostToDevice, s->stream));
		HIPCHK(hipMemcpyAsync(s->d_off, b->off, (size_t)b->n * 4, hipMemcpyHostToDevice, s->stream));
		HIPCHK(hipMemcpyAsync(s->d_len, b->len, (size_t)b->n * 2, hipMemcpyHostToDevice, s->stream));
	}
	HIPCHK(counters_arm(s));
	if (c->timing) {
		/* one launch: its dispatch stamps its own duration (no queueing gap before it);
		 * the classify + BPF pair: events around both */
		if (!h_match)
			mosrx__stamp_next(s->kev0, s->kev1);
		else
			HIPCHK(hipEventRecord(s->kev0, s->stream));
	}
	if (h_match) {
		mosrx_batch db = *b;
		db.frames = dframes;
		db.off = doff;
		db.len = dlen;
		rc = cls_bpf_launch(c, &db, s->d_res, s->d_cnt, s->d_fh, s->stream);
	} else {
		rc = launch(c, b, dframes, doff, dlen, s->d_res, s->d_cnt, h_fhash ? s->d_fh : NULL,
		            h_ti ? s->d_ti : NULL, s->stream);
	}
	mosrx__stamp_next(NULL, NULL);
	if (rc)
		return rc;
	if (c->timing && h_match)
		HIPCHK(hipEventRecord(s->kev1, s->stream));
	s->timed = c->timing;
	HIPCHK(hipMemcpyAsync(h_out, s->d_res, (size_t)b->n * sizeof(mosrx_result), hipMemcpyDeviceToHost,
	                      s->stream));
	if (h_fhash || h_match)
		HIPCHK(hipMemcpyAsync(h_fhash ? h_fhash : h_match, s->d_fh, (size_t)b->n * 4, hipMemcpyDeviceToHost,
		                      s->stream));
	if (h_ti)
		HIPCHK(hipMemcpyAsync(h_ti, s->d_ti, (size_t)b->n * sizeof(mosrx_tcpinfo), hipMemcpyDeviceToHost,
		                      s->stream));
	HIPCHK(hipMemcpyAsync(s->h_cnt, s->d_cnt, MOSRX_CNT_WORDS * 4, hipMemcpyDeviceToHost, s->stream));
	HIPCHK(hipEventRecord(s->done, s->stream));
	s->busy = 1;
	s->counted = 1;
	return 0;
}

int mosrx_classify_host(mosrx_ctx *c, const mosrx_batch *b, mosrx_result *h_out)
{
	int rc;
	if (!c || (rc = mosrx__check_batch(b, 0)))
		return c ? rc : -EINVAL;
	if ((rc = mosrx_classify_host_submit(c, 0, b, h_out)))
		return rc;
	return mosrx_classify_host_wait(c, 0);
}

int mosrx_classify_host_ex(mosrx_ctx *c, const mosrx_batch *b, mosrx_result *h_out, uint32_t *h_fhash,
                           mosrx_tcpinfo *h_tcpinfo)
{
	int rc;
	if (!c || (rc = mosrx__check_batch(b, 0)))
		return c ? rc : -EINVAL;
	if (!h_fhash && !h_tcpinfo)
		return mosrx_classify_host(c, b, h_out);
	if (c->slot[0].busy)
		return -EBUSY;
	if (b->n == 0)
		return 0;
	if (!h_out)
		return -EINVAL;
	HIPCHK(hipSetDevice(c->device));
	if ((rc = host_enqueue(c, &c->slot[0], b, h_out, h_fhash, NULL, h_tcpinfo)))
		return rc;
	return mosrx_classify_host_wait(c, 0);
}

int mosrx_classify_host_fh(mosrx_ctx *c, const mosrx_batch *b, mosrx_result *h_out, uint32_t *h_fhash)
{
	return mosrx_classify_host_ex(c, b, h_out, h_fhash, NULL);
}

int mosrx_classify_host_submit(mosrx_ctx *c, int slot, const mosrx_batch *b, mosrx_result *h_out)
{
	int rc;
	if (!c || slot < 0 || slot >= NSLOT)
		return -EINVAL;
	if ((rc = mosrx__check_batch(b, 0)))
		return rc;
	if (c->slot[slot].busy)
		return -EBUSY;
	if (b->n == 0) {
		c->slot[slot].busy = 2;   /* nothing enqueued */
		return 0;
	}
	if (!h_out)
		return -EINVAL;
	HIPCHK(hipSetDevice(c->device));
	return host_enqueue(c, &c->slot[slot], b, h_out, NULL, NULL, NULL);
}

int mosrx_classify_bpf_host_submit(mosrx_ctx *c, int slot, const mosrx_batch *b, mosrx_result *h_out,
                                   uint32_t *h_match)
{
	int rc;
	if (!c || slot < 0 || slot >= NSLOT)
		return -EINVAL;
	if ((rc = mosrx__check_batch(b, 0)))
		return rc;
	if (c->slot[slot].busy)
		return -EBUSY;
	if (b->n == 0) {
		c->slot[slot].busy = 2;   /* nothing enqueued */
		return 0;
	}
	if (!h_out || !h_match)
		return -EINVAL;
	HIPCHK(hipSetDevice(c->device));
	return host_enqueue(c, &c->slot[slot], b, h_out, NULL, h_match, NULL);
}

int mosrx_classify_bpf_host(mosrx_ctx *c, const mosrx_batch *b, mosrx_result *h_out, uint32_t *h_match)
{
	int rc;
	if ((rc = mosrx_classify_bpf_host_submit(c, 0, b, h_out, h_match)))
		return rc;
	return mosrx_classify_host_wait(c, 0);
}

int mosrx_classify_host_wait(mosrx_ctx *c, int slot)
{
	struct slot *s;
	if (!c || slot < 0 || slot >= NSLOT)
		return -EINVAL;
	s = &c->slot[slot];
	if (!s->busy)
		return -EINVAL;
	if (s->busy == 1)
		HIPCHK(hipEventSynchronize(s->done));
	{
		uint32_t r, k;
		for (r = 0; r < MOSRX_R_COUNT; r++)
			c->h_cnt[r] = 0;
		if (s->busy == 1 && s->counted) {
			/* the batch's counts: what its launch added to every shard since the last wait */
			for (k = 0; k < MOSRX_CNT_SHARDS; k++)
				for (r = 0; r < MOSRX_R_COUNT; r++) {
					const uint32_t w = k * MOSRX_CNT_STRIDE + r;
					c->h_cnt[r] += s->h_cnt[w] - s->h_prev[w];
					s->h_prev[w] = s->h_cnt[w];
				}
			s->cnt_dirty = 0;
		}
	}
	c->last_kernel_ms = -1.0f;
	if (s->busy == 1 && s->timed && hipEventElapsedTime(&c->last_kernel_ms, s->kev0, s->kev1) != hipSuccess)
		c->last_kernel_ms = -1.0f;
	s->busy = 0;
	return 0;
}

int mosrx_classify_host_reserve(mosrx_ctx *c, uint64_t frames_bytes, uint32_t n)
{
	int i, rc;
	if (!c || !n)
		return -EINVAL;
	HIPCHK(hipSetDevice(c->device));
	for (i = 0; i < NSLOT; i++)
		if (c->slot[i].busy)
			return -EBUSY;
	for (i = 0; i < NSLOT; i++)
		if ((rc = mosrx__slot_reserve(c, &c->slot[i], frames_bytes, n)))
			return rc;
	return 0;
}

int mosrx_classify_host_ready(mosrx_ctx *c, int slot)
{
	hipError_t e;
	if (!c || slot < 0 || slot >= NSLOT)
		return -EINVAL;
	if (c->slot[slot].busy != 1)
		return 1;
	e = hipEventQuery(c->slot[slot].done);
	return e == hipSuccess ? 1 : e == hipErrorNotReady ? 0 : -EIO;
}

int mosrx_set_counters(mosrx_ctx *c, int on)
{
	if (!c)
		return -EINVAL;
	c->no_counters = !on;
	return 0;
}

int mosrx_set_direct(mosrx_ctx *c, uint64_t max_bytes, uint32_t max_frames)
{
	if (!c)
		return -EINVAL;
	c->direct_max = max_bytes;
	c->direct_frames = max_frames;
	return 0;
}

int mosrx_slot_direct(mosrx_ctx *c, int slot)
{
	if (!c || slot < 0 || slot >= NSLOT)
		return -EINVAL;
	return c->slot[slot].direct;
}

int mosrx_set_timing(mosrx_ctx *c, int on)
{
	if (!c)
		return -EINVAL;
	c->timing = on ? 1 : 0;
	return 0;
}

int mosrx_last_kernel_ms(mosrx_ctx *c, float *ms)
{
	if (!c || !ms)
		return -EINVAL;
	if (c->last_kernel_ms < 0)
		return -ENODATA;
	*ms = c->last_kernel_ms;
	return 0;
}

/* ---- a group of host batches in one launch (gpu_module_func's rx ring) ---- */
struct region { const uint8_t *lo; uint64_t len; int own; uint8_t *dev; uint64_t alloc; };
struct out_dev { void *out, *ti, *fh, *match; };   /* a direct group's output arrays, device addresses */

/* Device copies of every region of the group: regions in address order are
 * gathered into copy runs wherever the gap to the next one is under an eighth
 * of the run + 4 KiB (packed stages, or consecutive runs lent by one source)
 * and both lie in the same known pinned allocation (so no copy spans two
 * allocations or an unmapped gap between them), and each run keeps its host
 * address modulo 256 on the device, so a frame buffer stays 16-byte aligned.
 * A frame buffer that is not 16-byte aligned on the host is copied on its own
 * to an aligned device address. */
static int group_copy(struct slot *s, struct region *r, uint32_t nr, uint64_t *dev_bytes, int issue)
{
	uint32_t i, j;
	uint64_t cur = 0;
	struct region *ord[3 * MOSRX_MAX_GROUP];
	for (i = 0; i < nr; i++) {        /* insertion sort by address (nr <= 192) */
		for (j = i; j > 0 && ord[j - 1]->lo > r[i].lo; j--)
			ord[j] = ord[j - 1];
		ord[j] = &r[i];
	}
	for (i = 0; i < nr;) {
		const uint8_t *lo = ord[i]->lo, *hi = lo + ord[i]->len;
		uint64_t base;
		j = i + 1;
		if (!ord[i]->own && ord[i]->alloc)
			while (j < nr && !ord[j]->own && ord[j]->alloc == ord[i]->alloc &&
			       (uint64_t)(ord[j]->lo > hi ? ord[j]->lo - hi : 0) <= ((uint64_t)(hi - lo) >> 3) + 4096) {
				if (ord[j]->lo + ord[j]->len > hi)
					hi = ord[j]->lo + ord[j]->len;
				j++;
			}
		base = ((cur + 255) & ~(uint64_t)255) + (ord[i]->own ? 0 : ((uintptr_t)lo & 255));
		if (issue) {
			uint32_t k;
			for (k = i; k < j; k++)
				ord[k]->dev = s->d_frames + base + (uint64_t)(ord[k]->lo - lo);
			HIPCHK(hipMemcpyAsync(s->d_frames + base, lo, (size_t)(hi - lo), hipMemcpyHostToDevice, s->stream));
		}
		cur = base + (uint64_t)(hi - lo);
		i = j;
	}
	*dev_bytes = cur;
	return 0;
}

/* Direct groups (mosrx_set_direct): a group whose frames and descriptors
 * total at most c->direct_max bytes in at most c->direct_frames frames, every
 * region in a known pinned range with a device address for this context's GPU
 * (frame buffers 16-byte aligned, their extent rounded up to 16 bytes as the
 * kernels' buffer resources do), is read by the kernel
 * in place over PCIe: no H2D copy and no batch-table copy (the kernel reads
 * the pinned table).  Each copy of the copying path is a blit or SDMA
 * dispatch plus a queue handoff, 4-12 us apiece, ~80 us per group cycle with
 * 3 blits and one SDMA copy (profiles/r06/cycle); a small group's PCIe
 * transfer inside the kernel is shorter than that chain.  The regions' device
 * addresses go into r[].dev; *bytes: the input bytes (the kernel-shape
 * choice's byte count).  0: copy the group. */
static int direct_regions(const mosrx_ctx *c, const struct slot *s, struct region *r, uint32_t nr, uint64_t ntot,
                          uint64_t *bytes)
{
	uint64_t in = 0;
	uint32_t i;
	for (i = 0; i < nr; i++)
		in += r[i].len;
	if (!c->direct_max || in > c->direct_max || ntot > c->direct_frames || !s->hq_dev)
		return 0;
	for (i = 0; i < nr; i++) {   /* r[]: (frames, off, len) per non-empty batch */
		const int fr = i % 3 == 0;
		if (fr && r[i].own)
			return 0;
		if (!(r[i].dev = (uint8_t *)mosrx__host_dev_of(r[i].lo, fr ? (r[i].len + 15) & ~(uint64_t)15 : r[i].len,
		                                               c->device)))
			return 0;
	}
	*bytes = in;
	return 1;
}

/* The device addresses of a direct group's output arrays, when every one of
 * them is pinned too and aligned to its element's store (16 / 8 bytes for the
 * records, 4 for the side arrays): the kernel then writes them in place (no
 * D2H copies). */
static int direct_outputs(int device, const mosrx_batch *b, uint32_t nb, mosrx_result *const *h_out, size_t rsz,
                          mosrx_tcpinfo *const *h_ti, uint32_t *const *h_fh, uint32_t *const *h_match,
                          struct out_dev *od)
{
	uint32_t i;
	for (i = 0; i < nb; i++) {
		const uint64_t n = b[i].n;
		memset(&od[i], 0, sizeof(od[i]));
		if (!n)
			continue;
		if (((uintptr_t)h_out[i] & (rsz - 1)) || (h_ti && ((uintptr_t)h_ti[i] & 3)) ||
		    (h_fh && ((uintptr_t)h_fh[i] & 3)) || (h_match && ((uintptr_t)h_match[i] & 3)))
			return 0;
		if (!(od[i].out = mosrx__host_dev_of(h_out[i], n * rsz, device)) ||
		    (h_ti && !(od[i].ti = mosrx__host_dev_of(h_ti[i], n * sizeof(mosrx_tcpinfo), device))) ||
		    (h_fh && !(od[i].fh = mosrx__host_dev_of(h_fh[i], n * 4, device))) ||
		    (h_match && !(od[i].match = mosrx__host_dev_of(h_match[i], n * 4, device))))
			return 0;
	}
	return 1;
}

int mosrx_classify_host_group_submit(mosrx_ctx *c, int slot, const mosrx_batch *b, uint32_t nb,
                                     mosrx_result *const *h_out, mosrx_tcpinfo *const *h_tcpinfo)
{
	return mosrx_classify_host_group_submit_ex(c, slot, b, nb, h_out, h_tcpinfo, NULL);
}

/* One launch over a group of host batches: records, and the side arrays asked
 * for (pkt_info, flow hashes, and with h_match the installed BPF set's masks:
 * the fused classify + BPF queue kernel, or the classify queue + the set's
 * kernel per batch while the set has no compiled form). */
static int group_submit(mosrx_ctx *c, int slot, const mosrx_batch *b, uint32_t nb, mosrx_result *const *h_out,
                        mosrx_tcpinfo *const *h_tcpinfo, uint32_t *const *h_fhash, uint32_t *const *h_match,
                        int compact)
{
	/* compact: h_out[i] are mosrx_result8 arrays (8-byte records, VAR_C8); flow hashes and masks, no pkt_info */
	const size_t rsz = compact ? sizeof(mosrx_result8) : sizeof(mosrx_result);
	struct region r[3 * MOSRX_MAX_GROUP];
	uint32_t i, nr = 0, tiles = 0, maxl = 0, ntot = 0, tile;
	uint64_t dev_bytes = 0, pre = 0;
	mosrx_qparams qp;
	struct slot *s;
	struct out_dev od[MOSRX_MAX_GROUP];
	int rc, unknown = 0, kind, tpb_ok = 1;
	int fused = 0, uni = 0, direct, out_direct;
	if (!c || slot < 0 || slot >= NSLOT || !b || !h_out || nb == 0 || nb > MOSRX_MAX_GROUP ||
	    (h_match && h_tcpinfo) || (compact && h_tcpinfo))
		return -EINVAL;
	s = &c->slot[slot];
	if (s->busy)
		return -EBUSY;
	for (i = 0; i < nb; i++) {
		if ((rc = mosrx__check_batch(&b[i], 0)))
			return rc;
		if (b[i].n && (!h_out[i] || (h_tcpinfo && !h_tcpinfo[i]) || (h_fhash && !h_fhash[i]) ||
		               (h_match && !h_match[i])))
			return -EINVAL;
		if (!b[i].max_len)
			unknown = 1;
		maxl = b[i].max_len > maxl ? b[i].max_len : maxl;
		ntot += b[i].n;
		if (!b[i].n)
			continue;
		r[nr++] = (struct region){b[i].frames, b[i].frames_bytes, ((uintptr_t)b[i].frames & 15) != 0, NULL,
		                          mosrx__host_range_of(b[i].frames, b[i].frames_bytes)};
		r[nr++] = (struct region){(const uint8_t *)b[i].off, (uint64_t)b[i].n * 4, 0, NULL,
		                          mosrx__host_range_of(b[i].off, (uint64_t)b[i].n * 4)};
		r[nr++] = (struct region){(const uint8_t *)b[i].len, (uint64_t)b[i].n * 2, 0, NULL,
		                          mosrx__host_range_of(b[i].len, (uint64_t)b[i].n * 2)};
	}
	if (ntot == 0) {
		s->busy = 2;
		s->direct = 0;
		return 0;
	}
	HIPCHK(hipSetDevice(c->device));
	direct = direct_regions(c, s, r, nr, ntot, &dev_bytes);
	out_direct = direct && direct_outputs(c->device, b, nb, h_out, rsz, h_tcpinfo, h_fhash, h_match, od);
	if (!direct) {
		group_copy(s, r, nr, &dev_bytes, 0);
		if ((rc = mosrx__slot_reserve(c, s, dev_bytes, ntot)))
			return rc;
		if ((rc = group_copy(s, r, nr, &dev_bytes, 1)))
			return rc;
	} else if (!out_direct && (rc = mosrx__slot_reserve(c, s, 0, ntot))) {
		return rc;
	}
	kind = kind_of(c, unknown ? 0 : maxl, dev_bytes, ntot);   /* one shape for the whole group */
	tile = MOSRX_KIND_FRAMES(kind);
	if (h_match) {
		mosrx__bpf_poll(c);   /* the set's compiled kernels, once its compile is in */
		fused = (compact ? c->bpf_fu[FU_QS8] && c->bpf_fu[FU_QM8] : c->bpf_fu[FU_QS] && c->bpf_fu[FU_QM]) &&
		        (kind == MOSRX_KIND_SMALL || kind == MOSRX_KIND_S13);
	}
	for (i = 0, nr = 0; i < nb; i++) {
		mosrx_qdesc *d = &s->h_qdesc[i];
		memset(d, 0, sizeof(*d));
		d->tile_base = tiles;
		d->out = (mosrx_result *)((uint8_t *)s->d_res + pre * rsz);
		if (fused)
			d->bmatch = s->d_match + pre;
		else
			d->tinfo = h_tcpinfo ? s->d_ti + pre : NULL;
		d->fhash = h_fhash ? s->d_fh + pre : NULL;
		if (out_direct && b[i].n) {   /* the kernel writes the caller's pinned arrays in place */
			d->out = (mosrx_result *)od[i].out;
			if (fused)
				d->bmatch = (uint32_t *)od[i].match;
			else
				d->tinfo = (mosrx_tcpinfo *)od[i].ti;
			d->fhash = (uint32_t *)od[i].fh;
		}
		if (b[i].n) {
			d->frames = r[nr].dev;
			d->off = (const uint32_t *)r[nr + 1].dev;
			d->len = (const uint16_t *)r[nr + 2].dev;
			d->frames_bytes = (uint32_t)b[i].frames_bytes;
			d->n = b[i].n;
			d->uni = mosrx_uni_pack(&b[i]);   /* the copy keeps the layout: offsets are relative to frames */
			uni |= d->uni != 0;
			nr += 3;
		}
		tiles += (b[i].n + tile - 1) / tile;
		if ((b[i].n + tile - 1) / tile != (b[0].n + tile - 1) / tile)
			tpb_ok = 0;
		pre += b[i].n;
	}
	if (!direct)
		HIPCHK(hipMemcpyAsync(s->d_qdesc, s->h_qdesc, nb * sizeof(mosrx_qdesc), hipMemcpyHostToDevice, s->stream));
	if (!c->no_counters)
		HIPCHK(counters_arm(s));
	qp.desc = direct ? s->hq_dev : s->d_qdesc;
	qp.tables = c->d_tables;
	qp.counters = c->no_counters ? NULL : s->d_cnt;
	qp.nb = nb;
	qp.flags = c->kflags;
	qp.tpb = tpb_ok ? tiles / nb : 0;
	qp.tinfo = h_tcpinfo ? 1u : compact ? 2u : 0u;
	qp.uni = (uint32_t)uni;
	if (c->timing) {
		/* one launch (the queue kernel, fused or not): its dispatch stamps the
		 * kernel's own duration -- events recorded around it would also count the
		 * wait behind the other slot's kernel; the per-batch BPF fallback: events */
		if (!h_match || fused)
			mosrx__stamp_next(s->kev0, s->kev1);
		else
			HIPCHK(hipEventRecord(s->kev0, s->stream));
	}
	if (fused) {
		if ((rc = mosrx__bpf_fused_queue_launch(c, &qp, tiles, kind == MOSRX_KIND_SMALL,
		                                        mosrx__tail_variant(c, dev_bytes, ntot), s->stream)))
			return rc;
	} else {
		if ((rc = mosrx_launch_queue(&qp, tiles, kind, mosrx__tail_variant(c, dev_bytes, ntot), s->stream)))
			return rc;
		for (i = 0, pre = 0; h_match && i < nb; pre += b[i].n, i++)   /* the set per batch, same stream */
			if ((rc = mosrx__bpf_launch_dev(c, s->h_qdesc[i].frames, b[i].frames_bytes, s->h_qdesc[i].off,
			                                s->h_qdesc[i].len, b[i].n,
			                                out_direct && b[i].n ? (uint32_t *)od[i].match : s->d_match + pre,
			                                s->stream)))
				return rc;
	}
	mosrx__stamp_next(NULL, NULL);   /* (a stamp pair no launch took is not left for the next one) */
	if (c->timing && h_match && !fused)
		HIPCHK(hipEventRecord(s->kev1, s->stream));
	s->timed = c->timing;
	/* results: one copy when the host buffers follow each other, else per batch */
	for (i = 0, pre = 0; !out_direct && i < nb;) {
		uint32_t j = i + 1;
		uint64_t n = b[i].n;
		while (j < nb && (uint8_t *)h_out[j] == (uint8_t *)h_out[j - 1] + b[j - 1].n * rsz &&
		       (!h_tcpinfo || h_tcpinfo[j] == h_tcpinfo[j - 1] + b[j - 1].n) &&
		       (!h_fhash || h_fhash[j] == h_fhash[j - 1] + b[j - 1].n) &&
		       (!h_match || h_match[j] == h_match[j - 1] + b[j - 1].n))
			n += b[j++].n;
		if (n) {
			HIPCHK(hipMemcpyAsync(h_out[i], (uint8_t *)s->d_res + pre * rsz, (size_t)n * rsz, hipMemcpyDeviceToHost,
			                      s->stream));
			if (h_tcpinfo)
				HIPCHK(hipMemcpyAsync(h_tcpinfo[i], s->d_ti + pre, (size_t)n * sizeof(mosrx_tcpinfo),
				                      hipMemcpyDeviceToHost, s->stream));
			if (h_fhash)
				HIPCHK(hipMemcpyAsync(h_fhash[i], s->d_fh + pre, (size_t)n * 4, hipMemcpyDeviceToHost, s->stream));
			if (h_match)
				HIPCHK(hipMemcpyAsync(h_match[i], s->d_match + pre, (size_t)n * 4, hipMemcpyDeviceToHost,
				                      s->stream));
		}
		pre += n;
		i = j;
	}
	if (!c->no_counters)
		HIPCHK(hipMemcpyAsync(s->h_cnt, s->d_cnt, MOSRX_CNT_WORDS * 4, hipMemcpyDeviceToHost, s->stream));
	HIPCHK(hipEventRecord(s->done, s->stream));
	s->busy = 1;
	s->counted = !c->no_counters;
	s->direct = direct;
	return 0;
}

int mosrx_classify_host_group_submit_ex(mosrx_ctx *c, int slot, const mosrx_batch *b, uint32_t nb,
                                        mosrx_result *const *h_out, mosrx_tcpinfo *const *h_tcpinfo,
                                        uint32_t *const *h_fhash)
{
	return group_submit(c, slot, b, nb, h_out, h_tcpinfo, h_fhash, NULL, 0);
}

int mosrx_classify_host_group_submit_c8(mosrx_ctx *c, int slot, const mosrx_batch *b, uint32_t nb,
                                        mosrx_result8 *const *h_out8, uint32_t *const *h_fhash)
{
	return group_submit(c, slot, b, nb, (mosrx_result *const *)h_out8, NULL, h_fhash, NULL, 1);
}

int mosrx_classify_host_group_submit_bpf_c8(mosrx_ctx *c, int slot, const mosrx_batch *b, uint32_t nb,
                                            mosrx_result8 *const *h_out8, uint32_t *const *h_fhash,
                                            uint32_t *const *h_match)
{
	if (!h_match)
		return -EINVAL;
	return group_submit(c, slot, b, nb, (mosrx_result *const *)h_out8, NULL, h_fhash, h_match, 1);
}

int mosrx_classify_host_group_submit_bpf(mosrx_ctx *c, int slot, const mosrx_batch *b, uint32_t nb,
                                         mosrx_result *const *h_out, uint32_t *const *h_fhash,
                                         uint32_t *const *h_match)
{
	if (!h_match)
		return -EINVAL;
	return group_submit(c, slot, b, nb, h_out, NULL, h_fhash, h_match, 0);
}

int mosrx_classify_host_submit_ex(mosrx_ctx *c, int slot, const mosrx_batch *b, mosrx_result *h_out,
                                  mosrx_tcpinfo *h_tcpinfo)
{
	int rc;
	if (!h_tcpinfo)
		return mosrx_classify_host_submit(c, slot, b, h_out);
	if (!c || slot < 0 || slot >= NSLOT)
		return -EINVAL;
	if ((rc = mosrx__check_batch(b, 0)))
		return rc;
	if (c->slot[slot].busy)
		return -EBUSY;
	if (b->n == 0) {
		c->slot[slot].busy = 2;
		return 0;
	}
	if (!h_out)
		return -EINVAL;
	HIPCHK(hipSetDevice(c->device));
	return host_enqueue(c, &c->slot[slot], b, h_out, NULL, NULL, h_tcpinfo);
}

int mosrx_last_counters(mosrx_ctx *c, uint64_t counts[MOSRX_R_COUNT])
{
	int i;
	if (!c || !counts)
		return -EINVAL;
	for (i = 0; i < MOSRX_R_COUNT; i++)
		counts[i] = c->h_cnt[i];
	return 0;
}

int mosrx_sync(mosrx_ctx *c)
{
	if (!c)
		return -EINVAL;
	HIPCHK(hipStreamSynchronize(c->stream));
	return 0;
}

int mosrx_dev_alloc(mosrx_ctx *c, size_t bytes, void **dptr)
{
	if (!c || !dptr)
		return -EINVAL;
	HIPCHK(hipSetDevice(c->device));
	if (hipMalloc(dptr, bytes ? bytes : 1) != hipSuccess)
		return -ENOMEM;
	return 0;
}

int mosrx_dev_free(mosrx_ctx *c, void *dptr)
{
	if (!c)
		return -EINVAL;
	HIPCHK(hipFree(dptr));
	return 0;
}

/* ---- pinned host ranges (mosrx_source.h) ----------------------------------
 * Every pinned allocation the library knows (its own, the sources', the
 * caller's registered ones), sorted by address: a submit looks up each of its
 * regions (3 per batch) by binary search under a read lock, so concurrent rx
 * threads do not serialise on it. */
#define MAX_RANGES 4096
/* dev: the range's device address (hipHostGetDevicePointer at add), 0 when
 * the runtime gave none -- such a range is copied, never read in place;
 * dev_id: the HIP device current at add, the only one it is read in place by
 * (a context on another GPU copies it) */
static struct range { uintptr_t lo, hi; uint64_t id; int reg; uintptr_t dev; int dev_id; } g_ranges[MAX_RANGES];
static uint32_t g_nranges;
static uint64_t g_range_seq;
static uint64_t g_range_maxlen;   /* longest range ever added: no range starting further below can hold a */
static pthread_rwlock_t g_range_lock = PTHREAD_RWLOCK_INITIALIZER;

/* first range whose lo > a */
static uint32_t range_upper(uintptr_t a)
{
	uint32_t lo = 0, hi = g_nranges;
	while (lo < hi) {
		const uint32_t mid = (lo + hi) / 2;
		if (g_ranges[mid].lo <= a)
			lo = mid + 1;
		else
			hi = mid;
	}
	return lo;
}

static int range_add(const void *p, uint64_t len, int reg)
{
	int rc = -ENOSPC;
	void *dev = NULL;
	int dev_id = -1;
	if (p && (hipGetDevice(&dev_id) != hipSuccess || hipHostGetDevicePointer(&dev, (void *)p, 0) != hipSuccess))
		dev = NULL;
	pthread_rwlock_wrlock(&g_range_lock);
	if (p && len && g_nranges < MAX_RANGES) {
		const uint32_t at = range_upper((uintptr_t)p);
		memmove(&g_ranges[at + 1], &g_ranges[at], (g_nranges - at) * sizeof(g_ranges[0]));
		g_ranges[at].lo = (uintptr_t)p;
		g_ranges[at].hi = (uintptr_t)p + len;
		g_ranges[at].id = ++g_range_seq;
		g_ranges[at].reg = reg;
		g_ranges[at].dev = (uintptr_t)dev;
		g_ranges[at].dev_id = dev_id;
		g_nranges++;
		if (len > g_range_maxlen)
			g_range_maxlen = len;
		rc = 0;
	}
	pthread_rwlock_unlock(&g_range_lock);
	return rc;
}

/* Remove the range starting at p; its `reg` flag, or -1 if none. */
static int range_del(const void *p)
{
	int reg = -1;
	uint32_t at;
	pthread_rwlock_wrlock(&g_range_lock);
	at = range_upper((uintptr_t)p);
	if (at > 0 && g_ranges[at - 1].lo == (uintptr_t)p) {
		reg = g_ranges[at - 1].reg;
		memmove(&g_ranges[at - 1], &g_ranges[at], (g_nranges - at) * sizeof(g_ranges[0]));
		g_nranges--;
	}
	pthread_rwlock_unlock(&g_range_lock);
	return reg;
}

void mosrx__host_range_add(const void *p, uint64_t len)
{
	range_add(p, len, 0);
}

void mosrx__host_range_del(const void *p)
{
	range_del(p);
}

/* The id of the known range holding [p, p + len), 0 if none: the ranges
 * starting at or below p, nearest first (usually the first one holds it; a
 * registered sub-range of another allocation can sit in between), back to
 * where no range is long enough to reach p. */
uint64_t mosrx__host_range_of(const void *p, uint64_t len)
{
	const uintptr_t a = (uintptr_t)p, b = a + len;
	uint64_t id = 0;
	uint32_t k;
	if (b < a)
		return 0;
	pthread_rwlock_rdlock(&g_range_lock);
	for (k = range_upper(a); k-- > 0 && a - g_ranges[k].lo < g_range_maxlen;)
		if (b <= g_ranges[k].hi) {
			id = g_ranges[k].id;
			break;
		}
	pthread_rwlock_unlock(&g_range_lock);
	return id;
}

/* The address on HIP device `device` of [p, p + len) when a known range with
 * a device address for that device holds it (a direct group's region), else
 * NULL. */
void *mosrx__host_dev_of(const void *p, uint64_t len, int device)
{
	const uintptr_t a = (uintptr_t)p, b = a + len;
	void *dev = NULL;
	uint32_t k;
	if (b < a)
		return NULL;
	pthread_rwlock_rdlock(&g_range_lock);
	for (k = range_upper(a); k-- > 0 && a - g_ranges[k].lo < g_range_maxlen;)
		if (b <= g_ranges[k].hi) {
			if (g_ranges[k].dev && g_ranges[k].dev_id == device)
				dev = (void *)(g_ranges[k].dev + (a - g_ranges[k].lo));
			break;
		}
	pthread_rwlock_unlock(&g_range_lock);
	return dev;
}

int mosrx_host_register(mosrx_ctx *c, void *hptr, size_t bytes, int flags)
{
	int rc;
	if (!c || !hptr || !bytes || (flags & ~MOSRX_HOST_PINNED))
		return -EINVAL;
	HIPCHK(hipSetDevice(c->device));
	if (!(flags & MOSRX_HOST_PINNED) && hipHostRegister(hptr, bytes, hipHostRegisterDefault) != hipSuccess)
		return -ENOMEM;
	if ((rc = range_add(hptr, bytes, !(flags & MOSRX_HOST_PINNED)))) {
		if (!(flags & MOSRX_HOST_PINNED))
			hipHostUnregister(hptr);
		return rc;
	}
	return 0;
}

int mosrx_host_unregister(mosrx_ctx *c, void *hptr)
{
	int reg;
	if (!c || !hptr)
		return -EINVAL;
	if ((reg = range_del(hptr)) < 0)
		return -ENOENT;
	if (reg) {
		HIPCHK(hipSetDevice(c->device));
		HIPCHK(hipHostUnregister(hptr));
	}
	return 0;
}

/* Pinned host memory, NUMA-local: hipHostMallocNumaUser places the pages by
 * the calling thread's memory policy (mOS binds each mTCP thread to its core
 * and that core's node before init_handle, core/src/cpu.c:56-87), i.e. on the
 * node of the thread that stages and consumes the frames. */
int mosrx_host_alloc(mosrx_ctx *c, size_t bytes, void **hptr)
{
	if (!c || !hptr)
		return -EINVAL;
	HIPCHK(hipSetDevice(c->device));   /* the range is read in place by this device (direct groups) */
	if (hipHostMalloc(hptr, bytes ? bytes : 1, hipHostMallocDefault | hipHostMallocNumaUser) != hipSuccess &&
	    hipHostMalloc(hptr, bytes ? bytes : 1, hipHostMallocDefault) != hipSuccess)
		return -ENOMEM;
	mosrx__host_range_add(*hptr, bytes ? bytes : 1);
	return 0;
}

int mosrx_host_free(mosrx_ctx *c, void *hptr)
{
	if (!c)
		return -EINVAL;
	mosrx__host_range_del(hptr);
	HIPCHK(hipHostFree(hptr));
	return 0;
}

int mosrx_memcpy_h2d(mosrx_ctx *c, void *dst, const void *src, size_t bytes)
{
	if (!c)
		return -EINVAL;
	HIPCHK(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, c->stream));
	HIPCHK(hipStreamSynchronize(c->stream));
	return 0;
}

int mosrx_launch_pull(void *dst, const void *src, uint64_t bytes, void *stream);

int mosrx_memcpy_h2d_pull(mosrx_ctx *c, void *dst, const void *src, size_t bytes)
{
	void *dsrc = NULL;
	if (!c || !dst || !src)
		return -EINVAL;
	HIPCHK(hipSetDevice(c->device));
	if (hipHostGetDevicePointer(&dsrc, (void *)src, 0) != hipSuccess || !dsrc)
		return -EINVAL;   /* not pinned host memory the device can reach */
	if (mosrx_launch_pull(dst, dsrc, bytes, c->stream))
		return -EIO;
	HIPCHK(hipStreamSynchronize(c->stream));
	return 0;
}

int mosrx_memcpy_d2h(mosrx_ctx *c, void *dst, const void *src, size_t bytes)
{
	if (!c)
		return -EINVAL;
	HIPCHK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, c->stream));
	HIPCHK(hipStreamSynchronize(c->stream));
	return 0;
}

void *mosrx_stream(mosrx_ctx *c) { return c ? (void *)c->stream : NULL; }

int mosrx_time_dev(mosrx_ctx *c, const mosrx_batch *b, uint32_t nb, mosrx_result *const *d_out,
                   uint32_t iters, float *ms)
{
	uint32_t i;
	int rc;
	if (!c || !b || !d_out || !ms || nb == 0)
		return -EINVAL;
	HIPCHK(hipSetDevice(c->device));
	HIPCHK(hipEventRecord(c->ev0, c->stream));
	for (i = 0; i < iters; i++)
		if ((rc = mosrx_classify_dev(c, &b[i % nb], d_out[i % nb], c->stream)))
			return rc;
	HIPCHK(hipEventRecord(c->ev1, c->stream));
	HIPCHK(hipEventSynchronize(c->ev1));
	HIPCHK(hipEventElapsedTime(ms, c->ev0, c->ev1));
	return 0;
}

int mosrx_time_host(mosrx_ctx *c, const mosrx_batch *b, uint32_t nb, mosrx_result *const *h_out,
                    uint32_t iters, float *ms)
{
	uint32_t i;
	int rc, k;
	if (!c || !b || !h_out || !ms || nb == 0)
		return -EINVAL;
	HIPCHK(hipSetDevice(c->device));
	for (i = 0; i < nb; i++)   /* size both slots before timing */
		for (k = 0; k < NSLOT; k++)
			if ((rc = mosrx__slot_reserve(c, &c->slot[k], b[i].frames_bytes, b[i].n)))
				return rc;
	HIPCHK(hipDeviceSynchronize());
	HIPCHK(hipEventRecord(c->ev0, c->stream));
	for (k = 0; k < NSLOT; k++)
		HIPCHK(hipStreamWaitEvent(c->slot[k].stream, c->ev0, 0));
	for (k = 0; k < NSLOT; k++)
		if (c->slot[k].busy)
			return -EBUSY;
	for (i = 0; i < iters; i++) {
		struct slot *s = &c->slot[i % NSLOT];
		if ((rc = host_enqueue(c, s, &b[i % nb], h_out[i % nb], NULL, NULL, NULL)))
			return rc;
	}
	for (k = 0; k < NSLOT; k++) {
		HIPCHK(hipEventRecord(c->slot[k].done, c->slot[k].stream));
		HIPCHK(hipStreamWaitEvent(c->stream, c->slot[k].done, 0));
		c->slot[k].busy = 0;
	}
	HIPCHK(hipEventRecord(c->ev1, c->stream));
	HIPCHK(hipEventSynchronize(c->ev1));
	HIPCHK(hipEventElapsedTime(ms, c->ev0, c->ev1));
	return 0;
}

/* One enqueue of operation `op` on batch b (see mosrx_time_op). */
static int run_op(mosrx_ctx *c, int op, int arg, const mosrx_batch *b, void *out, void *aux, hipStream_t s)
{
	switch (op) {
	case MOSRX_OP_CLASSIFY: return mosrx_classify_dev(c, b, (mosrx_result *)out, s);
	case MOSRX_OP_CLASSIFY_FH: return mosrx_classify_dev_fh(c, b, (mosrx_result *)out, (uint32_t *)aux, s);
	case MOSRX_OP_BPF: return mosrx_bpf_dev(c, b, (uint32_t *)out, s);
	case MOSRX_OP_TX_CSUM: return mosrx_tx_csum_dev(c, b, arg, s);
	case MOSRX_OP_CLASSIFY_BPF: return mosrx_classify_bpf_dev(c, b, (mosrx_result *)out, (uint32_t *)aux, s);
	case MOSRX_OP_CLASSIFY_TI: return mosrx_classify_dev_ex(c, b, (mosrx_result *)out, NULL, (mosrx_tcpinfo *)aux, s);
	case MOSRX_OP_TX_CHECKS: return mosrx_tx_csum_dev_checks(c, b, arg, (mosrx_tx_check *)out, s);
	default: return -EINVAL;
	}
}

/* Streams for the multi-stream timing, kept for the context's life so a timed
 * call holds launches only (creating streams costs milliseconds). */
int mosrx__ensure_streams(mosrx_ctx *c, uint32_t n)
{
	while (c->nxs < n) {
		if (hipStreamCreateWithFlags(&c->xs[c->nxs], hipStreamNonBlocking) != hipSuccess)
			return -EIO;
		if (hipEventCreateWithFlags(&c->xdone[c->nxs], hipEventDisableTiming) != hipSuccess) {
			hipStreamDestroy(c->xs[c->nxs]);
			return -EIO;
		}
		c->nxs++;
	}
	return 0;
}

static int time_streams(mosrx_ctx *c, int op, int arg, const mosrx_batch *b, uint32_t nb, void *const *out,
                        void *const *aux, uint32_t iters, uint32_t nstreams, float *ms)
{
	uint32_t i, k;
	int rc;
	if ((rc = mosrx__ensure_streams(c, nstreams)))
		return rc;
	HIPCHK(hipEventRecord(c->ev0, c->stream));
	for (k = 0; k < nstreams; k++)
		HIPCHK(hipStreamWaitEvent(c->xs[k], c->ev0, 0));
	/* batch i on stream i % nstreams: independent batches overlap their
	 * launch/drain phases the way several rx queues would */
	for (i = 0; i < iters; i++)
		if ((rc = run_op(c, op, arg, &b[i % nb], out ? out[i % nb] : NULL, aux ? aux[i % nb] : NULL,
		                 c->xs[i % nstreams])))
			return rc;
	for (k = 0; k < nstreams; k++) {
		HIPCHK(hipEventRecord(c->xdone[k], c->xs[k]));
		HIPCHK(hipStreamWaitEvent(c->stream, c->xdone[k], 0));
	}
	HIPCHK(hipEventRecord(c->ev1, c->stream));
	HIPCHK(hipEventSynchronize(c->ev1));
	HIPCHK(hipEventElapsedTime(ms, c->ev0, c->ev1));
	return 0;
}

static int time_kernels(mosrx_ctx *c, int op, int arg, const mosrx_batch *b, uint32_t nb, void *const *out,
                        void *const *aux, uint32_t iters, float *avg_ms)
{
	hipEvent_t *ev;
	uint32_t i;
	int rc = 0;
	double tot = 0;
	ev = calloc((size_t)iters * 2, sizeof(*ev));
	if (!ev)
		return -ENOMEM;
	for (i = 0; i < iters * 2 && !rc; i++)
		if (hipEventCreate(&ev[i]) != hipSuccess)
			rc = -EIO;
	for (i = 0; i < iters && !rc; i++) {
		if (hipEventRecord(ev[2 * i], c->stream) != hipSuccess) { rc = -EIO; break; }
		if ((rc = run_op(c, op, arg, &b[i % nb], out ? out[i % nb] : NULL, aux ? aux[i % nb] : NULL, c->stream)))
			break;
		if (hipEventRecord(ev[2 * i + 1], c->stream) != hipSuccess) { rc = -EIO; break; }
	}
	if (!rc && hipStreamSynchronize(c->stream) != hipSuccess)
		rc = -EIO;
	for (i = 0; i < iters && !rc; i++) {
		float ms = 0;
		if (hipEventElapsedTime(&ms, ev[2 * i], ev[2 * i + 1]) != hipSuccess) { rc = -EIO; break; }
		tot += ms;
	}
	for (i = 0; i < iters * 2; i++)
		if (ev[i])
			hipEventDestroy(ev[i]);
	free(ev);
	if (!rc)
		*avg_ms = (float)(tot / iters);
	return rc;
}

int mosrx_time_op(mosrx_ctx *c, int op, int arg, const mosrx_batch *b, uint32_t nb, void *const *out,
                  void *const *aux, uint32_t iters, uint32_t nstreams, float *total_ms, float *avg_kernel_ms)
{
	int rc;
	if (!c || !b || nb == 0 || iters == 0 || nstreams == 0 || nstreams > MOSRX_MAX_STREAMS ||
	    op < MOSRX_OP_CLASSIFY || op > MOSRX_OP_TX_CHECKS || (op != MOSRX_OP_TX_CSUM && !out) ||
	    ((op == MOSRX_OP_CLASSIFY_FH || op == MOSRX_OP_CLASSIFY_BPF || op == MOSRX_OP_CLASSIFY_TI) && !aux))
		return -EINVAL;
	HIPCHK(hipSetDevice(c->device));
	if (total_ms && (rc = time_streams(c, op, arg, b, nb, out, aux, iters, nstreams, total_ms)))
		return rc;
	if (avg_kernel_ms && (rc = time_kernels(c, op, arg, b, nb, out, aux, iters, avg_kernel_ms)))
		return rc;
	return 0;
}

/* One launch of the operation being timed (launch i). */
typedef int (*stamped_fn)(mosrx_ctx *c, uint32_t i, void *arg);

/* Average kernel duration over `iters` back-to-back launches on the context
 * stream, each stamped by its own dispatch (mosrx__stamp_next): -ENOTSUP when
 * a launch of the operation was not exactly one kernel of mosrx_kernels.hip. */
static int time_stamped(mosrx_ctx *c, uint32_t iters, stamped_fn run, void *arg, float *avg_ms)
{
	hipEvent_t *ev;
	uint32_t i;
	int rc = 0;
	double tot = 0;
	ev = calloc((size_t)iters * 2, sizeof(*ev));
	if (!ev)
		return -ENOMEM;
	for (i = 0; i < iters * 2 && !rc; i++)
		if (hipEventCreate(&ev[i]) != hipSuccess)
			rc = -EIO;
	for (i = 0; i < iters && !rc; i++) {
		const uint32_t n0 = mosrx__launch_count();
		mosrx__stamp_next(ev[2 * i], ev[2 * i + 1]);
		rc = run(c, i, arg);
		mosrx__stamp_next(NULL, NULL);
		if (!rc && mosrx__launch_count() - n0 != 1)
			rc = -ENOTSUP;
	}
	if (hipStreamSynchronize(c->stream) != hipSuccess && !rc)
		rc = -EIO;
	for (i = 0; i < iters && !rc; i++) {
		float ms = 0;
		if (hipEventElapsedTime(&ms, ev[2 * i], ev[2 * i + 1]) != hipSuccess) { rc = -EIO; break; }
		tot += ms;
	}
	for (i = 0; i < iters * 2; i++)
		if (ev[i])
			hipEventDestroy(ev[i]);
	free(ev);
	if (!rc)
		*avg_ms = (float)(tot / iters);
	return rc;
}

struct op_run { int op, arg; const mosrx_batch *b; uint32_t nb; void *const *out, *const *aux; };

static int op_once(mosrx_ctx *c, uint32_t i, void *a)
{
	const struct op_run *r = a;
	return run_op(c, r->op, r->arg, &r->b[i % r->nb], r->out ? r->out[i % r->nb] : NULL,
	              r->aux ? r->aux[i % r->nb] : NULL, c->stream);
}

int mosrx_time_op_dispatch(mosrx_ctx *c, int op, int arg, const mosrx_batch *b, uint32_t nb, void *const *out,
                           void *const *aux, uint32_t iters, float *avg_ms)
{
	struct op_run r = {op, arg, b, nb, out, aux};
	if (!c || !b || nb == 0 || iters == 0 || !avg_ms || op < MOSRX_OP_CLASSIFY || op > MOSRX_OP_TX_CHECKS ||
	    (op != MOSRX_OP_TX_CSUM && !out) ||
	    ((op == MOSRX_OP_CLASSIFY_FH || op == MOSRX_OP_CLASSIFY_BPF || op == MOSRX_OP_CLASSIFY_TI) && !aux))
		return -EINVAL;
	/* (the BPF ops are one launch with the fused kernel / the set's own kernel;
	 * classify + the set's kernel, two, is refused by the launch count) */
	HIPCHK(hipSetDevice(c->device));
	return time_stamped(c, iters, op_once, &r, avg_ms);
}

struct queue_run { mosrx_queue *const *q; uint32_t nq; };

static int queue_once(mosrx_ctx *c, uint32_t i, void *a)
{
	const struct queue_run *r = a;
	return mosrx_queue_run(c, r->q[i % r->nq], c->stream);
}

int mosrx_time_queue_dispatch(mosrx_ctx *c, mosrx_queue *const *q, uint32_t nq, uint32_t iters, float *avg_ms)
{
	struct queue_run r = {q, nq};
	if (!c || !q || nq == 0 || iters == 0 || !avg_ms)
		return -EINVAL;
	HIPCHK(hipSetDevice(c->device));
	return time_stamped(c, iters, queue_once, &r, avg_ms);
}

struct empty_run { int kind; uint32_t tiles; };

static int empty_once(mosrx_ctx *c, uint32_t i, void *a)
{
	const struct empty_run *r = a;
	(void)i;
	return mosrx_launch_empty(r->kind, r->tiles, c->stream);
}

int mosrx_probe_stamp_floor(mosrx_ctx *c, const mosrx_batch *b, uint32_t iters, float *avg_ms)
{
	struct empty_run r;
	if (!c || !b || b->n == 0 || iters == 0 || !avg_ms)
		return -EINVAL;
	r.kind = tile_for(c, b);
	r.tiles = (uint32_t)((b->n + MOSRX_KIND_FRAMES(r.kind) - 1) / MOSRX_KIND_FRAMES(r.kind));
	HIPCHK(hipSetDevice(c->device));
	return time_stamped(c, iters, empty_once, &r, avg_ms);
}

int mosrx_time_dev_kernels(mosrx_ctx *c, const mosrx_batch *b, uint32_t nb, mosrx_result *const *d_out,
                           uint32_t iters, float *avg_ms)
{
	if (!avg_ms)
		return -EINVAL;
	return mosrx_time_op(c, MOSRX_OP_CLASSIFY, 0, b, nb, (void *const *)d_out, NULL, iters, 1, NULL, avg_ms);
}

int mosrx_time_dev_streams(mosrx_ctx *c, const mosrx_batch *b, uint32_t nb, mosrx_result *const *d_out,
                           uint32_t iters, uint32_t nstreams, float *ms)
{
	if (!ms)
		return -EINVAL;
	return mosrx_time_op(c, MOSRX_OP_CLASSIFY, 0, b, nb, (void *const *)d_out, NULL, iters, nstreams, ms, NULL);
}

int mosrx_probe_read_bw(mosrx_ctx *c, uint64_t bytes, uint32_t nbuf, uint32_t iters, float *gbps)
{
	void **bufs;
	uint32_t *sink = NULL;
	uint32_t i;
	float ms = 0;
	int rc = 0;
	if (!c || !gbps || nbuf == 0 || iters == 0 || bytes < 16)
		return -EINVAL;
	bytes &= ~(uint64_t)15;
	HIPCHK(hipSetDevice(c->device));
	bufs = calloc(nbuf, sizeof(*bufs));
	if (!bufs)
		return -ENOMEM;
	for (i = 0; i < nbuf && !rc; i++)
		if (hipMalloc(&bufs[i], bytes) != hipSuccess ||
		    hipMemsetAsync(bufs[i], (int)(i + 1), bytes, c->stream) != hipSuccess)
			rc = -ENOMEM;
	if (!rc && hipMalloc((void **)&sink, 4) != hipSuccess)
		rc = -ENOMEM;
	for (i = 0; i < nbuf && !rc; i++)   /* warm-up pass */
		rc = mosrx_launch_read_bw(bufs[i], bytes, sink, c->stream);
	if (!rc && hipEventRecord(c->ev0, c->stream) != hipSuccess)
		rc = -EIO;
	for (i = 0; i < iters && !rc; i++)
		rc = mosrx_launch_read_bw(bufs[i % nbuf], bytes, sink, c->stream);
	if (!rc && (hipEventRecord(c->ev1, c->stream) != hipSuccess || hipEventSynchronize(c->ev1) != hipSuccess ||
	            hipEventElapsedTime(&ms, c->ev0, c->ev1) != hipSuccess))
		rc = -EIO;
	if (!rc)
		*gbps = (float)((double)bytes * iters / (ms * 1e-3) / 1e9);
	hipStreamSynchronize(c->stream);
	for (i = 0; i < nbuf; i++)
		if (bufs[i])
			hipFree(bufs[i]);
	if (sink)
		hipFree(sink);
	free(bufs);
	return rc;
}

int mosrx_device_sync(mosrx_ctx *c)
{
	if (!c)
		return -EINVAL;
	HIPCHK(hipSetDevice(c->device));
	HIPCHK(hipDeviceSynchronize());
	return 0;
}

/* ---- batch queue (one launch over many resident batches) ---- */
struct mosrx_queue {
	mosrx_qdesc *d_desc;
	mosrx_qdesc *h_desc;   /* host copy: the per-batch BPF launches of a queue with masks */
	uint32_t nb;
	uint32_t total_tiles;
	uint32_t tpb;   /* tiles per batch if uniform, else 0 */
	int tile;
	uint64_t bytes, n;   /* frame bytes and frames of all batches (tail policy) */
	int compact;         /* 8-byte records */
	int uni;             /* some batch carries a layout hint */
	int match;           /* the descriptors' bmatch: the installed BPF set's masks */
	uint32_t **d_match;  /* per batch (the non-fused form) */
};

int mosrx_queue_create_ex(mosrx_ctx *c, const mosrx_batch *b, uint32_t nb, void *const *d_out,
                          uint32_t *const *d_fhash, uint32_t *const *d_match, int flags, mosrx_queue **q)
{
	mosrx_qdesc *h;
	mosrx_queue *qq;
	uint32_t i, tiles = 0, maxl = 0, tile;
	uint64_t bytes = 0, frames = 0;
	const int compact = (flags & MOSRX_QUEUE_COMPACT) != 0;
	int rc, unknown = 0, kind;
	if (!c || !b || !d_out || !q || nb == 0 || (flags & ~MOSRX_QUEUE_COMPACT))
		return -EINVAL;
	*q = NULL;
	for (i = 0; i < nb; i++) {
		if ((rc = mosrx__check_batch(&b[i], 1)))
			return rc;
		if (b[i].n && (!d_out[i] || ((uintptr_t)d_out[i] & (compact ? 7 : 15)) ||
		               (d_fhash && (!d_fhash[i] || ((uintptr_t)d_fhash[i] & 3))) ||
		               (d_match && (!d_match[i] || ((uintptr_t)d_match[i] & 3)))))
			return -EINVAL;
		if (!b[i].max_len)
			unknown = 1;
		if (b[i].max_len > maxl)
			maxl = b[i].max_len;
		bytes += b[i].frames_bytes;
		frames += b[i].n;
	}
	kind = kind_of(c, unknown ? 0 : maxl, bytes, frames);   /* one shape for the whole queue */
	tile = MOSRX_KIND_FRAMES(kind);
	h = calloc(nb, sizeof(*h));
	qq = calloc(1, sizeof(*qq));
	if (!h || !qq || (d_match && !(qq->d_match = calloc(nb, sizeof(*qq->d_match))))) {
		free(h);
		if (qq)
			free(qq->d_match);
		free(qq);
		return -ENOMEM;
	}
	for (i = 0; i < nb; i++) {
		h[i].frames = b[i].frames;
		h[i].off = b[i].off;
		h[i].len = b[i].len;
		h[i].out = (mosrx_result *)d_out[i];
		h[i].fhash = d_fhash ? d_fhash[i] : NULL;
		if (d_match) {
			h[i].bmatch = d_match[i];
			qq->d_match[i] = d_match[i];
		}
		h[i].frames_bytes = (uint32_t)b[i].frames_bytes;
		h[i].n = b[i].n;
		h[i].uni = mosrx_uni_pack(&b[i]);
		qq->uni |= h[i].uni != 0;
		h[i].tile_base = tiles;
		tiles += (b[i].n + (uint32_t)tile - 1) / (uint32_t)tile;
	}
	if (hipSetDevice(c->device) != hipSuccess ||
	    hipMalloc((void **)&qq->d_desc, (size_t)nb * sizeof(*h)) != hipSuccess ||
	    hipMemcpy(qq->d_desc, h, (size_t)nb * sizeof(*h), hipMemcpyHostToDevice) != hipSuccess) {
		if (qq->d_desc)
			hipFree(qq->d_desc);
		free(h);
		free(qq->d_match);
		free(qq);
		return -ENOMEM;
	}
	qq->h_desc = h;
	qq->nb = nb;
	qq->total_tiles = tiles;
	qq->tpb = tiles % nb == 0 ? tiles / nb : 0u;
	for (i = 0; i < nb && qq->tpb; i++)
		if ((b[i].n + (uint32_t)tile - 1) / (uint32_t)tile != qq->tpb)
			qq->tpb = 0;
	qq->tile = kind;
	qq->compact = compact;
	qq->match = d_match != NULL;
	qq->bytes = bytes;
	qq->n = frames;
	*q = qq;
	return 0;
}

int mosrx_queue_create(mosrx_ctx *c, const mosrx_batch *b, uint32_t nb, mosrx_result *const *d_out,
                       mosrx_queue **q)
{
	return mosrx_queue_create_ex(c, b, nb, (void *const *)d_out, NULL, NULL, 0, q);
}

int mosrx_queue_run(mosrx_ctx *c, const mosrx_queue *q, void *stream)
{
	mosrx_qparams qp;
	const hipStream_t s = stream ? (hipStream_t)stream : c ? c->stream : NULL;
	const int variant = c ? mosrx__tail_variant(c, q ? q->bytes : 0, q ? q->n : 0) : 0;
	uint32_t i;
	int rc;
	if (!c || !q)
		return -EINVAL;
	qp.desc = q->d_desc;
	qp.tables = c->d_tables;
	qp.counters = NULL;
	qp.nb = q->nb;
	qp.flags = c->kflags;
	qp.tpb = q->tpb;
	qp.tinfo = q->compact ? 2u : 0u;
	qp.uni = (uint32_t)q->uni;
	if (!q->match)
		return mosrx_launch_queue(&qp, q->total_tiles, q->tile, variant, s);
	mosrx__bpf_poll(c);
	if (q->compact ? c->bpf_fu[FU_QS8] && c->bpf_fu[FU_QM8] : c->bpf_fu[FU_QS] && c->bpf_fu[FU_QM])
		return mosrx__bpf_fused_queue_launch(c, &qp, q->total_tiles, q->tile == MOSRX_KIND_SMALL, variant, s);
	if ((rc = mosrx_launch_queue(&qp, q->total_tiles, q->tile, variant, s)))
		return rc;
	for (i = 0; i < q->nb; i++)
		if ((rc = mosrx__bpf_launch_dev(c, q->h_desc[i].frames, q->h_desc[i].frames_bytes, q->h_desc[i].off,
		                                q->h_desc[i].len, q->h_desc[i].n, q->d_match[i], s)))
			return rc;
	return 0;
}

void mosrx_queue_destroy(mosrx_ctx *c, mosrx_queue *q)
{
	if (!q)
		return;
	if (c)
		hipSetDevice(c->device);
	if (q->d_desc)
		hipFree(q->d_desc);
	free(q->h_desc);
	free(q->d_match);
	free(q);
}

int mosrx_time_queue(mosrx_ctx *c, mosrx_queue *const *q, uint32_t nq, uint32_t iters,
                     float *total_ms, float *avg_kernel_ms)
{
	uint32_t i;
	int rc;
	if (!c || !q || nq == 0 || !total_ms || iters == 0)
		return -EINVAL;
	HIPCHK(hipSetDevice(c->device));
	HIPCHK(hipEventRecord(c->ev0, c->stream));
	for (i = 0; i < iters; i++)
		if ((rc = mosrx_queue_run(c, q[i % nq], c->stream)))
			return rc;
	HIPCHK(hipEventRecord(c->ev1, c->stream));
	HIPCHK(hipEventSynchronize(c->ev1));
	HIPCHK(hipEventElapsedTime(total_ms, c->ev0, c->ev1));
	if (avg_kernel_ms) {
		double tot = 0;
		for (i = 0; i < iters && i < 64; i++) {
			float ms = 0;
			HIPCHK(hipEventRecord(c->ev0, c->stream));
			if ((rc = mosrx_queue_run(c, q[i % nq], c->stream)))
				return rc;
			HIPCHK(hipEventRecord(c->ev1, c->stream));
			HIPCHK(hipEventSynchronize(c->ev1));
			HIPCHK(hipEventElapsedTime(&ms, c->ev0, c->ev1));
			tot += ms;
		}
		*avg_kernel_ms = (float)(tot / (i ? i : 1));
	}
	return 0;
}
