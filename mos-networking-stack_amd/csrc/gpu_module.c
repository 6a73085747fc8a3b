/*
 * gpu_module.c — `gpu_module_func`, an io_module_func backend (io_module.h:63-78)
 * that receives frames from a raw-socket / loopback source into pinned
 * staging and classifies each batch on the GPU before the rx loop sees it.
 *
 * recv_pkts (core.c:899) pulls up to `batch` frames into pinned memory, runs
 * H2D -> classify kernel -> D2H (mosrx_classify_host_*), and returns the
 * count; get_rptr (core.c:905) hands out the staged frames; the per-frame
 * verdicts are read through dev_ioctl(MOSRX_PKT_RX_RESULTS) or per packet
 * through dev_ioctl(PKT_RX_RSS) (dpdk_module.c:568-571).  With `pipeline` set,
 * batch k+1 is received and classified while the application consumes batch
 * k, keeping the reference's pointer lifetime (valid until the next recv_pkts).
 * A source that holds its frames in pinned memory lends a run of them as the
 * batch (mosrx_source.h `borrow`, no host copy); one that can copy a run at
 * once fills the stage in runs (`fill`); any other is read frame by frame.
 *
 * Threading follows mOS: one context per mTCP thread, every call for a context
 * from that thread (core.c:1282-1349), so the module takes no locks on the fast
 * path.  Per-thread state is found by context pointer; the module never reads
 * `struct mtcp_thread_context` fields, so it builds against mOS's mtcp.h or
 * standalone.
 */
#include <errno.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/mosrx_io_module.h"
#include "mosrx_source.h"

#define MAX_THREADS 64
#define TX_FRAME_LEN 2048    /* ETHERNET_FRAME_LEN (mtcp.h:64-68) */

/* One pinned block per stage, descriptors first: off[batch] | len[batch] | frames.
 * A full batch is then one contiguous span and crosses PCIe in one copy
 * (mosrx_api.c batch_span). */
struct stage {
	uint8_t *blk;             /* pinned block holding off, len and frames */
	uint8_t *own;             /* the block's frame area */
	uint8_t *frames;          /* this batch's frames: own, or a run borrowed from the source */
	uint32_t *off;
	uint16_t *len;
	mosrx_result *res;        /* pinned */
	uint32_t *match;          /* pinned, BPF match masks (monitor filters configured) */
	uint64_t cap_bytes;
	uint32_t n;
	uint64_t bytes;
};

struct if_state {
	mosrx_ctx *mc;
	struct stage st[MOSRX_NSLOT];
	int cur;                  /* stage exposed to the application, -1 none */
	int inflight;             /* stage being classified, -1 none */
};

struct gpu_priv {
	struct mtcp_thread_context *ctx;
	int cpu;
	struct if_state ifs[MOSRX_MAX_DEVICES];
	uint8_t tx_buf[MOSRX_MAX_DEVICES][TX_FRAME_LEN];
	uint32_t tx_pending[MOSRX_MAX_DEVICES];
	uint64_t tx_packets, tx_bytes;
};

static mosrx_gpu_module_cfg g_cfg;
static int g_configured;
static pthread_mutex_t g_lock = PTHREAD_MUTEX_INITIALIZER;
static struct { struct mtcp_thread_context *ctx; int cpu; struct gpu_priv *priv; } g_tab[MAX_THREADS];
static int g_next_cpu;

void mosrx_gpu_module_cfg_default(mosrx_gpu_module_cfg *cfg)
{
	memset(cfg, 0, sizeof(*cfg));
	cfg->batch = 32768;
	cfg->max_frame = 2048;
	cfg->gpu_base = 0;
	cfg->ngpu = 0;
	cfg->pipeline = 1;
	mosrx_params_default(&cfg->params);
}

int mosrx_gpu_module_configure(const mosrx_gpu_module_cfg *cfg)
{
	if (!cfg || cfg->num_ifs == 0 || cfg->num_ifs > MOSRX_MAX_DEVICES || cfg->batch == 0 ||
	    cfg->max_frame < 64 || cfg->max_frame > 65535)
		return -EINVAL;
	pthread_mutex_lock(&g_lock);
	g_cfg = *cfg;
	g_configured = 1;
	pthread_mutex_unlock(&g_lock);
	return 0;
}

int mosrx_gpu_module_bind(struct mtcp_thread_context *ctx, int cpu)
{
	int i, rc = -ENOSPC;
	pthread_mutex_lock(&g_lock);
	for (i = 0; i < MAX_THREADS; i++)
		if (g_tab[i].ctx == ctx || !g_tab[i].ctx) {
			g_tab[i].ctx = ctx;
			g_tab[i].cpu = cpu;
			rc = 0;
			break;
		}
	pthread_mutex_unlock(&g_lock);
	return rc;
}

static struct gpu_priv *priv_of(struct mtcp_thread_context *ctx)
{
	int i;
	for (i = 0; i < MAX_THREADS && g_tab[i].ctx; i++)
		if (g_tab[i].ctx == ctx)
			return g_tab[i].priv;
	return NULL;
}

static void gpu_load_module_upper_half(void)
{
	if (!g_configured) {
		fprintf(stderr, "[mosrx] gpu_module: mosrx_gpu_module_configure() not called\n");
		exit(EXIT_FAILURE);   /* fatal init error, as pcap_module.c:141-155 */
	}
}

static void stage_free(mosrx_ctx *mc, struct stage *s)
{
	if (s->blk) mosrx_host_free(mc, s->blk);
	if (s->res) mosrx_host_free(mc, s->res);
	if (s->match) mosrx_host_free(mc, s->match);
	memset(s, 0, sizeof(*s));
}

static void gpu_destroy_handle(struct mtcp_thread_context *ctx);

static void gpu_init_handle(struct mtcp_thread_context *ctx)
{
	struct gpu_priv *pv;
	int i, k, cpu = -1, ngpu, slot = -1;

	pthread_mutex_lock(&g_lock);
	for (i = 0; i < MAX_THREADS; i++) {
		if (g_tab[i].ctx == ctx) { slot = i; cpu = g_tab[i].cpu; break; }
		if (!g_tab[i].ctx) { slot = i; g_tab[i].ctx = ctx; cpu = g_tab[i].cpu = g_next_cpu; break; }
	}
	g_next_cpu++;
	pthread_mutex_unlock(&g_lock);
	if (slot < 0) {
		fprintf(stderr, "[mosrx] gpu_module: too many threads\n");
		exit(EXIT_FAILURE);
	}
	pv = calloc(1, sizeof(*pv));
	if (!pv)
		exit(EXIT_FAILURE);
	pv->ctx = ctx;
	pv->cpu = cpu;
	ngpu = g_cfg.ngpu;
	for (i = 0; i < (int)g_cfg.num_ifs; i++) {
		struct if_state *is = &pv->ifs[i];
		int dev = g_cfg.gpu_base + (ngpu > 0 ? cpu % ngpu : cpu);
		int rc = mosrx_open(dev, &g_cfg.params, &is->mc);
		if (rc && ngpu <= 0)
			rc = mosrx_open(g_cfg.gpu_base, &g_cfg.params, &is->mc);
		if (rc) {
			fprintf(stderr, "[mosrx] gpu_module: mosrx_open(%d): %s\n", dev, mosrx_strerror(rc));
			exit(EXIT_FAILURE);
		}
		is->cur = is->inflight = -1;
		if (g_cfg.bpf_nprog && (rc = mosrx_bpf_set(is->mc, g_cfg.bpf_progs, g_cfg.bpf_nprog))) {
			fprintf(stderr, "[mosrx] gpu_module: mosrx_bpf_set: %s\n", mosrx_strerror(rc));
			exit(EXIT_FAILURE);
		}
		for (k = 0; k < MOSRX_NSLOT; k++) {
			struct stage *s = &is->st[k];
			const uint64_t dsc = ((uint64_t)g_cfg.batch * 6 + 15) & ~15ull;
			s->cap_bytes = (uint64_t)g_cfg.batch * ((g_cfg.max_frame + 15u + 16u) & ~15u) + 64;
			if (mosrx_host_alloc(is->mc, dsc + s->cap_bytes, (void **)&s->blk) ||
			    mosrx_host_alloc(is->mc, (size_t)g_cfg.batch * sizeof(mosrx_result), (void **)&s->res) ||
			    (g_cfg.bpf_nprog && mosrx_host_alloc(is->mc, (size_t)g_cfg.batch * 4, (void **)&s->match))) {
				fprintf(stderr, "[mosrx] gpu_module: pinned staging allocation failed\n");
				exit(EXIT_FAILURE);
			}
			s->off = (uint32_t *)s->blk;
			s->len = (uint16_t *)(s->blk + (size_t)g_cfg.batch * 4);
			s->own = s->frames = s->blk + dsc;
		}
	}
	g_tab[slot].priv = pv;
}

/* Receive up to `batch` frames from the netdev's source into stage s. */
static void stage_fill(struct stage *s, mosrx_source *src)
{
	uint64_t pos = 2;
	uint32_t i = 0;
	const uint32_t mf = g_cfg.max_frame;
	s->frames = s->own;
	if (src && src->borrow) {     /* zero-copy: the source's pinned run is the batch */
		const uint8_t *f = NULL;
		uint64_t fb = 0;
		s->n = src->borrow(src, g_cfg.batch, mf, &f, &fb, s->off, s->len);
		if (s->n) {
			s->frames = (uint8_t *)f;
			s->bytes = fb;
		} else {
			s->bytes = 2;
		}
		return;
	}
	if (src && src->fill) {
		s->n = src->fill(src, s->frames, s->cap_bytes, s->off, s->len, g_cfg.batch, mf, &s->bytes);
		return;
	}
	while (i < g_cfg.batch && src && pos + mf + 16 <= s->cap_bytes) {
		int l = src->next(src, s->frames + pos, mf);
		if (l <= 0)
			break;
		s->off[i] = (uint32_t)pos;
		s->len[i] = (uint16_t)l;
		i++;
		pos = ((pos + (uint64_t)l - 2 + 15) & ~15ull) + 2;   /* next frame at 16 B + 2 */
	}
	s->n = i;
	s->bytes = pos;
}

static int stage_submit(struct if_state *is, int k)
{
	struct stage *s = &is->st[k];
	mosrx_batch b;
	b.frames = s->frames;
	b.frames_bytes = s->bytes;
	b.off = s->off;
	b.len = s->len;
	b.n = s->n;
	b.max_len = g_cfg.max_frame;
	if (g_cfg.bpf_nprog)
		return mosrx_classify_bpf_host_submit(is->mc, k, &b, s->res, s->match);
	return mosrx_classify_host_submit(is->mc, k, &b, s->res);
}

static int32_t gpu_recv_pkts(struct mtcp_thread_context *ctx, int ifidx)
{
	struct gpu_priv *pv = priv_of(ctx);
	struct if_state *is;
	mosrx_source *src;
	int k;

	if (!pv || ifidx < 0 || ifidx >= (int)g_cfg.num_ifs)
		return -1;
	is = &pv->ifs[ifidx];
	src = g_cfg.src[ifidx];
	if (is->inflight < 0) {           /* nothing in flight: receive + classify now */
		k = is->cur < 0 ? 0 : is->cur ^ 1;
		stage_fill(&is->st[k], src);
		if (stage_submit(is, k))
			return -1;
		is->inflight = k;
	}
	k = is->inflight;
	if (mosrx_classify_host_wait(is->mc, k))
		return -1;
	is->cur = k;
	is->inflight = -1;
	if (g_cfg.pipeline && is->st[k].n) {   /* classify the next batch behind the app's work */
		int nk = k ^ 1;
		stage_fill(&is->st[nk], src);
		if (is->st[nk].n && stage_submit(is, nk) == 0)
			is->inflight = nk;
	}
	return (int32_t)is->st[k].n;
}

static uint8_t *gpu_get_rptr(struct mtcp_thread_context *ctx, int ifidx, int index, uint16_t *len)
{
	struct gpu_priv *pv = priv_of(ctx);
	struct stage *s;
	if (!pv || ifidx < 0 || ifidx >= (int)g_cfg.num_ifs || pv->ifs[ifidx].cur < 0)
		return NULL;
	s = &pv->ifs[ifidx].st[pv->ifs[ifidx].cur];
	if (index < 0 || (uint32_t)index >= s->n)
		return NULL;
	*len = s->len[index];
	return s->frames + s->off[index];
}

static void gpu_release_pkt(struct mtcp_thread_context *ctx, int ifidx, unsigned char *pkt, int len)
{
	/* staging is recycled wholesale on the next recv_pkts */
	(void)ctx; (void)ifidx; (void)pkt; (void)len;
}

static uint8_t *gpu_get_wptr(struct mtcp_thread_context *ctx, int ifidx, uint16_t len)
{
	struct gpu_priv *pv = priv_of(ctx);
	if (!pv || ifidx < 0 || ifidx >= MOSRX_MAX_DEVICES || len > TX_FRAME_LEN)
		return NULL;
	pv->tx_pending[ifidx] = len;
	return pv->tx_buf[ifidx];
}

/* TX is out of scope for the rx classifier: frames handed to send_pkts are
 * counted and dropped, like a pcap_inject to a closed interface. */
static int32_t gpu_send_pkts(struct mtcp_thread_context *ctx, int nif)
{
	struct gpu_priv *pv = priv_of(ctx);
	if (!pv || nif < 0 || nif >= MOSRX_MAX_DEVICES)
		return 0;
	if (pv->tx_pending[nif]) {
		pv->tx_packets++;
		pv->tx_bytes += pv->tx_pending[nif];
		pv->tx_pending[nif] = 0;
		return 1;
	}
	return 0;
}

static int gpu_get_nif(struct ifreq *ifr)
{
	uint32_t i;
	for (i = 0; i < g_cfg.num_ifs; i++)
		if (!strncmp(ifr->ifr_name, g_cfg.if_names[i], IFNAMSIZ))
			return (int)i;
	return -1;
}

static int32_t gpu_dev_ioctl(struct mtcp_thread_context *ctx, int nif, int cmd, void *argp)
{
	struct gpu_priv *pv = priv_of(ctx);
	struct stage *s;
	if (!pv || !argp || nif < 0 || nif >= (int)g_cfg.num_ifs)
		return -1;
	switch (cmd) {
	case PKT_RX_RSS: {
		RssInfo *ri = argp;
		if (pv->ifs[nif].cur < 0)
			return -1;
		s = &pv->ifs[nif].st[pv->ifs[nif].cur];
		if (ri->pktidx < 0 || (uint32_t)ri->pktidx >= s->n)
			return -1;
		ri->hash_value = s->res[ri->pktidx].rss;
		return 0;
	}
	case MOSRX_PKT_RX_RESULTS:
		if (pv->ifs[nif].cur < 0)
			return -1;
		*(const mosrx_result **)argp = pv->ifs[nif].st[pv->ifs[nif].cur].res;
		return 0;
	case MOSRX_PKT_RX_MATCH:
		if (pv->ifs[nif].cur < 0 || !g_cfg.bpf_nprog)
			return -1;
		*(const uint32_t **)argp = pv->ifs[nif].st[pv->ifs[nif].cur].match;
		return 0;
	case DRV_NAME:
		*(const char **)argp = "mosrx_gpu";
		return 0;
	default:   /* PKT_TX_*_CSUM: not offloaded, the stack computes them (ip_out.c:169-174) */
		return -1;
	}
}

static void gpu_destroy_handle(struct mtcp_thread_context *ctx)
{
	struct gpu_priv *pv = priv_of(ctx);
	uint32_t i;
	int k;
	if (!pv)
		return;
	for (i = 0; i < g_cfg.num_ifs; i++) {
		struct if_state *is = &pv->ifs[i];
		if (!is->mc)
			continue;
		if (is->inflight >= 0)
			mosrx_classify_host_wait(is->mc, is->inflight);
		for (k = 0; k < MOSRX_NSLOT; k++)
			stage_free(is->mc, &is->st[k]);
		mosrx_close(is->mc);
	}
	pthread_mutex_lock(&g_lock);
	for (k = 0; k < MAX_THREADS; k++)
		if (g_tab[k].ctx == ctx)
			g_tab[k].priv = NULL;
	pthread_mutex_unlock(&g_lock);
	free(pv);
}

io_module_func gpu_module_func = {
	.load_module_upper_half = gpu_load_module_upper_half,
	.load_module_lower_half = NULL,
	.init_handle            = gpu_init_handle,
	.link_devices           = NULL,
	.release_pkt            = gpu_release_pkt,
	.get_wptr               = gpu_get_wptr,
	.set_wptr               = NULL,
	.send_pkts              = gpu_send_pkts,
	.get_rptr               = gpu_get_rptr,
	.get_nif                = gpu_get_nif,
	.recv_pkts              = gpu_recv_pkts,
	.select                 = NULL,
	.destroy_handle         = gpu_destroy_handle,
	.dev_ioctl              = gpu_dev_ioctl,
};
