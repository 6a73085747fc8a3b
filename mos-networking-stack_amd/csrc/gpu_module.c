/*
 * gpu_module.c — `gpu_module_func`, an io_module_func backend (io_module.h:63-78)
 * that receives frames from a raw-socket / loopback source into pinned
 * staging and classifies each batch on the GPU before the rx loop sees it.
 * It is the peer of pcap_module_func (pcap_module.c:162-177): frames come in
 * through recv_pkts / get_rptr and go out through get_wptr / send_pkts.
 *
 * recv_pkts (core.c:899) hands out the next classified batch; get_rptr
 * (core.c:905) the staged frames; the per-frame verdicts are read through
 * dev_ioctl(MOSRX_PKT_RX_RESULTS) or per packet through dev_ioctl(PKT_RX_RSS)
 * (dpdk_module.c:568-571).  Batches are received in groups (cfg.group: a
 * fixed count, or MOSRX_GROUP_AUTO, the default: every batch the source has
 * ready, up to cfg.group_bytes of frames): a group's batches are staged back
 * to back in one pinned block and classified by ONE kernel launch (the batch
 * queue), then handed out one per recv_pkts, so small batches do not pay a
 * launch each.  cfg.group_max_us bounds a group by time as well: no more
 * frames than the measured PCIe + classify rate moves, or the host's rx loop
 * walks, within that many microseconds (group_cap), so a frame's residency
 * stays near a few times the budget at any load.
 * With `pipeline` set, the next group is received and classified while the
 * application consumes the current one, keeping the reference's pointer
 * lifetime (valid until the next recv_pkts).  A source that holds its frames
 * in pinned memory lends a run of them as the batch (mosrx_source.h `borrow`,
 * no host copy; the run goes back with `give_back` when its group is
 * recycled); one that can copy a run at once fills the stage in runs (`fill`);
 * any other is read frame by frame.
 *
 * TX: get_wptr (eth_out.c:80-84, :118-123) returns a slot of the netdev's TX
 * buffer; send_pkts (core.c:1004-1006) hands every buffered frame to the
 * netdev's source (AF_PACKET send = pcap_inject, or a pcap dump), as
 * pcap_send_pkts does (pcap_module.c:67-79); a full buffer is flushed by the
 * next get_wptr, like dpdk_get_wptr.  With cfg.tx_csum the module takes mOS's
 * checksum offload requests the way dpdk_dev_ioctl does (PKT_TX_IP_CSUM /
 * PKT_TX_TCP_CSUM on the frame get_wptr handed out last, dpdk_module.c:556-566;
 * mOS then skips ip_fast_csum / TCPCalcChecksum, ip_out.c:169-174,
 * tcp_out.c:207-218) and send_pkts fills those checks on the GPU (the TX
 * rewrite kernel, mosrx_tx_csum_host) before the frames leave.
 *
 * Threading follows mOS: one context per mTCP thread, every call for a context
 * from that thread (core.c:1282-1349), so the module takes no locks on the fast
 * path.  Per-thread state is found by context pointer.  Inside an mOS build
 * the module reads two fields of `struct mtcp_thread_context`: `cpu` (the
 * mTCP core, which picks the thread's GPU and per-thread source when the
 * application did not bind the context) and `mtcp_manager` (the stack state it
 * follows, mos_state); standalone it never dereferences the context, so it
 * builds against mOS's mtcp.h or without it.
 */
#include <errno.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "../../include/mosrx_io_module.h"
#include "mosrx_source.h"
#ifdef MOSRX_HAVE_MOS_IO_MODULE
#include "config.h"    /* g_config, num_queues (config.h:160-170) */
#include "mtcp.h"      /* mtcp_thread_context.mtcp_manager -> num_msp / num_esp (mtcp.h:243-244, :304-312) */
#endif

#define MAX_THREADS 64
#define TX_FRAME_LEN 2048    /* ETHERNET_FRAME_LEN (mtcp.h:64-68) */

/* One stage = one batch: off[batch] | len[batch] | frames, inside its group's
 * pinned block.  A group's stages are packed back to back, so a whole group is
 * (nearly) one contiguous span and crosses PCIe in one copy. */
struct stage {
	uint8_t *frames;          /* this batch's frames: in the group block, or a run borrowed from the source */
	uint32_t *off;
	uint16_t *len;
	mosrx_result *res;        /* pinned, in the group's record array */
	mosrx_tcpinfo *ti;        /* pinned, pkt_info TCP fields (cfg.tcpinfo) */
	uint32_t *match;          /* pinned, BPF match masks (a filter set installed) */
	uint32_t *fh;             /* pinned, flow-table hashes (cfg.flowhash) */
	uint32_t n, max_len;
	uint32_t rec0;            /* its first record's index in the group's record arrays */
	uint32_t stride;          /* frame i at off[0] + i * stride (a fixed-size packing), else 0: the layout hint */
	uint64_t bytes;
	int borrowed;             /* frames lent by the source: give them back when the group is recycled */
	/* what its records were made under: mOS's socket counts, the netdev's
	 * parameter / filter generation, the programs behind its masks, and
	 * which side arrays the launch filled (pkt_info fields are not made in a
	 * BPF pass) */
	uint32_t msp, esp, gen, nprog, has_fh, has_ti;
	int compact;              /* its records are mosrx_result8 (cfg.compact): RES8 */
};
/* A compact stage's records: group_submit re-points s->res into the group's
 * array of 8-byte slots (packed back to back, so they come back in one copy);
 * between group_fill and that submit s->res still points at a 16-byte slot, so
 * RES8 is meaningful only once the stage was submitted (s->compact set). */
#define RES8(s) ((mosrx_result8 *)(s)->res)

struct group {
	uint8_t *blk;             /* pinned block the group's stages are packed into */
	uint64_t blk_bytes;
	mosrx_result *res;        /* pinned, rec_cap records */
	mosrx_tcpinfo *ti;
	uint32_t *match;
	uint32_t *fh;
	uint64_t rec_cap;         /* frames the record arrays hold */
	struct stage *st;         /* cap_st stages */
	uint32_t cap_st;
	uint32_t nst;             /* stages filled */
};

struct if_state {
	mosrx_ctx *mc;
	mosrx_params params;      /* the context's stack state (SET_PARAMS, or mOS's own counts) */
	mosrx_source *src;
	struct group g[MOSRX_NSLOT];
	int cur;                  /* group exposed to the application, -1 none */
	uint32_t cur_idx;         /* its batch exposed now */
	int inflight;             /* group being classified, -1 none */
	uint32_t gen;             /* bumped by SET_PARAMS / SET_BPF: older records are classified again */
	/* the latency cap's rates (cfg.group_max_us), EWMAs: a group's submit ->
	 * records ready per frame byte, and the host's time per frame from a group's
	 * exposure to the recv_pkts that moves past it (the app's walk + the next
	 * group's fill and submit) */
	double ns_per_byte, ns_per_frame;
	uint64_t t_submit[MOSRX_NSLOT], t_expose;
	uint64_t cap_frames_last; /* the cap the last group_fill applied (UINT64_MAX: none) */
	uint32_t nprog;           /* programs of the installed BPF set (0: none) */
	/* TX: frames written through get_wptr, sent by send_pkts */
	uint8_t *tx_buf;          /* tx_cap x TX_FRAME_LEN */
	uint16_t *tx_len;
	uint8_t *tx_fl;           /* per TX frame: checks requested through dev_ioctl (TXF_*) */
	uint32_t *tx_poff;        /* the TX rewrite's descriptors (tx_cap each) */
	uint16_t *tx_plen;
	uint32_t tx_n;
	mosrx_ctx *mc_tx;         /* the TX rewrite's own context (opened on first use) */
};
#define TXF_IP  1u            /* PKT_TX_IP_CSUM */
#define TXF_TCP 2u            /* PKT_TX_TCP_CSUM */

struct gpu_priv {
	struct mtcp_thread_context *ctx;
	int cpu;
	struct if_state ifs[MOSRX_MAX_DEVICES];
	mosrx_gpu_module_stats stats;
};

static mosrx_gpu_module_cfg g_cfg;
static int g_configured;
static pthread_mutex_t g_lock = PTHREAD_MUTEX_INITIALIZER;
static struct { struct mtcp_thread_context *ctx; int cpu; struct gpu_priv *priv; } g_tab[MAX_THREADS];
static mosrx_source *g_src_cpu[MAX_THREADS][MOSRX_MAX_DEVICES];
static int g_next_cpu;

void mosrx_gpu_module_cfg_default(mosrx_gpu_module_cfg *cfg)
{
	memset(cfg, 0, sizeof(*cfg));
	cfg->batch = 32768;
	cfg->max_frame = 2048;
	cfg->gpu_base = 0;
	cfg->ngpu = 0;
	cfg->pipeline = 1;
	cfg->tx_batch = 64;
	cfg->group = MOSRX_GROUP_AUTO;
	cfg->group_bytes = 0;
	cfg->numa = 1;
	cfg->direct_kb = MOSRX_DIRECT_DEFAULT_KB;
	cfg->direct_frames = MOSRX_DIRECT_DEFAULT_FRAMES;
	mosrx_params_default(&cfg->params);
}

int mosrx_gpu_module_configure(const mosrx_gpu_module_cfg *cfg)
{
	if (!cfg || cfg->num_ifs == 0 || cfg->num_ifs > MOSRX_MAX_DEVICES || cfg->batch == 0 ||
	    cfg->max_frame < 64 || cfg->max_frame > 65535 || cfg->group > MOSRX_MAX_GROUP ||
	    cfg->bpf_nprog > MOSRX_BPF_MAX_PROGS || cfg->params.num_local > MOSRX_MAX_LOCAL ||
	    (cfg->compact && cfg->tcpinfo) || cfg->direct_kb > (1u << 22))
		return -EINVAL;
	pthread_mutex_lock(&g_lock);
	g_cfg = *cfg;
	if (!g_cfg.tx_batch)
		g_cfg.tx_batch = 64;
	g_configured = 1;
	pthread_mutex_unlock(&g_lock);
	return 0;
}

int mosrx_gpu_module_get_cfg(mosrx_gpu_module_cfg *cfg)
{
	if (!cfg || !g_configured)
		return -EINVAL;
	pthread_mutex_lock(&g_lock);
	*cfg = g_cfg;
	pthread_mutex_unlock(&g_lock);
	return 0;
}

int mosrx_gpu_module_bind(struct mtcp_thread_context *ctx, int cpu)
{
	int i, rc = -ENOSPC;
	pthread_mutex_lock(&g_lock);
	if (!ctx || cpu < 0) {
		pthread_mutex_unlock(&g_lock);
		return -EINVAL;
	}
	for (i = 0; i < MAX_THREADS; i++)     /* this context's slot, else the first free one */
		if (g_tab[i].ctx == ctx)
			break;
	if (i == MAX_THREADS)
		for (i = 0; i < MAX_THREADS && g_tab[i].ctx; i++)
			;
	if (i < MAX_THREADS) {
		g_tab[i].ctx = ctx;
		g_tab[i].cpu = cpu;
		rc = 0;
	}
	pthread_mutex_unlock(&g_lock);
	return rc;
}

int mosrx_gpu_module_bind_source(int cpu, int ifidx, mosrx_source *src)
{
	if (cpu < 0 || cpu >= MAX_THREADS || ifidx < 0 || ifidx >= MOSRX_MAX_DEVICES)
		return -EINVAL;
	pthread_mutex_lock(&g_lock);
	g_src_cpu[cpu][ifidx] = src;
	pthread_mutex_unlock(&g_lock);
	return 0;
}

/* NUMA node of HIP device d, looked up once (-1: unknown or not a device). */
#define NODE_CACHE 64
static int g_gpu_node[NODE_CACHE];
static int g_gpu_node_known[NODE_CACHE];
static int gpu_node_of(int d)
{
	int n;
	if (d < 0 || d >= NODE_CACHE)
		return -1;
	pthread_mutex_lock(&g_lock);
	if (!g_gpu_node_known[d]) {
		g_gpu_node[d] = mosrx_gpu_numa_node(d);
		g_gpu_node_known[d] = 1;
	}
	n = g_gpu_node[d];
	pthread_mutex_unlock(&g_lock);
	return n;
}

/* Per-core sharding: thread `cpu` drives a GPU on its NUMA
 * node (topology.c: round robin over the node's GPUs), else gpu_base + cpu % ngpu. */
int mosrx_gpu_module_device_of(int cpu, int ndev)
{
	const int ngpu = g_cfg.ngpu > 0 ? g_cfg.ngpu : ndev - g_cfg.gpu_base;
	int dev, k;
	if (cpu < 0 || ngpu <= 0)
		return -EINVAL;
	dev = g_cfg.gpu_base + cpu % ngpu;
	if (g_cfg.numa && ngpu <= NODE_CACHE) {
		int nodes[NODE_CACHE], i;
		for (i = 0; i < ngpu; i++)
			nodes[i] = g_cfg.gpu_base + i < ndev ? gpu_node_of(g_cfg.gpu_base + i) : -1;
		if ((k = mosrx_numa_pick(cpu, nodes, ngpu)) >= 0)
			dev = g_cfg.gpu_base + k;
	}
	return dev < ndev ? dev : -EINVAL;
}

/* Slots are freed by destroy_handle, so the table can have holes: scan it all. */
static struct gpu_priv *priv_of(struct mtcp_thread_context *ctx)
{
	int i;
	if (!ctx)
		return NULL;
	for (i = 0; i < MAX_THREADS; i++)
		if (g_tab[i].ctx == ctx)
			return g_tab[i].priv;
	return NULL;
}

int mosrx_gpu_module_set_timing(struct mtcp_thread_context *ctx, int on)
{
	struct gpu_priv *pv = priv_of(ctx);
	uint32_t i;
	if (!pv)
		return -EINVAL;
	for (i = 0; i < g_cfg.num_ifs; i++)
		if (pv->ifs[i].mc)
			mosrx_set_timing(pv->ifs[i].mc, on);
	return 0;
}

int mosrx_gpu_module_stats_of(struct mtcp_thread_context *ctx, mosrx_gpu_module_stats *st)
{
	struct gpu_priv *pv = priv_of(ctx);
	if (!pv || !st)
		return -EINVAL;
	*st = pv->stats;
	/* netdev 0's latency-cap state */
	st->group_cap_frames = pv->ifs[0].cap_frames_last == UINT64_MAX ? 0 : pv->ifs[0].cap_frames_last;
	st->ns_per_frame_host = pv->ifs[0].ns_per_frame;
	st->ns_per_byte_dev = pv->ifs[0].ns_per_byte;
	return 0;
}

#ifdef MOSRX_HAVE_MOS_IO_MODULE
/* Not configured by the application: do what pcap_load_module_upper_half does
 * (pcap_module.c:124-160) -- one capture per netdev of mOS's configuration,
 * here an AF_PACKET ring -- with the defaults (groups sized to what the ring
 * has ready, num_queues 1 as pcap_module.c:159). */
static void gpu_configure_from_mos(void)
{
	mosrx_gpu_module_cfg cfg;
	const struct netdev_conf *nd = g_config.mos->netdev_table;
	int i;
	mosrx_gpu_module_cfg_default(&cfg);
	if (nd->num <= 0 || nd->num > MOSRX_MAX_DEVICES) {
		fprintf(stderr, "[mosrx] gpu_module: %d netdevs (1..%d supported)\n", nd->num, MOSRX_MAX_DEVICES);
		exit(EXIT_FAILURE);
	}
	cfg.num_ifs = (uint32_t)nd->num;
	cfg.compact = 1;   /* mOS's consumer (mos_rx.c) reads 8-byte records */
	for (i = 0; i < nd->num; i++) {
		char var[64];
		const char *pcap, *tx;
		strncpy(cfg.if_names[i], nd->ent[i]->dev_name, sizeof(cfg.if_names[i]) - 1);
		/* offline replay: MOSRX_PCAP_<netdev>=file reads a capture instead of the
		 * interface (MOSRX_PCAP_LOOPS times, default 1), MOSRX_TX_PCAP_<netdev>=file
		 * dumps what mOS sends on it -- an unmodified mOS application run over a
		 * recorded trace, e.g. BASELINE config #1's simple_firewall */
		snprintf(var, sizeof(var), "MOSRX_PCAP_%s", cfg.if_names[i]);
		pcap = getenv(var);
		if (pcap) {
			const char *loops = getenv("MOSRX_PCAP_LOOPS");
			cfg.src[i] = mosrx_source_pcap(pcap, loops ? (uint32_t)strtoul(loops, NULL, 10) : 1);
		} else {
			cfg.src[i] = mosrx_source_afpacket(cfg.if_names[i]);
		}
		if (!cfg.src[i]) {   /* as pcap_create failing (pcap_module.c:140-144) */
			fprintf(stderr, "[mosrx] gpu_module: %s '%s' not found (or no CAP_NET_RAW)\n",
			        pcap ? "capture" : "interface", pcap ? pcap : cfg.if_names[i]);
			exit(EXIT_FAILURE);
		}
		snprintf(var, sizeof(var), "MOSRX_TX_PCAP_%s", cfg.if_names[i]);
		if ((tx = getenv(var)) && mosrx_source_tx_pcap(cfg.src[i], tx)) {
			fprintf(stderr, "[mosrx] gpu_module: TX dump '%s' cannot be written\n", tx);
			exit(EXIT_FAILURE);
		}
	}
	if (mosrx_gpu_module_configure(&cfg))
		exit(EXIT_FAILURE);
}
#endif

static void gpu_load_module_upper_half(void)
{
#ifdef MOSRX_HAVE_MOS_IO_MODULE
	if (!g_configured)
		gpu_configure_from_mos();
#endif
	if (!g_configured) {
		fprintf(stderr, "[mosrx] gpu_module: mosrx_gpu_module_configure() not called\n");
		exit(EXIT_FAILURE);   /* fatal init error, as pcap_module.c:141-155 */
	}
#ifdef MOSRX_HAVE_MOS_IO_MODULE
	{
		/* the stack state the verdicts depend on, from mOS's own configuration:
		 * forward (eth_in.c:22) and the netdevs' addresses (icmp.c:193-200) */
		int i;
		g_cfg.params.forward = g_config.mos->forward;
		if (!g_cfg.params.num_local)
			for (i = 0; i < g_config.mos->netdev_table->num && i < MOSRX_MAX_LOCAL; i++)
				g_cfg.params.local_ip[g_cfg.params.num_local++] = g_config.mos->netdev_table->ent[i]->ip_addr;
	}
	/* GetRSSCPUCore's queue count (util.c:114-131, api.c:1056): every backend
	 * sets it (pcap_module.c:159, dpdk_module.c:704, :800) */
	num_queues = g_cfg.params.num_queues;
#endif
}

/* The stack state ProcessPacket would see right now: inside an mOS build the
 * thread's mtcp_manager counts its monitor and end-host sockets (num_msp /
 * num_esp, incremented by socket creation, socket.c:77-78), and the backend
 * follows them with no call from the core; standalone, 0 (the application
 * passes changes with dev_ioctl(MOSRX_PKT_SET_PARAMS)). */
static int mos_state(const struct gpu_priv *pv, uint32_t *msp, uint32_t *esp)
{
#ifdef MOSRX_HAVE_MOS_IO_MODULE
	const struct mtcp_manager *m = pv->ctx ? pv->ctx->mtcp_manager : NULL;
	if (m) {
		*msp = m->num_msp;
		*esp = m->num_esp;
		return 1;
	}
#else
	(void)pv; (void)msp; (void)esp;
#endif
	return 0;
}

/* Bring the context's stack state up to mOS's before a launch. */
static int follow_mos_state(struct gpu_priv *pv, struct if_state *is)
{
	uint32_t msp, esp;
	if (mos_state(pv, &msp, &esp) && (msp != is->params.num_msp || esp != is->params.num_esp)) {
		is->params.num_msp = msp;
		is->params.num_esp = esp;
		return mosrx_set_params(is->mc, &is->params);
	}
	return 0;
}

static void group_free(mosrx_ctx *mc, struct group *g)
{
	if (g->blk) mosrx_host_free(mc, g->blk);
	if (g->res) mosrx_host_free(mc, g->res);
	if (g->ti) mosrx_host_free(mc, g->ti);
	if (g->match) mosrx_host_free(mc, g->match);
	if (g->fh) mosrx_host_free(mc, g->fh);
	free(g->st);
	memset(g, 0, sizeof(*g));
}

/* Room one stage may take in the block: descriptors + the largest frames. */
static uint64_t stage_bytes(void)
{
	const uint64_t dsc = ((uint64_t)g_cfg.batch * 6 + 15) & ~15ull;
	return dsc + (uint64_t)g_cfg.batch * ((g_cfg.max_frame + 15u + 16u) & ~15u) + 512;
}

/* Frame bytes an auto group's block holds.  cfg.group_bytes, else
 * MOSRX_GROUP_AUTO_BYTES; inside mOS, where every mTCP thread holds two such
 * blocks per netdev (pinned), the default is scaled so that all of them
 * together stay near MOSRX_PINNED_BUDGET (mos.conf's num_cores x netdevs),
 * never under MOSRX_GROUP_AUTO_MIN_BYTES.  INTEGRATION.md §5 gives the
 * footprint. */
#define MOSRX_PINNED_BUDGET        (4ull << 30)
#define MOSRX_GROUP_AUTO_MIN_BYTES (32ull << 20)
static uint64_t auto_bytes(void)
{
	uint64_t b = MOSRX_GROUP_AUTO_BYTES;
	if (g_cfg.group_bytes)
		return g_cfg.group_bytes;
#ifdef MOSRX_HAVE_MOS_IO_MODULE
	if (g_config.mos && g_config.mos->num_cores > 0) {
		const uint64_t per = MOSRX_PINNED_BUDGET / ((uint64_t)g_config.mos->num_cores * g_cfg.num_ifs * MOSRX_NSLOT);
		if (per < b)
			b = per < MOSRX_GROUP_AUTO_MIN_BYTES ? MOSRX_GROUP_AUTO_MIN_BYTES : per;
	}
#endif
	return b;
}

/* Explicit groups reserve `group` worst-case stages.  Auto groups hold up to
 * MOSRX_MAX_GROUP stages in a block of auto_bytes(): stages are packed by the
 * bytes their frames really take, the last one stops where the block is full
 * (a short batch, which ends the group), and records are there for the
 * frames that can fit (a staged frame takes >= 64 bytes of block).  When the
 * host cannot pin that much, the block is halved until it can, down to one
 * worst-case batch: smaller groups, not a dead mTCP thread. */
/* The BPF match arrays: with the group when filters are configured, and
 * always inside mOS, where a monitor can bind a filter at any time -- pinning
 * them at the first bind would stall the mTCP thread for milliseconds. */
#ifdef MOSRX_HAVE_MOS_IO_MODULE
#define MATCH_UP_FRONT 1
#else
#define MATCH_UP_FRONT (g_cfg.bpf_nprog != 0)
#endif

static int group_alloc_sized(mosrx_ctx *mc, struct group *g, uint64_t bytes)
{
	memset(g, 0, sizeof(*g));
	if (g_cfg.group == MOSRX_GROUP_AUTO) {
		g->cap_st = MOSRX_MAX_GROUP;
		g->blk_bytes = bytes;
		g->rec_cap = bytes / 64 + g_cfg.batch;
		if (g->rec_cap > (uint64_t)g_cfg.batch * MOSRX_MAX_GROUP)
			g->rec_cap = (uint64_t)g_cfg.batch * MOSRX_MAX_GROUP;
	} else {
		g->cap_st = (uint32_t)(bytes / stage_bytes());
		g->blk_bytes = stage_bytes() * g->cap_st;
		g->rec_cap = (uint64_t)g_cfg.batch * g->cap_st;
	}
	g->st = calloc(g->cap_st, sizeof(*g->st));
	if (!g->st || mosrx_host_alloc(mc, g->blk_bytes, (void **)&g->blk) ||
	    mosrx_host_alloc(mc, g->rec_cap * sizeof(mosrx_result), (void **)&g->res) ||
	    (g_cfg.tcpinfo && mosrx_host_alloc(mc, g->rec_cap * sizeof(mosrx_tcpinfo), (void **)&g->ti)) ||
	    (MATCH_UP_FRONT && mosrx_host_alloc(mc, g->rec_cap * 4, (void **)&g->match)) ||
	    (g_cfg.flowhash && mosrx_host_alloc(mc, g->rec_cap * 4, (void **)&g->fh)))
		return -ENOMEM;
	return 0;
}

static int group_alloc(mosrx_ctx *mc, struct group *g)
{
	const uint64_t floor = stage_bytes();
	uint64_t want = g_cfg.group == MOSRX_GROUP_AUTO ? auto_bytes() : stage_bytes() * g_cfg.group;
	if (want < floor)
		want = floor;
	for (;;) {
		if (!group_alloc_sized(mc, g, want))
			return 0;
		group_free(mc, g);
		if (want <= floor)
			return -ENOMEM;
		want = want / 2 > floor ? want / 2 : floor;
		fprintf(stderr, "[mosrx] gpu_module: pinned staging short: group block reduced to %llu MiB\n",
		        (unsigned long long)(want >> 20));
	}
}

static void gpu_destroy_handle(struct mtcp_thread_context *ctx);

static void gpu_init_handle(struct mtcp_thread_context *ctx)
{
	struct gpu_priv *pv;
	int i, k, cpu = -1, slot = -1, ndev = 0;

	pthread_mutex_lock(&g_lock);
	for (i = 0; i < MAX_THREADS; i++)     /* bound by mosrx_gpu_module_bind */
		if (g_tab[i].ctx == ctx) { slot = i; cpu = g_tab[i].cpu; break; }
	if (slot < 0) {
#ifdef MOSRX_HAVE_MOS_IO_MODULE
		/* the mTCP core the thread was created for: MTCPRunThread sets ctx->cpu
		 * (core.c:1302) before it calls init_handle (core.c:1313), and the
		 * threads call it concurrently, so registration order is not stable */
		cpu = ctx ? ctx->cpu : -1;
#else
		cpu = g_next_cpu;                  /* standalone: registration order */
#endif
		for (i = 0; i < MAX_THREADS; i++)
			if (!g_tab[i].ctx) { slot = i; g_tab[i].ctx = ctx; g_tab[i].cpu = cpu; g_next_cpu++; break; }
	}
	pthread_mutex_unlock(&g_lock);
	if (cpu < 0) {
		fprintf(stderr, "[mosrx] gpu_module: context without a cpu\n");
		exit(EXIT_FAILURE);
	}
	if (slot < 0) {
		fprintf(stderr, "[mosrx] gpu_module: too many threads\n");
		exit(EXIT_FAILURE);
	}
	pv = calloc(1, sizeof(*pv));
	if (!pv)
		exit(EXIT_FAILURE);
	pv->ctx = ctx;
	pv->cpu = cpu;
	ndev = mosrx_device_count();
	pv->stats.cpu = cpu;
	pv->stats.device = mosrx_gpu_module_device_of(cpu, ndev);
	pv->stats.cpu_node = mosrx_cpu_numa_node(cpu);
	pv->stats.gpu_node = pv->stats.device >= 0 ? gpu_node_of(pv->stats.device) : -1;
	for (i = 0; i < (int)g_cfg.num_ifs; i++) {
		struct if_state *is = &pv->ifs[i];
		int dev = mosrx_gpu_module_device_of(cpu, ndev);
		int rc = dev < 0 ? -ENODEV : mosrx_open(dev, &g_cfg.params, &is->mc);
		if (rc) {
			fprintf(stderr, "[mosrx] gpu_module: mosrx_open(%d): %s\n", dev, mosrx_strerror(rc));
			exit(EXIT_FAILURE);
		}
		is->params = g_cfg.params;
		/* no per-group reason counters: mOS counts NETSTAT from the records (the
		 * consumer, eth_in.c:42-45, :80-84), and their copy back is one more
		 * operation in every group's chain */
		mosrx_set_counters(is->mc, 0);
		/* small groups (light load) with no copies: the kernel reads the pinned
		 * staging and writes the pinned records in place */
		mosrx_set_direct(is->mc, (uint64_t)g_cfg.direct_kb << 10, g_cfg.direct_frames);
		is->src = (cpu < MAX_THREADS && g_src_cpu[cpu][i]) ? g_src_cpu[cpu][i] : g_cfg.src[i];
		is->cur = is->inflight = -1;
		if (g_cfg.bpf_nprog && (rc = mosrx_bpf_set(is->mc, g_cfg.bpf_progs, g_cfg.bpf_nprog))) {
			fprintf(stderr, "[mosrx] gpu_module: mosrx_bpf_set: %s\n", mosrx_strerror(rc));
			exit(EXIT_FAILURE);
		}
		is->nprog = g_cfg.bpf_nprog;
		for (k = 0; k < MOSRX_NSLOT; k++)
			if (group_alloc(is->mc, &is->g[k])) {
				fprintf(stderr, "[mosrx] gpu_module: pinned staging allocation failed\n");
				exit(EXIT_FAILURE);
			}
		/* the device side of the largest group, up front: a slot that grew in the
		 * middle of traffic would stall the mTCP thread for milliseconds (the
		 * copies' 256-byte run alignment: 3 runs per batch at most) */
		{
			const uint64_t fb = is->g[0].blk_bytes + (uint64_t)is->g[0].cap_st * 3 * 256;
			const uint64_t n = is->g[0].rec_cap;
			if ((rc = mosrx_classify_host_reserve(is->mc, fb, n > UINT32_MAX ? UINT32_MAX : (uint32_t)n)))
				fprintf(stderr, "[mosrx] gpu_module: device staging not reserved (%s): slots grow on demand\n",
				        mosrx_strerror(rc));
		}
		/* pinned when the TX rewrite copies it to the GPU and back (cfg.tx_csum) */
		if (!g_cfg.tx_csum)
			is->tx_buf = malloc((size_t)g_cfg.tx_batch * TX_FRAME_LEN);
		else if (mosrx_host_alloc(is->mc, (size_t)g_cfg.tx_batch * TX_FRAME_LEN, (void **)&is->tx_buf))
			is->tx_buf = NULL;
		is->tx_len = calloc(g_cfg.tx_batch, sizeof(uint16_t));
		is->tx_fl = calloc(g_cfg.tx_batch, 1);
		is->tx_poff = calloc(g_cfg.tx_batch, sizeof(uint32_t));
		is->tx_plen = calloc(g_cfg.tx_batch, sizeof(uint16_t));
		if (!is->tx_buf || !is->tx_len || !is->tx_fl || !is->tx_poff || !is->tx_plen)
			exit(EXIT_FAILURE);
	}
	pthread_mutex_lock(&g_lock);
	g_tab[slot].priv = pv;
	pthread_mutex_unlock(&g_lock);
}

/* Receive up to `batch` frames from the netdev's source into stage s, whose
 * descriptors start at *pos in the group block (advanced past what it used). */
static void stage_fill(struct group *g, struct stage *s, mosrx_source *src, uint64_t *pos, uint32_t max_n)
{
	const uint32_t mf = g_cfg.max_frame;
	uint64_t at = (*pos + 255) & ~255ull, fpos = 2, cap;
	uint32_t i = 0, m = 0;
	s->off = (uint32_t *)(g->blk + at);
	s->len = (uint16_t *)(g->blk + at + (size_t)g_cfg.batch * 4);
	at += ((uint64_t)g_cfg.batch * 6 + 15) & ~15ull;
	s->frames = g->blk + at;
	cap = g->blk_bytes - at;
	s->borrowed = 0;
	s->n = 0;
	if (src && src->borrow) {         /* zero-copy: the source's pinned run is the batch */
		const uint8_t *f = NULL;
		uint64_t fb = 0;
		s->n = src->borrow(src, max_n, mf, &f, &fb, s->off, s->len);
		if (s->n) {
			s->frames = (uint8_t *)f;
			s->bytes = fb;
			s->borrowed = 1;
		} else {
			s->bytes = 2;
		}
		fpos = 0;
	} else if (src) {                 /* the source's batch form, or frame by frame (mosrx_source_fill) */
		const int k = mosrx_source_fill(src, s->frames, cap, s->off, s->len, max_n, mf, &s->bytes);
		s->n = k > 0 ? (uint32_t)k : 0;
		if (k <= 0)
			s->bytes = 2;
		fpos = s->bytes;
	} else {
		s->bytes = 2;
	}
	/* a short batch's descriptors as one run, len[] right after off[n]: one copy
	 * to the device instead of two (the reserved arrays' unused tails would keep
	 * them apart); borrowed frames leave the block to the descriptors, so the
	 * next stage's follow this one's and a group's descriptors are one run */
	if (s->n && s->n < g_cfg.batch) {
		uint16_t *len2 = (uint16_t *)(s->off + s->n);
		memmove(len2, s->len, (size_t)s->n * 2);
		s->len = len2;
	}
	/* the batch's real largest frame picks the kernel shape; equal frames packed
	 * at one stride (the fill's back-to-back small frames, a ring of fixed-size
	 * buffers) are handed over with that layout as a hint (mosrx_batch.layout) */
	s->stride = s->n > 1 && s->off[1] > s->off[0] ? s->off[1] - s->off[0] : 0;
	for (i = 0; i < s->n; i++) {
		m = s->len[i] > m ? s->len[i] : m;
		if (s->off[i] != s->off[0] + i * s->stride)
			s->stride = 0;
	}
	s->max_len = m;
	*pos = s->borrowed ? (uint64_t)((uint8_t *)(s->len + s->n) - g->blk) : at + fpos;
}

/* Receive a group: up to cap_st batches (auto: until the block's bytes of
 * frames), stopping early when the source runs dry -- a batch that comes back
 * short ends the group, so nothing waits for frames that are not there yet.
 * Filters or not, the group is one launch (the fused classify + BPF queue
 * kernel when a set is installed). */
static uint64_t mono_ns(void)
{
	struct timespec ts;
	clock_gettime(CLOCK_MONOTONIC, &ts);
	return (uint64_t)ts.tv_sec * 1000000000ull + (uint64_t)ts.tv_nsec;
}

/* The latency cap (cfg.group_max_us): the frames and frame bytes a group may
 * take so that, at the rates measured on this netdev so far, neither its
 * transfer + classification nor the host's walk of it takes longer than the
 * budget; never under MOSRX_GROUP_MIN_FRAMES (a group that small is all fixed
 * costs).  UINT64_MAX when there is no budget or no measurement yet. */
#define MOSRX_GROUP_MIN_FRAMES 4096u
static void group_cap(const struct if_state *is, uint64_t *frames, uint64_t *bytes)
{
	const double budget = (double)g_cfg.group_max_us * 1e3;
	*frames = *bytes = UINT64_MAX;
	if (!g_cfg.group_max_us)
		return;
	if (is->ns_per_frame > 0) {
		*frames = (uint64_t)(budget / is->ns_per_frame);
		if (*frames < MOSRX_GROUP_MIN_FRAMES)
			*frames = MOSRX_GROUP_MIN_FRAMES;
	}
	if (is->ns_per_byte > 0)
		*bytes = (uint64_t)(budget / is->ns_per_byte);
}

static void ewma(double *e, double x)
{
	*e = *e > 0 ? 0.75 * *e + 0.25 * x : x;
}

static void group_fill(struct if_state *is, struct group *g)
{
	const uint32_t cap = g->cap_st;
	uint64_t pos = 0, recs = 0, fbytes = 0, cap_frames, cap_bytes;
	uint32_t i;
	group_cap(is, &cap_frames, &cap_bytes);
	is->cap_frames_last = cap_frames;
	g->nst = 0;
	for (i = 0; i < cap; i++) {
		struct stage *s = &g->st[i];
		const uint32_t want = cap_frames - recs < g_cfg.batch ? (uint32_t)(cap_frames - recs) : g_cfg.batch;
		/* room for this stage: a worst-case one (explicit groups), or its
		 * descriptors and one largest frame (auto: it stops where the block ends) */
		const uint64_t need = g_cfg.group == MOSRX_GROUP_AUTO
		                          ? (((uint64_t)g_cfg.batch * 6 + 15) & ~15ull) + 256 + g_cfg.max_frame + 32
		                          : stage_bytes();
		if (pos + need > g->blk_bytes || recs + g_cfg.batch > g->rec_cap)
			break;
		stage_fill(g, s, is->src, &pos, want);
		s->rec0 = (uint32_t)recs;
		s->res = g->res + recs;
		s->ti = g->ti ? g->ti + recs : NULL;
		s->match = g->match ? g->match + recs : NULL;
		s->fh = g->fh ? g->fh + recs : NULL;
		if (!s->n)
			break;
		g->nst++;
		recs += s->n;
		fbytes += s->bytes;
		if (s->n < want || recs >= cap_frames || fbytes >= cap_bytes)
			break;
		if (g_cfg.group == MOSRX_GROUP_AUTO && fbytes >= g->blk_bytes)
			break;
	}
}

static uint64_t group_frame_bytes(const struct group *g)
{
	uint64_t b = 0;
	uint32_t i;
	for (i = 0; i < g->nst; i++)
		b += g->st[i].bytes;
	return b;
}

static uint64_t group_frames(const struct group *g)
{
	uint64_t n = 0;
	uint32_t i;
	for (i = 0; i < g->nst; i++)
		n += g->st[i].n;
	return n;
}

/* Hand the group's borrowed runs back to the source (they are no longer exposed). */
static void group_recycle(struct group *g, mosrx_source *src)
{
	uint32_t i;
	for (i = 0; i < g->nst; i++)
		if (g->st[i].borrowed && src && src->give_back)
			src->give_back(src);
	g->nst = 0;
}

/* A received group that could not be classified: its frames are dropped and
 * counted (rx_drops), borrowed runs go back to the source. */
static void group_drop(struct gpu_priv *pv, struct if_state *is, int k)
{
	uint32_t i;
	for (i = 0; i < is->g[k].nst; i++)
		pv->stats.rx_drops += is->g[k].st[i].n;
	group_recycle(&is->g[k], is->src);
}

static void stage_batch(const struct stage *s, mosrx_batch *b)
{
	b->frames = s->frames;
	b->frames_bytes = s->bytes;
	b->off = s->off;
	b->len = s->len;
	b->n = s->n;
	b->max_len = s->max_len;
	b->layout = s->stride ? MOSRX_BATCH_UNIFORM : 0;
	b->off0 = s->n ? s->off[0] : 0;
	b->stride = s->stride;
	b->reserved = 0;
}

/* Classify stages [first, nst) of group k on pipeline slot k, under mOS's
 * current stack state and the installed filter set: one launch for all of
 * them (the batch queue; with filters the fused classify + BPF queue kernel,
 * which also makes the flow hashes). */
static int group_submit(struct gpu_priv *pv, struct if_state *is, int k, uint32_t first)
{
	struct group *g = &is->g[k];
	mosrx_batch b[MOSRX_MAX_GROUP];
	mosrx_result *out[MOSRX_MAX_GROUP];
	mosrx_result8 *out8[MOSRX_MAX_GROUP];
	mosrx_tcpinfo *ti[MOSRX_MAX_GROUP];
	uint32_t *fh[MOSRX_MAX_GROUP], *mt[MOSRX_MAX_GROUP];
	uint32_t i, nb = g->nst - first;
	if (follow_mos_state(pv, is))
		return -1;
	const int compact = g_cfg.compact;
	for (i = first; i < g->nst; i++) {
		struct stage *s = &g->st[i];
		stage_batch(s, &b[i - first]);
		/* the records' slots in the group's array: 8 or 16 bytes each, back to back */
		s->res = compact ? (mosrx_result *)((mosrx_result8 *)g->res + s->rec0) : g->res + s->rec0;
		out[i - first] = s->res;
		out8[i - first] = RES8(s);
		ti[i - first] = s->ti;
		fh[i - first] = s->fh;
		mt[i - first] = s->match;
		s->msp = is->params.num_msp;
		s->esp = is->params.num_esp;
		s->gen = is->gen;
		s->nprog = is->nprog;
		s->has_fh = s->fh != NULL;
		s->has_ti = s->ti != NULL && !is->nprog;
		s->compact = compact;
	}
	if (compact && is->nprog)   /* 8-byte records + the set's masks: the fused kernel's 8-byte form */
		return mosrx_classify_host_group_submit_bpf_c8(is->mc, k, b, nb, out8, g_cfg.flowhash ? fh : NULL, mt);
	if (compact)
		return mosrx_classify_host_group_submit_c8(is->mc, k, b, nb, out8, g_cfg.flowhash ? fh : NULL);
	if (is->nprog)
		return mosrx_classify_host_group_submit_bpf(is->mc, k, b, nb, out, g_cfg.flowhash ? fh : NULL, mt);
	/* one batch, no copy-free groups: the single-batch submit (no batch table:
	 * the kernel takes the batch as arguments); with cfg.direct_kb a lone batch
	 * takes the group path, which can run it with no copies */
	if (nb == 1 && !g_cfg.flowhash && !g_cfg.direct_kb)
		return mosrx_classify_host_submit_ex(is->mc, k, &b[0], out[0], ti[0]);
	return mosrx_classify_host_group_submit_ex(is->mc, k, b, nb, out, g_cfg.tcpinfo ? ti : NULL,
	                                           g_cfg.flowhash ? fh : NULL);
}

static int group_wait(struct gpu_priv *pv, struct if_state *is, int k, int count)
{
	float ms;
	uint32_t i;
	if (mosrx_classify_host_wait(is->mc, k))
		return -1;
	if (count) {
		pv->stats.rx_batches += is->g[k].nst;
		for (i = 0; i < is->g[k].nst; i++)
			pv->stats.rx_frames += is->g[k].st[i].n;
	}
	if (mosrx_last_kernel_ms(is->mc, &ms) == 0) {
		pv->stats.kernel_ms += ms;
		pv->stats.kernel_launches++;
	}
	return 0;
}

/* Were the stage's records made under something other than what ProcessPacket
 * would see now?  mOS's socket counts (a monitor or end-host socket came or
 * went, socket.c:77-78), or the application's parameters / filter set. */
static int stage_stale(const struct gpu_priv *pv, const struct if_state *is, const struct stage *s)
{
	uint32_t msp, esp;
	if (s->gen != is->gen)
		return 1;
	return mos_state(pv, &msp, &esp) && (msp != s->msp || esp != s->esp);
}

/* Classify stages [first, nst) of the exposed / just-waited group k again,
 * blocking (slot k is idle: its group was waited). */
static int group_reclassify(struct gpu_priv *pv, struct if_state *is, int k, uint32_t first)
{
	pv->stats.rx_reclassified += is->g[k].nst - first;
	if (group_submit(pv, is, k, first) || group_wait(pv, is, k, 0))
		return -1;
	return 0;
}

static int32_t gpu_recv_pkts(struct mtcp_thread_context *ctx, int ifidx)
{
	struct gpu_priv *pv = priv_of(ctx);
	struct if_state *is;
	int k;

	if (!pv || ifidx < 0 || ifidx >= (int)g_cfg.num_ifs)
		return -1;
	is = &pv->ifs[ifidx];
	/* the next batch of the group already classified -- again first if the
	 * stack state or the filters changed since (ProcessPacket reads the
	 * socket counts live, per frame) */
	if (is->cur >= 0 && is->cur_idx + 1 < is->g[is->cur].nst) {
		struct group *g = &is->g[is->cur];
		is->cur_idx++;
		if (stage_stale(pv, is, &g->st[is->cur_idx]) && group_reclassify(pv, is, is->cur, is->cur_idx)) {
			/* the rest of the group is lost; the next call moves on */
			uint32_t i;
			for (i = is->cur_idx; i < g->nst; i++)
				pv->stats.rx_drops += g->st[i].n;
			is->cur_idx = g->nst - 1;
			return -1;
		}
		return (int32_t)g->st[is->cur_idx].n;
	}
	/* the exposed group is done with (get_rptr pointers expire here) */
	k = is->cur < 0 ? 0 : is->cur ^ 1;
	if (is->cur >= 0) {
		const uint64_t n = group_frames(&is->g[is->cur]);
		if (n && is->t_expose)   /* the host's time per frame of this group (the latency cap's walk rate) */
			ewma(&is->ns_per_frame, (double)(mono_ns() - is->t_expose) / (double)n);
		group_recycle(&is->g[is->cur], is->src);
	}
	is->cur = -1;                     /* nothing exposed until a group is ready */
	if (is->inflight < 0) {           /* nothing in flight: receive + classify now */
		group_fill(is, &is->g[k]);
		if (!is->g[k].nst)
			return 0;
		if (group_submit(pv, is, k, 0)) {
			group_drop(pv, is, k);
			return -1;
		}
		is->t_submit[k] = mono_ns();
		is->inflight = k;
	}
	k = is->inflight;
	is->inflight = -1;
	{
		/* the group's submit -> records ready, per frame byte: exact when the wait
		 * blocks; an upper bound when the group was done before we came for it */
		const int done = mosrx_classify_host_ready(is->mc, k) == 1;
		if (group_wait(pv, is, k, 1)) {
			group_drop(pv, is, k);
			return -1;
		}
		const uint64_t b = group_frame_bytes(&is->g[k]);
		const double x = b ? (double)(mono_ns() - is->t_submit[k]) / (double)b : 0;
		if (b && (!done || is->ns_per_byte <= 0 || x < is->ns_per_byte))
			ewma(&is->ns_per_byte, x);
	}
	/* classified in flight under a state that has changed since: again, under
	 * the state the rx loop runs with now */
	if (stage_stale(pv, is, &is->g[k].st[0]) && group_reclassify(pv, is, k, 0)) {
		group_drop(pv, is, k);
		return -1;
	}
	is->cur = k;
	is->cur_idx = 0;
	is->t_expose = mono_ns();
	{
		const uint64_t n = group_frames(&is->g[k]);
		pv->stats.rx_groups++;
		if (n > pv->stats.max_group_frames)
			pv->stats.max_group_frames = n;
		if (mosrx_slot_direct(is->mc, k) == 1)
			pv->stats.rx_direct_groups++;
	}
	if (g_cfg.pipeline) {             /* classify the next group behind the app's work */
		int nk = k ^ 1;
		group_fill(is, &is->g[nk]);
		if (is->g[nk].nst) {
			if (group_submit(pv, is, nk, 0) == 0) {
				is->t_submit[nk] = mono_ns();
				is->inflight = nk;
			} else {
				group_drop(pv, is, nk);
			}
		}
	}
	return (int32_t)is->g[k].st[0].n;
}

static const struct stage *cur_stage(struct gpu_priv *pv, int ifidx)
{
	const struct if_state *is;
	if (!pv || ifidx < 0 || ifidx >= (int)g_cfg.num_ifs || pv->ifs[ifidx].cur < 0)
		return NULL;
	is = &pv->ifs[ifidx];
	return &is->g[is->cur].st[is->cur_idx];
}

static uint8_t *gpu_get_rptr(struct mtcp_thread_context *ctx, int ifidx, int index, uint16_t *len)
{
	const struct stage *s = cur_stage(priv_of(ctx), ifidx);
	if (!s || index < 0 || (uint32_t)index >= s->n)
		return NULL;
	*len = s->len[index];
	return s->frames + s->off[index];
}

static void gpu_release_pkt(struct mtcp_thread_context *ctx, int ifidx, unsigned char *pkt, int len)
{
	/* staging is recycled wholesale on the next recv_pkts */
	(void)ctx; (void)ifidx; (void)pkt; (void)len;
}

/* The checks mOS left to the "NIC" (dev_ioctl PKT_TX_*_CSUM): filled on the
 * GPU, one TX rewrite pass per distinct request (in practice one: mOS asks for
 * both on every TCP frame it builds).  A pass that fails leaves its frames
 * without checksums: they are dropped (TXF bit 7) and counted as TX errors,
 * as a NIC would, never sent with a stale check. */
static void tx_csum_fill(struct gpu_priv *pv, struct if_state *is)
{
	uint32_t *off = is->tx_poff, i, n, fl;
	uint16_t *len = is->tx_plen;
	for (fl = 1; fl <= (TXF_IP | TXF_TCP); fl++) {
		mosrx_batch b = {0};
		uint32_t m = 0;
		uint64_t end = 0;
		int rc;
		for (i = n = 0; i < is->tx_n; i++)
			if (is->tx_fl[i] == fl) {
				off[n] = i * TX_FRAME_LEN;
				len[n] = is->tx_len[i];
				m = len[n] > m ? len[n] : m;
				end = (uint64_t)off[n] + len[n];
				n++;
			}
		if (!n)
			continue;
		if (!is->mc_tx) {
			const int dev = mosrx_gpu_module_device_of(pv->cpu, mosrx_device_count());
			if (dev < 0 || mosrx_open(dev, &is->params, &is->mc_tx))
				is->mc_tx = NULL;
		}
		b.frames = is->tx_buf;
		b.frames_bytes = end;         /* up to the last frame of the pass: what crosses PCIe */
		b.off = off;
		b.len = len;
		b.n = n;
		b.max_len = m;
		rc = is->mc_tx ? mosrx_tx_csum_host(is->mc_tx, &b, ((fl & TXF_IP) ? MOSRX_TX_IP_CSUM : 0) |
		                                                       ((fl & TXF_TCP) ? MOSRX_TX_TCP_CSUM : 0))
		               : -ENODEV;
		if (rc) {
			fprintf(stderr, "[mosrx] gpu_module: TX checksum pass: %s\n", mosrx_strerror(rc));
			for (i = 0; i < is->tx_n; i++)
				if (is->tx_fl[i] == fl)
					is->tx_fl[i] |= 0x80;
		} else {
			pv->stats.tx_csum_offloaded += n;
		}
	}
}

/* Hand every buffered TX frame of netdev nif to its source. */
static int32_t tx_flush(struct gpu_priv *pv, int nif)
{
	struct if_state *is = &pv->ifs[nif];
	uint32_t i;
	int32_t sent = 0;
	for (i = 0; i < is->tx_n && g_cfg.tx_csum; i++)
		if (is->tx_fl[i]) {
			tx_csum_fill(pv, is);
			break;
		}
	for (i = 0; i < is->tx_n; i++) {
		if (is->tx_fl[i] & 0x80) {
			pv->stats.tx_errors++;
			continue;
		}
		if (mosrx_source_send(is->src, is->tx_buf + (size_t)i * TX_FRAME_LEN, is->tx_len[i]) == 0) {
			sent++;
			pv->stats.tx_packets++;
			pv->stats.tx_bytes += is->tx_len[i];
		} else {
			pv->stats.tx_errors++;
		}
	}
	is->tx_n = 0;
	if (sent && is->src)
		mosrx_source_tx_flush(is->src);
	return sent;
}

static uint8_t *gpu_get_wptr(struct mtcp_thread_context *ctx, int ifidx, uint16_t len)
{
	struct gpu_priv *pv = priv_of(ctx);
	struct if_state *is;
	if (!pv || ifidx < 0 || ifidx >= (int)g_cfg.num_ifs || len > TX_FRAME_LEN)
		return NULL;
	is = &pv->ifs[ifidx];
	if (is->tx_n == g_cfg.tx_batch)   /* full: send what is buffered first (dpdk_get_wptr) */
		tx_flush(pv, ifidx);
	is->tx_len[is->tx_n] = len;
	is->tx_fl[is->tx_n] = 0;
	return is->tx_buf + (size_t)(is->tx_n++) * TX_FRAME_LEN;
}

/* Frames written since the last call leave through the netdev's source;
 * returns how many were sent (pcap_send_pkts, pcap_module.c:67-79). */
static int32_t gpu_send_pkts(struct mtcp_thread_context *ctx, int nif)
{
	struct gpu_priv *pv = priv_of(ctx);
	if (!pv || nif < 0 || nif >= (int)g_cfg.num_ifs)
		return 0;
	return tx_flush(pv, nif);
}

static int gpu_get_nif(struct ifreq *ifr)
{
	uint32_t i;
	for (i = 0; i < g_cfg.num_ifs; i++)
		if (!strncmp(ifr->ifr_name, g_cfg.if_names[i], IFNAMSIZ))
			return (int)i;
	return -1;
}

/* Install a BPF program set on netdev is (the monitors' filters, bit j =
 * program j): the match arrays are allocated the first time, the stages of
 * both groups pointed at them, and the generation bumped so every batch not
 * yet handed out is classified again with the set.  The set is in effect at
 * once (mosrx_bpf_set_async: the interpreter kernel until the compile thread
 * has its hipRTC kernels loaded), so the mTCP thread never waits for a
 * compile. */
static int32_t set_bpf(struct gpu_priv *pv, struct if_state *is, const mosrx_bpf_set_arg *a)
{
	int k;
	uint32_t i;
	(void)pv;
	/* MOSRX_BPF_SYNC=1 (diagnostics): wait for the compile here, as before round 4 */
	static int sync_set = -1;
	if (sync_set < 0)
		sync_set = getenv("MOSRX_BPF_SYNC") && atoi(getenv("MOSRX_BPF_SYNC")) == 1;
	if (!a || a->nprog > MOSRX_BPF_MAX_PROGS ||
	    (sync_set ? mosrx_bpf_set(is->mc, a->progs, a->nprog) : mosrx_bpf_set_async(is->mc, a->progs, a->nprog)))
		return -1;
	for (k = 0; k < MOSRX_NSLOT && a->nprog; k++) {
		struct group *g = &is->g[k];
		if (!g->match && mosrx_host_alloc(is->mc, g->rec_cap * 4, (void **)&g->match))
			return -1;
		for (i = 0; i < g->nst; i++)
			g->st[i].match = g->match + g->st[i].rec0;
	}
	is->nprog = a->nprog;
	is->gen++;
	return 0;
}

static int32_t gpu_dev_ioctl(struct mtcp_thread_context *ctx, int nif, int cmd, void *argp)
{
	struct gpu_priv *pv = priv_of(ctx);
	const struct stage *s;
	if (!pv || !argp || nif < 0 || nif >= (int)g_cfg.num_ifs)
		return -1;
	s = cur_stage(pv, nif);
	switch (cmd) {
	case PKT_RX_RSS: {
		RssInfo *ri = argp;
		if (!s || ri->pktidx < 0 || (uint32_t)ri->pktidx >= s->n)
			return -1;
		ri->hash_value = s->compact ? RES8(s)[ri->pktidx].rss : s->res[ri->pktidx].rss;
		return 0;
	}
	case MOSRX_PKT_RX_RESULTS:
		if (!s || s->compact)
			return -1;
		*(const mosrx_result **)argp = s->res;
		return 0;
	case MOSRX_PKT_RX_RESULTS8:
		if (!s || !s->compact)
			return -1;
		*(const mosrx_result8 **)argp = RES8(s);
		return 0;
	case MOSRX_PKT_RX_MATCH:
		if (!s || !s->match || !s->nprog)
			return -1;
		*(const uint32_t **)argp = s->match;
		return 0;
	case MOSRX_PKT_RX_FHASH:
		if (!s || !s->has_fh)
			return -1;
		*(const uint32_t **)argp = s->fh;
		return 0;
	case MOSRX_PKT_RX_TCPINFO:
		if (!s || !s->has_ti)
			return -1;
		*(const mosrx_tcpinfo **)argp = s->ti;
		return 0;
	case MOSRX_PKT_SET_PARAMS:
		/* batches submitted from now on use the new stack state; a group in
		 * flight may have read the tables half rewritten, and every batch not
		 * yet handed out was made under the old state: the generation makes
		 * recv_pkts classify them again before they are exposed */
		if (mosrx_set_params(pv->ifs[nif].mc, (const mosrx_params *)argp))
			return -1;
		pv->ifs[nif].params = *(const mosrx_params *)argp;
		pv->ifs[nif].gen++;
		return 0;
	case MOSRX_PKT_SET_BPF:
		return set_bpf(pv, &pv->ifs[nif], (const mosrx_bpf_set_arg *)argp);
	case MOSRX_PKT_RX_STATE: {
		mosrx_rx_state *st = argp;
		if (!s)
			return -1;
		st->num_msp = s->msp;
		st->num_esp = s->esp;
		st->gen = s->gen;
		st->bpf_nprog = s->nprog;
		st->n = s->n;
		st->rec_bytes = s->compact ? 8u : 16u;
		return 0;
	}
	case MOSRX_PKT_RX_RECLASSIFY: {
		struct if_state *is = &pv->ifs[nif];
		if (!s)
			return -1;
		return group_reclassify(pv, is, is->cur, is->cur_idx) ? -1 : 0;
	}
	case DRV_NAME:
		*(const char **)argp = "mosrx_gpu";
		return 0;
	case PKT_TX_IP_CSUM:
	case PKT_TX_TCP_CSUM: {
		/* dpdk_dev_ioctl's offload (dpdk_module.c:556-566): the request is for
		 * the frame get_wptr handed out last on this netdev, argp its IP header;
		 * without cfg.tx_csum, or for anything else, -1 and mOS computes it */
		struct if_state *is = &pv->ifs[nif];
		const uint8_t *ip = argp, *f;
		if (!g_cfg.tx_csum || !is->tx_n)
			return -1;
		f = is->tx_buf + (size_t)(is->tx_n - 1) * TX_FRAME_LEN;
		if (ip != f + 14 || is->tx_len[is->tx_n - 1] < 34)
			return -1;
		is->tx_fl[is->tx_n - 1] |= cmd == PKT_TX_IP_CSUM ? TXF_IP : TXF_TCP;
		return 0;
	}
	default:
		return -1;
	}
}

static void gpu_destroy_handle(struct mtcp_thread_context *ctx)
{
	struct gpu_priv *pv = priv_of(ctx);
	uint32_t i;
	int k;
	if (!pv) {                         /* bound but never initialised: free the slot */
		pthread_mutex_lock(&g_lock);
		for (k = 0; ctx && k < MAX_THREADS; k++)
			if (g_tab[k].ctx == ctx)
				memset(&g_tab[k], 0, sizeof(g_tab[k]));
		pthread_mutex_unlock(&g_lock);
		return;
	}
	for (i = 0; i < g_cfg.num_ifs; i++) {
		struct if_state *is = &pv->ifs[i];
		if (!is->mc)
			continue;
		if (is->inflight >= 0)
			mosrx_classify_host_wait(is->mc, is->inflight);
		tx_flush(pv, (int)i);
		for (k = 0; k < MOSRX_NSLOT; k++) {
			group_recycle(&is->g[k], is->src);
			group_free(is->mc, &is->g[k]);
		}
		if (g_cfg.tx_csum)
			mosrx_host_free(is->mc, is->tx_buf);
		else
			free(is->tx_buf);
		free(is->tx_len);
		free(is->tx_fl);
		free(is->tx_poff);
		free(is->tx_plen);
		if (is->mc_tx)
			mosrx_close(is->mc_tx);
		mosrx_close(is->mc);
	}
	pthread_mutex_lock(&g_lock);
	for (k = 0; k < MAX_THREADS; k++)     /* the slot is free again */
		if (g_tab[k].ctx == ctx)
			memset(&g_tab[k], 0, sizeof(g_tab[k]));
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
