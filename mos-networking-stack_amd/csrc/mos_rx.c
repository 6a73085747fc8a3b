/*
 * mos_rx.c — mosrx_mos_process_packet: mOS's receive step per frame, taking
 * the checks' outcome from the GPU record instead of computing it
 * (include/mosrx_mos_rx.h).  Built inside mOS's tree only: it calls mOS's own
 * functions for every side effect and walks mOS's own structures.
 *
 * The record's reason code says which return of ProcessPacket the frame
 * reaches (include/mosrx.h MOSRX_R_*); what ProcessPacket does on the way
 * there is reproduced in its order:
 *
 *   eth_in.c:42-45      NETSTAT rx_packets / rx_bytes
 *   eth_in.c:60-78      non-IPv4: ProcessARPPacket, or DumpPacket + release_pkt,
 *                       or ForwardEthernetFrame (forward && num_msp)
 *   ip_in.c:41-51       tot_len < 20 -> -1; version != 4 -> release, 0
 *   ip_in.c:53-63       pkt_info IP fields; raw monitors whose filter matches:
 *                       MOS_ON_PKT_IN (the filter from the GPU match mask)
 *   ip_in.c:65-72       no monitor / end-host socket: forward, 1 (nothing verified)
 *   ip_in.c:74-77       bad IP checksum -> -1
 *   ip_in.c:79-94       ICMP to a local address: ProcessICMPPacket, 1;
 *                       other protocols: release or forward, 0
 *   tcp.c:418-427       pkt_info TCP fields (record + header); every raw
 *                       monitor: MOS_ON_PKT_IN
 *   tcp.c:429-444       too short -> -1; bad TCP checksum -> forward, -1
 *   tcp.c:445-514       the stream step: FindStream on the GPU's bucket, then
 *                       mOS's CreateStream / HandleSockStream /
 *                       HandleMonitorStream when tcp.c exports them (the
 *                       upstream patch, INTEGRATION.md §2b, -DMOSRX_MOS_TCP_EXPORTS);
 *                       otherwise -- they are static in tcp.c -- restated below
 *                       with mOS's exported functions
 *   eth_in.c:80-84      NETSTAT rx_errors for a negative return
 *
 * TRUNCATED frames (headers claiming bytes past the capture; the reference
 * reads past its buffer there) are dropped with -1.
 *
 * A batch whose records cannot be had (the backend could not classify it
 * again after a state or filter change, or handed out no records) is dropped
 * from that frame on, the way a NIC drops what it could not receive: each
 * frame is counted in rx_packets and rx_errors and released, -1, and mOS runs
 * on (the backend's own policy for a failed group, gpu_module.c group_drop).
 */
#include <assert.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "mtcp.h"
#include "arp.h"
#include "socket.h"
#include "eth_out.h"
#include "ip_out.h"
#include "mos_api.h"
#include "tcp_util.h"
#include "tcp_in.h"
#include "tcp_out.h"
#include "tcp_ring_buffer.h"
#include "tcp.h"
#include "fhash.h"
#include "icmp.h"
#include "debug.h"
#include "config.h"
#include "scalable_event.h"
#include "sfbpf.h"

#include "../../include/mosrx_io_module.h"
#include "../../include/mosrx_mos_rx.h"

#define MAX_CORES 64
#define NO_BIT    (-1)

/* tcp.c:258-270, defined with external linkage (`inline` under -fgnu89-inline)
 * but declared in no header */
void FillPacketContextTCPInfo(struct pkt_ctx *pctx, struct tcphdr *tcph);

/* A filter program mOS holds for a monitor, and where its result comes from.
 * Keyed by its instructions, not by where mOS keeps them: a monitor that
 * closes frees its compiled filter (FreeMonListener, socket.c:33-36) and the
 * next one's can land at the same address with the same length. */
#define FILT_INSNS 8192              /* instructions the table keeps copies of */
struct filt {
	const struct sfbpf_insn *insns;  /* mOS's program (fast path: the same pointer) */
	const struct sfbpf_insn *copy;   /* its instructions when installed (in t_view.arena) */
	uint32_t len;
	int mode;                    /* MOSRX_BPF_LEN_FRAME / _IP: the call site's buffer */
	int bit;                     /* bit of the GPU match mask, NO_BIT: EVAL_BPFFILTER */
	int seen;                    /* still bound by a monitor at the last check */
};

/* The batch the mTCP thread is walking (one view per thread: RunMainLoop
 * consumes a batch's frames in order on the thread that received it). */
struct rx_view {
	struct mtcp_manager *mtcp;
	int ifidx;
	const mosrx_result *res;     /* the batch's records: 16-byte ones, */
	const mosrx_result8 *res8;   /* or a compact batch's 8-byte ones (cfg.compact) */
	const uint32_t *match;       /* NULL: no masks for this batch */
	const uint32_t *fhash;       /* NULL: no flow-table hashes for this batch */
	mosrx_rx_state state;
	int dead_from;               /* >= 0: the batch's frames from this index on have no records (dropped) */
	/* the filter set installed on this thread's netdevs */
	struct filt filt[2 * MOSRX_BPF_MAX_PROGS + 64];
	uint32_t nfilt, ngpu;
	struct sfbpf_insn arena[FILT_INSNS];
	uint32_t narena;
};

static __thread struct rx_view t_view;
static mosrx_mos_rx_stats g_stats[MAX_CORES];

static mosrx_mos_rx_stats *stats_of(struct mtcp_manager *mtcp)
{
	const int cpu = mtcp->ctx ? mtcp->ctx->cpu : 0;
	return &g_stats[cpu >= 0 && cpu < MAX_CORES ? cpu : 0];
}

int mosrx_mos_rx_stats_of(int cpu, mosrx_mos_rx_stats *st)
{
	if (cpu < 0 || cpu >= MAX_CORES || !st)
		return -1;
	*st = g_stats[cpu];
	return 0;
}

static uint64_t now_ns(void)
{
	struct timespec t;
	clock_gettime(CLOCK_MONOTONIC, &t);
	return (uint64_t)t.tv_sec * 1000000000ull + (uint64_t)t.tv_nsec;
}

/* The batch has no usable records from frame `index` on: those frames are
 * dropped (counted by the caller), mOS carries on. */
static void view_lost(struct rx_view *v, struct mtcp_manager *mtcp, int index, const char *what)
{
	mosrx_mos_rx_stats *st = stats_of(mtcp);
	if (!st->gpu_errors++)
		fprintf(stderr, "[mosrx] mosrx_mos_process_packet: netdev %d: %s; the batch's remaining frames are "
		        "dropped (rx_errors)\n", v->ifidx, what);
	v->dead_from = index;
}

/* The exposed batch's records, masks and classification state. */
static void view_fetch(struct rx_view *v, struct mtcp_manager *mtcp, int ifidx)
{
	const io_module_func *iom = mtcp->iom;
	v->mtcp = mtcp;
	v->ifidx = ifidx;
	v->res = NULL;
	v->res8 = NULL;
	v->match = NULL;
	v->fhash = NULL;
	v->dead_from = -1;
	if (!iom->dev_ioctl || iom->dev_ioctl(mtcp->ctx, ifidx, MOSRX_PKT_RX_STATE, &v->state) ||
	    (v->state.rec_bytes == 8
	         ? iom->dev_ioctl(mtcp->ctx, ifidx, MOSRX_PKT_RX_RESULTS8, (void *)&v->res8) || !v->res8
	         : iom->dev_ioctl(mtcp->ctx, ifidx, MOSRX_PKT_RX_RESULTS, (void *)&v->res) || !v->res)) {
		v->res = NULL;
		v->res8 = NULL;
		v->state.n = 0x7FFFFFFF;   /* whatever get_rptr hands out goes the dropped way */
		view_lost(v, mtcp, 0, "no GPU records for the batch (is gpu_module_func mOS's I/O module?)");
		return;
	}
	if (v->res8)
		stats_of(mtcp)->batches_c8++;
	if (v->state.bpf_nprog && iom->dev_ioctl(mtcp->ctx, ifidx, MOSRX_PKT_RX_MATCH, (void *)&v->match))
		v->match = NULL;
	if (iom->dev_ioctl(mtcp->ctx, ifidx, MOSRX_PKT_RX_FHASH, (void *)&v->fhash))
		v->fhash = NULL;
}

/* What the consumer reads of a record, in either form: the reason code and
 * the TCP flags byte.  pkt_info's lengths come from the header itself
 * (FillPacketContextTCPInfo, tcp.c:258-270), as mOS takes them. */
static inline uint8_t rec_reason(const struct rx_view *v, int i)
{
	return v->res8 ? v->res8[i].reason : v->res[i].reason;
}

static inline uint8_t rec_flags(const struct rx_view *v, int i)
{
	return v->res8 ? v->res8[i].tcp_flags : v->res[i].tcp_flags;
}

/* FindStream (tcp.c:181-191) -> HTSearch (fhash.c:184-214) with the bucket the
 * GPU computed (HashFlow of the reversed tuple, mosrx_classify_dev_fh) instead
 * of hashing on the CPU; the bucket's list is walked as HTSearch walks it. */
static tcp_stream *find_stream(struct rx_view *v, int index, mtcp_manager_t mtcp, const tcp_stream *key,
                               unsigned int *hash)
{
	tcp_stream *w;
	unsigned int idx;
	if (!v->fhash)
		return HTSearch(mtcp->tcp_flow_table, key, hash);
	idx = v->fhash[index] & (NUM_BINS - 1);
	*hash = idx;
	stats_of(mtcp)->gpu_flow_hash++;
	TAILQ_FOREACH(w, &mtcp->tcp_flow_table->ht_table[idx], rcvvar->he_link)
		if (w->saddr == key->saddr && w->sport == key->sport && w->daddr == key->daddr && w->dport == key->dport)
			return w;
	return NULL;
}

/* Classify the rest of the exposed batch (from frame `index`) again -- the
 * stack state or the filter set changed under it -- and take the new records;
 * if that fails, the rest of the batch is dropped. */
static void view_reclassify(struct rx_view *v, struct mtcp_manager *mtcp, int ifidx, int index)
{
	static int one = 1;
	if (v->dead_from >= 0)
		return;
	if (mtcp->iom->dev_ioctl(mtcp->ctx, ifidx, MOSRX_PKT_RX_RECLASSIFY, &one)) {
		view_lost(v, mtcp, index, "reclassification failed");
		return;
	}
	stats_of(mtcp)->reclassified++;
	view_fetch(v, mtcp, ifidx);
}

/* The table entry of this program: its instructions, length and call site. */
static struct filt *filt_find(struct rx_view *v, const struct sfbpf_program *fc, int mode)
{
	uint32_t i;
	for (i = 0; i < v->nfilt; i++) {
		struct filt *f = &v->filt[i];
		if (f->len == fc->bf_len && f->mode == mode &&
		    !memcmp(f->copy, fc->bf_insns, (size_t)fc->bf_len * sizeof(*fc->bf_insns)))
			return f;
	}
	return NULL;
}

static void filt_add(struct rx_view *v, const struct sfbpf_program *fc, int mode, mosrx_bpf_prog *progs)
{
	struct filt *f;
	if (!fc->bf_insns || filt_find(v, fc, mode) || v->nfilt == sizeof(v->filt) / sizeof(v->filt[0]) ||
	    v->narena + fc->bf_len > FILT_INSNS)
		return;
	f = &v->filt[v->nfilt++];
	f->insns = fc->bf_insns;
	f->copy = v->arena + v->narena;
	memcpy(v->arena + v->narena, fc->bf_insns, (size_t)fc->bf_len * sizeof(*fc->bf_insns));
	v->narena += fc->bf_len;
	f->len = fc->bf_len;
	f->mode = mode;
	f->bit = NO_BIT;
	f->seen = 1;
	if (v->ngpu < MOSRX_BPF_MAX_PROGS) {
		progs[v->ngpu].insns = (const mosrx_bpf_insn *)f->copy;   /* struct sfbpf_insn layout */
		progs[v->ngpu].len = fc->bf_len;
		progs[v->ngpu].len_mode = mode;
		f->bit = (int)v->ngpu++;
	}
}

/* Put the monitors' current filters on the GPU: raw-packet filters over the
 * frame (ip_in.c:58-60: ethh, eth_len), stream SYN / orphan filters over the
 * IP datagram (tcp.c:50-52, :490-492: iph - 14, ip_len + 14), installed on
 * every netdev, then the exposed batch classified again with them. */
static void filters_sync(struct rx_view *v, struct mtcp_manager *mtcp, int ifidx, int index)
{
	mosrx_bpf_prog progs[MOSRX_BPF_MAX_PROGS];
	mosrx_bpf_set_arg a;
	struct mon_listener *walk;
	mosrx_mos_rx_stats *st = stats_of(mtcp);
	const uint64_t t0 = now_ns();
	int nif, ok = 1;
	v->nfilt = v->ngpu = 0;
	v->narena = 0;
	TAILQ_FOREACH(walk, &mtcp->monitors, link) {
		/* the orphan loop (tcp.c:486-496) reads stream_orphan_fcode of every
		 * monitor, raw ones included (their union, socket.h:52-60) */
		if (walk->socket->socktype == MOS_SOCK_MONITOR_RAW)
			filt_add(v, &walk->raw_pkt_fcode, MOSRX_BPF_LEN_FRAME, progs);
		else
			filt_add(v, &walk->stream_syn_fcode, MOSRX_BPF_LEN_IP, progs);
		filt_add(v, &walk->stream_orphan_fcode, MOSRX_BPF_LEN_IP, progs);
	}
	a.progs = progs;
	a.nprog = v->ngpu;
	for (nif = 0; nif < g_config.mos->netdev_table->num && nif < MOSRX_MAX_DEVICES; nif++)
		if (mtcp->iom->dev_ioctl(mtcp->ctx, nif, MOSRX_PKT_SET_BPF, &a))
			ok = 0;
	if (!ok) {   /* a program the GPU would not take (mosrx_bpf_set refused the set): mOS evaluates them */
		uint32_t i;
		a.nprog = 0;
		for (nif = 0; nif < g_config.mos->netdev_table->num && nif < MOSRX_MAX_DEVICES; nif++)
			mtcp->iom->dev_ioctl(mtcp->ctx, nif, MOSRX_PKT_SET_BPF, &a);
		for (i = 0; i < v->nfilt; i++)
			v->filt[i].bit = NO_BIT;
		v->ngpu = 0;
	}
	st->filter_installs++;
	st->filters_gpu = v->ngpu;
	st->filters_cpu = v->nfilt - v->ngpu;
	view_reclassify(v, mtcp, ifidx, index);
	{
		const uint64_t dt = now_ns() - t0;
		if (dt > st->max_filter_sync_ns)
			st->max_filter_sync_ns = dt;
	}
}

/* At a batch's first frame: does the installed table still hold exactly the
 * filters the monitors have bound?  A filter bound since is installed at its
 * first evaluation anyway; one whose monitor went away (its program freed,
 * perhaps reused at the same address by another) is dropped from the set
 * here, so stale programs never hold the GPU's 32 slots. */
static void filters_check(struct rx_view *v, struct mtcp_manager *mtcp, int ifidx)
{
	struct mon_listener *walk;
	uint32_t i;
	int stale = 0;
	if (!v->nfilt)
		return;
	for (i = 0; i < v->nfilt; i++)
		v->filt[i].seen = 0;
#define SEE(fc, mode)                                                     \
	do {                                                                  \
		if ((fc)->bf_insns) {                                             \
			struct filt *f_ = filt_find(v, (fc), (mode));                 \
			if (f_)                                                       \
				f_->seen = 1;                                             \
		}                                                                 \
	} while (0)
	TAILQ_FOREACH(walk, &mtcp->monitors, link) {
		if (walk->socket->socktype == MOS_SOCK_MONITOR_RAW)
			SEE(&walk->raw_pkt_fcode, MOSRX_BPF_LEN_FRAME);
		else
			SEE(&walk->stream_syn_fcode, MOSRX_BPF_LEN_IP);
		SEE(&walk->stream_orphan_fcode, MOSRX_BPF_LEN_IP);
	}
#undef SEE
	for (i = 0; i < v->nfilt; i++)
		stale |= !v->filt[i].seen;
	if (stale)
		filters_sync(v, mtcp, ifidx, 0);
}

/* EVAL_BPFFILTER(*fc, p, l) for frame `index` of the batch (include/bpf/sfbpf.h:84):
 * the GPU's mask bit when the filter is in the installed set. */
static int filter_eval(struct rx_view *v, int index, const struct sfbpf_program *fc, int mode, uint8_t *p, int l)
{
	struct filt *f = filt_find(v, fc, mode);
	/* bound since the last install (a full table or instruction arena keeps
	 * the rest on the CPU rather than installing again for every frame) */
	if (!f && v->nfilt < sizeof(v->filt) / sizeof(v->filt[0]) && v->narena + fc->bf_len <= FILT_INSNS) {
		filters_sync(v, v->mtcp, v->ifidx, index);
		f = filt_find(v, fc, mode);
	}
	if (f && f->bit != NO_BIT && v->match && v->dead_from < 0)
		return (v->match[index] >> f->bit) & 1;
	return EVAL_BPFFILTER((*fc), p, l);
}

/* ---- the stream step, tcp.c:445-514 ---------------------------------------- */

#ifdef MOSRX_MOS_TCP_EXPORTS
/* mOS's own stream functions, given external linkage by the upstream patch of
 * INTEGRATION.md §2b (tcp.c:25, :195, :275, :377: `static` dropped; gnu89
 * `inline` then emits an external definition): CreateStream (with
 * DetectStreamType inside it, so a SYN filter is evaluated by mOS on the CPU,
 * once per connection), HandleSockStream, HandleMonitorStream.  The consumer
 * keeps only FindStream's lookup on the GPU's bucket and the orphan path's
 * filters from the GPU masks. */
struct tcp_stream *CreateStream(mtcp_manager_t mtcp, struct pkt_ctx *pctx, unsigned int *hash);
void HandleSockStream(mtcp_manager_t mtcp, struct tcp_stream *cur_stream, struct pkt_ctx *pctx);
void HandleMonitorStream(mtcp_manager_t mtcp, struct tcp_stream *sendside_stream,
                         struct tcp_stream *recvside_stream, struct pkt_ctx *pctx);
#else
/* Without the patch those functions are static in tcp.c: restated here with
 * mOS's exported functions, the SYN filter from the GPU's mask. */
/* DetectStreamType, tcp.c:25-85: which sockets want a stream for this SYN. */
static uint32_t detect_stream_type(struct rx_view *v, int index, mtcp_manager_t mtcp, struct pkt_ctx *pctx,
                                   uint32_t ip, uint16_t port)
{
	struct mon_listener *walk;
	uint32_t rc = 0;
	int hits = 0;
	if (mtcp->num_msp > 0) {
		TAILQ_FOREACH(walk, &mtcp->monitors, link) {
			const struct sfbpf_program *fc;
			if (walk->socket->socktype != MOS_SOCK_MONITOR_STREAM)
				continue;
			fc = &walk->stream_syn_fcode;
			/* an unset filter takes every flow (tcp.c:50-52) */
			if (!(ISSET_BPFFILTER((*fc)) &&
			      filter_eval(v, index, fc, MOSRX_BPF_LEN_IP, (uint8_t *)pctx->p.iph - sizeof(struct ethhdr),
			                  pctx->p.ip_len + sizeof(struct ethhdr)) == 0)) {
				walk->is_stream_syn_filter_hit = 1;
				hits++;
			}
		}
		if (hits)
			rc = STREAM_TYPE(MOS_SOCK_MONITOR_STREAM_ACTIVE);
	}
	if (mtcp->listener) {   /* an end host listening on the destination (tcp.c:64-82) */
		const struct sockaddr_in *addr = &mtcp->listener->socket->saddr;
		if (addr->sin_port == port) {
			if (addr->sin_addr.s_addr != INADDR_ANY) {
				if (ip == addr->sin_addr.s_addr)
					rc |= STREAM_TYPE(MOS_SOCK_STREAM);
			} else {
				int i;
				for (i = 0; i < g_config.mos->netdev_table->num; i++)
					if (ip == g_config.mos->netdev_table->ent[i]->ip_addr)
						rc |= STREAM_TYPE(MOS_SOCK_STREAM);
			}
		}
	}
	return rc;
}

/* CreateServerStream, tcp.c:87-109 */
static tcp_stream *server_stream(mtcp_manager_t mtcp, int type, struct pkt_ctx *pctx)
{
	tcp_stream *s = CreateTCPStream(mtcp, NULL, type, pctx->p.iph->daddr, pctx->p.tcph->dest,
	                                pctx->p.iph->saddr, pctx->p.tcph->source, NULL);
	if (!s)
		return NULL;
	s->rcvvar->irs = pctx->p.seq;
	s->sndvar->peer_wnd = pctx->p.window;
	s->rcv_nxt = s->rcvvar->irs;
	s->sndvar->cwnd = 1;
	ParseTCPOptions(s, pctx->p.cur_ts, (uint8_t *)pctx->p.tcph + TCP_HEADER_LEN,
	                (pctx->p.tcph->doff << 2) - TCP_HEADER_LEN);
	return s;
}

/* CreateStream, tcp.c:195-256: a stream only for an initial SYN some socket wants.
 * SYN / ACK come from the record's flags byte (header byte 13). */
static tcp_stream *create_stream(struct rx_view *v, int index, mtcp_manager_t mtcp, struct pkt_ctx *pctx,
                                 unsigned int *hash)
{
	const uint8_t flags = rec_flags(v, index);
	uint32_t type;
	if (!((flags & TCP_FLAG_SYN) && !(flags & TCP_FLAG_ACK)))
		return NULL;
	type = detect_stream_type(v, index, mtcp, pctx, pctx->p.iph->daddr, pctx->p.tcph->dest);
	if (!type)
		return NULL;
	if (type == STREAM_TYPE(MOS_SOCK_STREAM))
		return server_stream(mtcp, type, pctx);
	if (type & STREAM_TYPE(MOS_SOCK_MONITOR_STREAM_ACTIVE))
		return CreateClientTCPStream(mtcp, NULL, type, pctx->p.iph->saddr, pctx->p.tcph->source,
		                             pctx->p.iph->daddr, pctx->p.tcph->dest, hash);
	return NULL;
}

/* HandleMonitorStream, tcp.c:377-406 */
static void monitor_stream(mtcp_manager_t mtcp, tcp_stream *snd, struct pkt_ctx *pctx)
{
	tcp_stream *rcv;
	UpdateMonitor(mtcp, snd, snd->pair_stream, pctx, true);
	rcv = snd->pair_stream;
	if (HAS_STREAM_TYPE(rcv, MOS_SOCK_STREAM)) {
		DoActionEndTCPPacket(mtcp, rcv, pctx);
		return;
	}
	if (pctx->forward)
		ForwardIPPacket(mtcp, pctx);
	if (rcv->stream_type == snd->stream_type && IS_STREAM_TYPE(rcv, MOS_SOCK_MONITOR_STREAM_ACTIVE)) {
		/* both sides finished (or unmonitored): the pair goes */
		const int rcv_done = (rcv->state == TCP_ST_TIME_WAIT && g_config.mos->tcp_tw_interval == 0) ||
		                     rcv->state == TCP_ST_CLOSED_RSVD || !rcv->status_mgmt;
		const int snd_done = (snd->state == TCP_ST_TIME_WAIT && g_config.mos->tcp_tw_interval == 0) ||
		                     snd->state == TCP_ST_CLOSED_RSVD || !snd->status_mgmt;
		if (rcv_done && snd_done)
			DestroyTCPStream(mtcp, rcv);
	}
}

#endif

/* tcp.c:445-514 for a segment that passed the checks. */
static int stream_step(struct rx_view *v, int index, mtcp_manager_t mtcp, struct pkt_ctx *pctx)
{
	struct iphdr *iph = pctx->p.iph;
	struct tcphdr *tcph = pctx->p.tcph;
	uint64_t events = MOS_ON_PKT_IN;
	unsigned int hash = 0;
	tcp_stream key, *cur;
	struct mon_listener *walk;

	stats_of(mtcp)->stream_step++;
	/* FindStream (tcp.c:181-191): the flow as the stream stores it, reversed */
	key.saddr = iph->daddr;
	key.sport = tcph->dest;
	key.daddr = iph->saddr;
	key.dport = tcph->source;
	cur = find_stream(v, index, mtcp, &key, &hash);
	if (!cur) {
		if (mtcp->listener == NULL && mtcp->num_msp == 0)
			return TRUE;                  /* a client-only end host: nothing to do (tcp.c:454-458) */
#ifdef MOSRX_MOS_TCP_EXPORTS
		cur = CreateStream(mtcp, pctx, &hash);
#else
		cur = create_stream(v, index, mtcp, pctx, &hash);
#endif
		if (!cur)
			events = MOS_ON_ORPHAN;
	}
	if (cur) {
		cur->cb_events = events;
		if (cur->rcvvar && cur->rcvvar->rcvbuf)
			pctx->p.offset = (uint64_t)seq2loff(cur->rcvvar->rcvbuf, pctx->p.seq, cur->rcvvar->irs + 1);
#ifdef MOSRX_MOS_TCP_EXPORTS
		if (IS_STREAM_TYPE(cur, MOS_SOCK_STREAM))
			HandleSockStream(mtcp, cur, pctx);
		else if (HAS_STREAM_TYPE(cur, MOS_SOCK_MONITOR_STREAM_ACTIVE))
			HandleMonitorStream(mtcp, cur, cur->pair_stream, pctx);
#else
		if (IS_STREAM_TYPE(cur, MOS_SOCK_STREAM)) {
			UpdateRecvTCPContext(mtcp, cur, pctx);    /* HandleSockStream, tcp.c:275-281 */
			DoActionEndTCPPacket(mtcp, cur, pctx);
		} else if (HAS_STREAM_TYPE(cur, MOS_SOCK_MONITOR_STREAM_ACTIVE)) {
			monitor_stream(mtcp, cur, pctx);
		}
#endif
		return TRUE;
	}
	/* an orphan: MOS_ON_ORPHAN for every monitor whose orphan filter takes it */
	TAILQ_FOREACH(walk, &mtcp->monitors, link) {
		const struct sfbpf_program *fc = &walk->stream_orphan_fcode;
		if (!(ISSET_BPFFILTER((*fc)) &&
		      filter_eval(v, index, fc, MOSRX_BPF_LEN_IP, (uint8_t *)pctx->p.iph - sizeof(struct ethhdr),
		                  pctx->p.ip_len + sizeof(struct ethhdr)) == 0))
			HandleCallback(mtcp, MOS_NULL, walk->socket, MOS_SIDE_BOTH, pctx, events);
	}
	if (mtcp->listener) {
		if (!(rec_flags(v, index) & TCP_FLAG_RST))   /* RFC 793: a RST is never answered */
			SendTCPPacketStandalone(mtcp, iph->daddr, tcph->dest, iph->saddr, tcph->source, 0,
			                        pctx->p.seq + pctx->p.payloadlen + 1, 0, TCP_FLAG_RST | TCP_FLAG_ACK,
			                        NULL, 0, pctx->p.cur_ts, 0, 0, -1);
	} else if (pctx->forward) {
		ForwardIPPacket(mtcp, pctx);
	}
	return TRUE;
}

/* ---- the frame ----------------------------------------------------------- */

static void release(mtcp_manager_t mtcp, struct pkt_ctx *pctx)
{
	if (mtcp->iom->release_pkt)
		mtcp->iom->release_pkt(mtcp->ctx, pctx->p.in_ifidx, (unsigned char *)pctx->p.ethh, pctx->p.eth_len);
}

/* The IPv4 part, ProcessInIPv4Packet (ip_in.c:30-101) + ProcessInTCPPacket
 * (tcp.c:408-514), from the record. */
static int ipv4(struct rx_view *v, int index, mtcp_manager_t mtcp, struct pkt_ctx *pctx)
{
	uint8_t reason = rec_reason(v, index);
	struct iphdr *iph = (struct iphdr *)((uint8_t *)pctx->p.ethh + sizeof(struct ethhdr));
	struct mon_listener *walk;

	if (reason == MOSRX_R_IP_SHORT)
		return ERROR;
	if (reason == MOSRX_R_IP_BADVER) {
		release(mtcp, pctx);
		return FALSE;
	}
	pctx->p.iph = iph;                           /* FillInPacketIPContext, ip_in.c:21-28 */
	pctx->p.ip_len = ntohs(iph->tot_len);
	TAILQ_FOREACH(walk, &mtcp->monitors, link)   /* raw monitors, ip_in.c:56-63 */
		if (walk->socket->socktype == MOS_SOCK_MONITOR_RAW && ISSET_BPFFILTER(walk->raw_pkt_fcode) &&
		    filter_eval(v, index, &walk->raw_pkt_fcode, MOSRX_BPF_LEN_FRAME, (uint8_t *)pctx->p.ethh,
		                pctx->p.eth_len))
			HandleCallback(mtcp, MOS_NULL, walk->socket, MOS_SIDE_BOTH, pctx, MOS_ON_PKT_IN);
	/* the verify gate (ip_in.c:67) reads the socket counts now: records made
	 * on the other side of it (a socket came or went since the batch was
	 * classified) are made again first */
	if (((mtcp->num_msp || mtcp->num_esp) != 0) != ((v->state.num_msp || v->state.num_esp) != 0))
		view_reclassify(v, mtcp, v->ifidx, index);
	if (v->dead_from >= 0) {                     /* no records for the rest of the batch: dropped */
		stats_of(mtcp)->gpu_dropped++;
		release(mtcp, pctx);
		return ERROR;
	}
	reason = rec_reason(v, index);               /* (a filter install reclassifies the batch too) */
	if (mtcp->num_msp == 0 && mtcp->num_esp == 0) {
		if (pctx->forward)
			ForwardIPPacket(mtcp, pctx);
		return TRUE;
	}
	if (reason == MOSRX_R_IP_BADCSUM)
		return ERROR;
	if (reason == MOSRX_R_ICMP_LOCAL && ProcessICMPPacket(mtcp, pctx))
		return TRUE;
	if (reason == MOSRX_R_NOT_TCP || reason == MOSRX_R_ICMP_LOCAL) {
		if (!mtcp->num_msp || !pctx->forward)
			release(mtcp, pctx);
		else
			ForwardIPPacket(mtcp, pctx);
		return FALSE;
	}
	/* TCP: mOS's own FillPacketContextTCPInfo (tcp.c:258-270; an external
	 * definition under -fgnu89-inline) on the header as ProcessInTCPPacket
	 * finds it (tcp.c:417): pkt_info's payload, payloadlen (u16, before the
	 * length check), seq, ack_seq, window.  The record's verdict says these
	 * bytes lie inside the capture (TRUNCATED frames never get here) */
	FillPacketContextTCPInfo(pctx, (struct tcphdr *)((uint8_t *)iph + (iph->ihl << 2)));
	TAILQ_FOREACH(walk, &mtcp->monitors, link)   /* tcp.c:424-427 */
		if (walk->socket->socktype == MOS_SOCK_MONITOR_RAW)
			HandleCallback(mtcp, MOS_NULL, walk->socket, MOS_SIDE_BOTH, pctx, MOS_ON_PKT_IN);
	if (reason == MOSRX_R_TCP_SHORT)
		return ERROR;
	if (reason == MOSRX_R_TCP_BADCSUM) {
		if (pctx->forward && mtcp->num_msp)
			ForwardIPPacket(mtcp, pctx);
		return ERROR;
	}
	return stream_step(v, index, mtcp, pctx);   /* TCP_OK (TCP_LEN_OK: skip_tcp_csum runs, nothing verified) */
}

int mosrx_mos_process_packet(struct mtcp_manager *mtcp, const int ifidx, const int index, uint32_t cur_ts,
                             unsigned char *pkt_data, int len)
{
	struct rx_view *v = &t_view;
	struct pkt_ctx pctx;
	uint8_t reason;
	int ret;

	if (index == 0 || v->mtcp != mtcp || v->ifidx != ifidx || (!v->res && !v->res8 && v->dead_from < 0)) {
		view_fetch(v, mtcp, ifidx);
		if (index == 0 && v->dead_from < 0)
			filters_check(v, mtcp, ifidx);
	}
	if (v->dead_from < 0 && (index < 0 || (uint32_t)index >= v->state.n))
		view_lost(v, mtcp, 0, "frame index past the batch's records");
	stats_of(mtcp)->frames++;

#ifdef NETSTAT
	mtcp->nstat.rx_packets[ifidx]++;
	mtcp->nstat.rx_bytes[ifidx] += len + ETHER_OVR;
#endif
	/* no records (a negative index has none either): dropped, as a NIC would */
	if (v->dead_from >= 0 && (index < 0 || index >= v->dead_from)) {
		stats_of(mtcp)->gpu_dropped++;
		if (mtcp->iom->release_pkt)
			mtcp->iom->release_pkt(mtcp->ctx, ifidx, pkt_data, len);
#ifdef NETSTAT
		mtcp->nstat.rx_errors[ifidx]++;
#endif
		return ERROR;
	}
	reason = rec_reason(v, index);
	memset(&pctx, 0, sizeof(pctx));              /* FillInPacketEthContext, eth_in.c:12-25 */
	pctx.p.cur_ts = cur_ts;
	pctx.p.in_ifidx = ifidx;
	pctx.out_ifidx = -1;
	pctx.p.ethh = (struct ethhdr *)pkt_data;
	pctx.p.eth_len = len;
	pctx.batch_index = index;
	pctx.forward = g_config.mos->forward;

	if (reason == MOSRX_R_ARP || reason == MOSRX_R_NON_IPV4) {
		if (!mtcp->num_msp || !pctx.forward) {
			if (reason == MOSRX_R_ARP) {
				ProcessARPPacket(mtcp, cur_ts, ifidx, pkt_data, len);
				return TRUE;
			}
			DumpPacket(mtcp, (char *)pkt_data, len, "??", ifidx);
			if (mtcp->iom->release_pkt)
				mtcp->iom->release_pkt(mtcp->ctx, ifidx, pkt_data, len);
			ret = ERROR;
		} else {
			ForwardEthernetFrame(mtcp, &pctx);
			return TRUE;
		}
	} else if (reason == MOSRX_R_TRUNCATED) {
		if (mtcp->iom->release_pkt)
			mtcp->iom->release_pkt(mtcp->ctx, ifidx, pkt_data, len);
		ret = ERROR;
	} else {
		ret = ipv4(v, index, mtcp, &pctx);
	}
#ifdef NETSTAT
	if (ret < 0)
		mtcp->nstat.rx_errors[ifidx]++;
#endif
	return ret;
}
