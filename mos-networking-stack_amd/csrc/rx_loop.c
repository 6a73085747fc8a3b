/*
 * rx_loop.c — the receive half of RunMainLoop (core.c:897-909) over any
 * io_module_func, consuming the GPU verdicts instead of re-running the checks,
 * and the per-round flush of frames written for transmission (core.c:999-1007).
 *
 *   for rx_inf in netdevs:                        core.c:897
 *     recv_cnt = iom->recv_pkts(ctx, rx_inf)      core.c:899
 *     for i < recv_cnt:                           core.c:902
 *       pkt = iom->get_rptr(ctx, rx_inf, i, &len) core.c:905
 *       ProcessPacket(...)                        core.c:906 -> here: NETSTAT + fn()
 *   for tx_inf in netdevs:                        core.c:999-1007
 *     iom->send_pkts(ctx, tx_inf)
 *
 * NETSTAT follows eth_in.c:42-45 and :80-84: rx_packets++, rx_bytes += len +
 * ETHER_OVR (24, mtcp.h:58), rx_errors++ when the verdict is negative.
 */
#include <errno.h>
#include <string.h>
#include <time.h>
#include <unistd.h>

#include "../../include/mosrx_io_module.h"

#define ETHER_OVR 24

static uint64_t now_ns(void);
static void latency_batch(mosrx_latency_probe *p, uint64_t n, uint64_t t_avail, uint64_t t_end);

static uint64_t now_us(void)
{
	struct timespec ts;
	clock_gettime(CLOCK_MONOTONIC, &ts);
	return (uint64_t)ts.tv_sec * 1000000u + (uint64_t)ts.tv_nsec / 1000u;
}

int mosrx_rx_loop_ex(const io_module_func *iom, struct mtcp_thread_context *ctx, int nif,
                     const mosrx_rx_loop_opts *o, mosrx_pkt_fn fn, void *arg, mosrx_rx_stats *st)
{
	int rx_inf;
	uint32_t idle = 0;
	uint64_t t0;
	if (!iom || !iom->recv_pkts || !iom->get_rptr || !st || !o || nif <= 0)
		return -EINVAL;
	memset(st, 0, sizeof(*st));
	t0 = o->max_us ? now_us() : 0;
	for (;;) {
		int any = 0;
		st->rounds++;
		for (rx_inf = 0; rx_inf < nif; rx_inf++) {
			const mosrx_result *res = NULL;
			const mosrx_result8 *res8 = NULL;
			mosrx_result one;
			int32_t recv_cnt = iom->recv_pkts(ctx, rx_inf);
			int32_t i;
			const uint64_t t_avail = o->probe && recv_cnt > 0 ? now_ns() : 0;
			if (recv_cnt < 0) {        /* RunMainLoop's for loop just skips it (core.c:899-902) */
				st->recv_errors++;
				continue;
			}
			if (recv_cnt == 0)
				continue;
			any = 1;
			st->batches++;
			/* the backend must be a classifying one: 16-byte records, or a compact batch's 8-byte ones */
			if (!iom->dev_ioctl ||
			    ((iom->dev_ioctl(ctx, rx_inf, MOSRX_PKT_RX_RESULTS, &res) || !res) &&
			     (iom->dev_ioctl(ctx, rx_inf, MOSRX_PKT_RX_RESULTS8, &res8) || !res8)))
				return -ENOTSUP;
			if (!res && !fn) {          /* 8-byte records, nothing to hand them to: the census only */
				for (i = 0; i < recv_cnt; i++) {
					uint16_t len = 0;
					if (!iom->get_rptr(ctx, rx_inf, i, &len))
						return -EIO;
					st->rx_packets++;
					st->rx_bytes += (uint64_t)len + ETHER_OVR;
					st->rx_errors += res8[i].verdict < 0;
					if (res8[i].reason < MOSRX_R_COUNT)
						st->by_reason[res8[i].reason]++;
				}
				if (o->probe)
					latency_batch(o->probe, (uint64_t)recv_cnt, t_avail, now_ns());
				continue;
			}
			memset(&one, 0, sizeof(one));
			for (i = 0; i < recv_cnt; i++) {
				uint16_t len = 0;
				const uint8_t *pkt = iom->get_rptr(ctx, rx_inf, i, &len);
				const mosrx_result *r = res ? &res[i] : &one;
				if (!pkt)
					return -EIO;
				if (!res) {           /* the compact record's fields, zero elsewhere */
					one.rss = res8[i].rss;
					one.reason = res8[i].reason;
					one.queue = res8[i].queue;
					one.verdict = res8[i].verdict;
					one.tcp_flags = res8[i].tcp_flags;
				}
				st->rx_packets++;
				st->rx_bytes += (uint64_t)len + ETHER_OVR;
				if (r->verdict < 0)
					st->rx_errors++;
				if (r->reason < MOSRX_R_COUNT)
					st->by_reason[r->reason]++;
				if (fn)
					fn(arg, rx_inf, i, pkt, len, r);
			}
			if (o->probe)
				latency_batch(o->probe, (uint64_t)recv_cnt, t_avail, now_ns());
		}
		if (iom->send_pkts)               /* core.c:999-1007: flush what the round wrote */
			for (rx_inf = 0; rx_inf < nif; rx_inf++)
				iom->send_pkts(ctx, rx_inf);
		if (o->max_pkts && st->rx_packets >= o->max_pkts)
			return 0;
		if (o->max_us && now_us() - t0 >= o->max_us)
			return 0;
		if (any) {
			idle = 0;
			continue;
		}
		if (o->idle_rounds && ++idle >= o->idle_rounds)
			return 0;
		if (o->idle_us)
			usleep(o->idle_us);
	}
}

int mosrx_rx_loop(const io_module_func *iom, struct mtcp_thread_context *ctx, int nif,
                  uint64_t max_pkts, mosrx_pkt_fn fn, void *arg, mosrx_rx_stats *st)
{
	const mosrx_rx_loop_opts o = {max_pkts, 1, 0, 0, NULL};   /* a finite source: stop at the first idle round */
	return mosrx_rx_loop_ex(iom, ctx, nif, &o, fn, arg, st);
}

/* ---- per-frame residency of a paced source (mosrx_rx_loop_opts.probe) ----
 * Frames from a paced source arrive at t0 + k * p and come through the
 * backend in order, so the k-th frame the loop receives is arrival k.  Per
 * batch of n frames starting at k0, the loop reads the clock twice: when
 * recv_pkts has returned it with its records (t_avail) and when its walk ends
 * (t_end).  Frame k0 + i then has
 *   recv -> verdict available  t_avail - (t0 + (k0 + i) p)
 *   recv -> consumed           t_avail + i (t_end - t_avail) / n - (t0 + (k0 + i) p)
 * (the walk taken as even over the batch), both linear in i, so each batch
 * goes into the log-spaced histograms by bins, not by frames: the probe costs
 * the loop two clock reads per batch, nothing per frame. */
static uint64_t now_ns(void)
{
	struct timespec ts;
	clock_gettime(CLOCK_MONOTONIC, &ts);
	return (uint64_t)ts.tv_sec * 1000000000ull + (uint64_t)ts.tv_nsec;
}

static uint32_t lat_bin(uint64_t v)
{
	uint32_t b;
	if (v < 16)
		return (uint32_t)v;
	b = 63u - (uint32_t)__builtin_clzll(v);
	return b * 16u + (uint32_t)((v >> (b - 4)) & 15u);
}

/* the lowest value of bin b + 1 (bins are contiguous and increasing) */
static double bin_end(uint32_t b)
{
	uint32_t e;
	if (b < 16)
		return (double)(b + 1);
	e = b / 16u;
	return (double)(16u + b % 16u + 1u) * (double)(1ull << (e - 4));
}

/* values a + i d, i in [0, n), clamped at 0, counted into hist; returns the largest */
static uint64_t hist_ramp(uint64_t *hist, double a, double d, uint64_t n)
{
	double lo = a, hi = a + d * (double)(n - 1);
	uint64_t done = 0;
	if (d < 0) {               /* count from the small end up: i runs backwards */
		a = hi;
		d = -d;
		hi = lo;
		lo = a;
	}
	while (done < n) {
		const double v = lo + d * (double)done;
		const uint32_t b = lat_bin(v > 0 ? (uint64_t)v : 0);
		uint64_t k;
		if (b >= MOSRX_LAT_BINS - 1 || d <= 0) {
			k = n - done;
		} else {
			/* values of this bin: v + j d < bin_end(b) */
			const double room = bin_end(b) - v;
			k = room > 0 ? (uint64_t)(room / d) + 1 : 1;
			if (k > n - done)
				k = n - done;
		}
		hist[b < MOSRX_LAT_BINS ? b : MOSRX_LAT_BINS - 1] += k;
		done += k;
	}
	return hi > 0 ? (uint64_t)hi : 0;
}

static void latency_batch(mosrx_latency_probe *p, uint64_t n, uint64_t t_avail, uint64_t t_end)
{
	uint64_t k0 = p->seen, skip = 0, m;
	double a;
	p->seen += n;
	if (!p->t0_ns && p->src)
		mosrx_source_paced_info(p->src, &p->t0_ns, &p->ns_per_frame, NULL);
	if (k0 + n <= p->skip || !p->t0_ns)
		return;
	if (k0 < p->skip)
		skip = p->skip - k0;
	k0 += skip;
	n -= skip;
	a = (double)t_avail - ((double)p->t0_ns + (double)k0 * p->ns_per_frame);
	m = hist_ramp(p->avail_hist, a, -p->ns_per_frame, n);
	if (m > p->avail_max_ns)
		p->avail_max_ns = m;
	m = hist_ramp(p->done_hist, a + (double)skip * (double)(t_end - t_avail) / (double)(n + skip),
	              (double)(t_end - t_avail) / (double)(n + skip) - p->ns_per_frame, n);
	if (m > p->done_max_ns)
		p->done_max_ns = m;
	p->recorded += n;
	p->batches++;
}

int mosrx_mos_forwards(const mosrx_result *res, int forward, uint32_t num_msp, uint32_t listener)
{
	if (!res || !forward)
		return 0;
	switch (res->reason) {
	case MOSRX_R_NON_IPV4:
	case MOSRX_R_ARP:             /* every non-IPv4 frame, ARP too, eth_in.c:60-77 */
	case MOSRX_R_NOT_TCP:
	case MOSRX_R_TCP_BADCSUM:
		return num_msp != 0;
	case MOSRX_R_NOVERIFY_PASS:
		return 1;
	case MOSRX_R_TCP_OK:
	case MOSRX_R_TCP_LEN_OK:
		return num_msp != 0 && !listener;     /* tcp.c:453-510, no stream for the flow */
	default:
		return 0;
	}
}

/* The frames mOS forwards (mosrx_mos_forwards), each as ForwardEthernetFrame
 * does (eth_out.c:105-129): the output netdev from the NIC forwarding table, a
 * TX buffer from get_wptr, a copy of the frame; the round's send_pkts sends it. */
void mosrx_forward_frame(void *arg, int ifidx, int index, const uint8_t *pkt, uint16_t len,
                         const mosrx_result *res)
{
	mosrx_forwarder *f = arg;
	int out;
	uint8_t *buf;
	(void)index;
	if (!f || !mosrx_mos_forwards(res, f->forward, f->num_msp, f->listener) || ifidx < 0 ||
	    ifidx >= MOSRX_MAX_DEVICES || (out = f->out_if[ifidx]) < 0 ||
	    !f->iom->get_wptr || !(buf = f->iom->get_wptr(f->ctx, out, len))) {
		if (f)
			f->dropped++;
		return;
	}
	memcpy(buf, pkt, len);
	f->forwarded++;
}
