/*
 * ref_harness.c — TEST INFRASTRUCTURE ONLY.
 *
 * Drives mOS's OWN compiled receive path (core/src objects built by
 * oracle/ref.mk from /root/reference, output in oracle/_ref/) over a trace
 * file, to pin the C restatement in mosrx_oracle.c and to generate the golden
 * vectors under tests/golden/.  It follows the reference's fake-backend test
 * pattern (core/test/scalable_event/test.c:21-43): a static mtcp_manager and
 * a zeroed io_module_func instead of a running stack.
 *
 * Usage: mosref <trace.in> <results.out>
 *   trace.in : "MRXT" | u32 ver (1 or 2) | u32 n | u64 frames_bytes |
 *              u32 num_msp | u32 num_esp | i32 forward | i32 num_queues | i32 queue_mode |
 *              [ver 2: u32 nlocal | u32 local_ip[16] (netdev ip_addr, network order)] |
 *              u32 off[n] | u16 len[n] | u8 frames[frames_bytes]
 *   results  : n x { i8 verdict, u8 have, u16 ip_csum, u16 tcp_csum, u16 fwd, u32 rss, i32 queue,
 *                    u32 fbucket,
 *                    u16 payloadlen, u16 payload_off, u32 seq, u32 ack_seq, u16 window,
 *                    u8 tcp_flags, u8 ihl_doff, u16 ip_len, u16 pad }
 *              then u64 rx_packets, rx_bytes, rx_errors (NETSTAT, eth_in.c:42-45,80-84)
 *   have bit0: ip_csum computed, bit1: tcp_csum computed, bit2: rss computed,
 *        bit3: frame skipped (would make the reference read past caplen),
 *        bit4: fbucket computed (TCP frames),
 *        bit5: pkt_info TCP fields computed (TCP frames): mOS's own
 *              FillInPacketIPContext (ip_in.c:21-27) + FillPacketContextTCPInfo
 *              (tcp.c:258-270) on a pkt_ctx, so payloadlen, payload - ethh, seq,
 *              ack_seq and window are the values ProcessInTCPPacket hands on;
 *              tcp_flags / ihl_doff are the tcphdr / iphdr bitfields it reads.
 *
 * The local addresses become netdev_table entries (config.h:54-74): ICMP frames
 * to one of them take ProcessICMPPacket's "to me" branch (icmp.c:187-227).  The
 * route table is empty, so an echo request's reply finds no output interface
 * (ip_out.c:12-37) and nothing is sent.
 *
 * forward (mos.conf `forward`, 0 or 1): mOS's forwarding calls need route /
 * ARP tables and TX buffers, so ForwardIPPacket and
 * ForwardEthernetFrame are wrapped (-Wl,--wrap) to record the call instead:
 * `fwd` is 1 when ProcessPacket forwarded the frame (eth_in.c:60-77,
 * ip_in.c:66-70 / :86-91, tcp.c:438-442, the stream engine's forward of a
 * monitor-only stack), which is what mosrx_mos_forwards must decide.
 * MOSREF_LISTENER=<port> in the environment gives the manager an end-host
 * listening socket on that port (INADDR_ANY, mtcp_listen's state that
 * ProcessInTCPPacket reads: tcp.c:453, :497-506; DetectStreamType :54-75);
 * with a port no frame targets, frames of unknown flows take the orphan path.
 *
 * Usage: mosref --time-pp <trace.in> <seconds>
 *   mOS's whole ProcessPacket (eth_in.c:27-87) on every frame, under the trace
 *   header's stack state (the flow table stays empty: no monitor socket is
 *   listening, so FindStream creates nothing), passes repeated for at least
 *   <seconds>; one JSON line.  The reference's per-frame rx cost as the rx loop
 *   pays it, stream lookup included.
 *
 * Usage: mosref --time <trace.in> <seconds> [threads]
 *   CPU baseline of the reference's own per-frame arithmetic on this host: the
 *   header checks of eth_in.c / ip_in.c / tcp.c, ip_fast_csum, TCPCalcChecksum,
 *   GetRSSHash and GetRSSCPUCore over every frame,
 *   passes repeated for at least <seconds>.  Prints one JSON line.  With
 *   `threads` > 1, one pthread per disjoint slice of the trace, all started
 *   together, each repeating passes over its own slice (mOS's per-core
 *   sharding: one mTCP thread per core, each on its own RSS queue's frames,
 *   core.c:1369-1466); the rate is every thread's frames over the longest
 *   thread's time.  ProcessPacket itself is not timed: past the checksum it
 *   runs FindStream and the stateful flow engine (out of scope).
 */
#include <arpa/inet.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "mtcp.h"
#include "config.h"
#include "io_module.h"
#include "ip_in.h"
#include "eth_in.h"
#include "tcp_util.h"
#include "fhash.h"
#include "logger.h"
#include "mtcp_util.h"
#include "tcp.h"
#include "socket.h"

int ProcessPacket(mtcp_manager_t mtcp, const int ifidx, const int index,
                  uint32_t cur_ts, unsigned char *pkt_data, int len);
uint32_t GetRSSHash(in_addr_t sip, in_addr_t dip, in_port_t sp, in_port_t dp);   /* util.c:61-62, no header declares it */
uint16_t TCPCalcChecksum(uint16_t *buf, uint16_t len, uint32_t saddr, uint32_t daddr);
void FillInPacketIPContext(struct pkt_ctx *pctx, struct iphdr *iph, int ip_len);   /* ip_in.c:21, gnu89 inline */

static int g_qmode = 1;
int __wrap_FetchEndianType(void) { return g_qmode; }

static int g_fwd;
void __wrap_ForwardIPPacket(mtcp_manager_t mtcp, struct pkt_ctx *pctx) { (void)mtcp; (void)pctx; g_fwd++; }
void __wrap_ForwardEthernetFrame(struct mtcp_manager *mtcp, struct pkt_ctx *pctx) { (void)mtcp; (void)pctx; g_fwd++; }

struct rec {
	int8_t verdict;
	uint8_t have;
	uint16_t ip_csum, tcp_csum, fwd;    /* fwd: ProcessPacket called a Forward* function */
	uint32_t rss;
	int32_t queue;
	uint32_t fbucket;   /* HashFlow() of FindStream's reversed tuple (tcp.c:185-190, fhash.c:72-92) */
	uint16_t payloadlen, payload_off;   /* pctx->p.payloadlen, pctx->p.payload - ethh */
	uint32_t seq, ack_seq;              /* pctx->p.seq, pctx->p.ack_seq (host order) */
	uint16_t window;                    /* pctx->p.window (host order) */
	uint8_t tcp_flags, ihl_doff;        /* tcph byte 13; (iph->ihl << 4) | tcph->doff */
	uint16_t ip_len, pad2;              /* pctx->p.ip_len */
};
_Static_assert(sizeof(struct rec) == 40, "record layout");

unsigned int HashFlow(const tcp_stream *flow);

static int rd(FILE *f, void *p, size_t n) { return fread(p, 1, n, f) == n ? 0 : -1; }

/* The scope of the GPU transform, computed by the reference's own functions. */
static uint32_t ref_frame(const uint8_t *f, uint32_t cap, int nq)
{
	struct iphdr *iph;
	struct tcphdr *th;
	unsigned ihl, ip_len, proto;
	uint32_t acc;
	uint16_t sp = 0, dp = 0;
	if (cap < 34 || f[12] != 0x08 || f[13] != 0x00)
		return 0;
	iph = (struct iphdr *)(f + 14);
	ihl = iph->ihl;
	ip_len = ntohs(iph->tot_len);
	proto = iph->protocol;
	if (ip_len < 20 || iph->version != 4 || 14 + ihl * 4 > cap || 14 + ip_len > cap ||
	    (proto == 6 && 14 + ihl * 4 + 20 > cap))
		return 1;
	acc = ip_fast_csum(iph, ihl);
	th = (struct tcphdr *)((uint8_t *)iph + ihl * 4);
	if (proto == 6) {
		sp = ntohs(th->source);
		dp = ntohs(th->dest);
		if (ip_len >= (ihl + th->doff) * 4) {
			uint16_t payloadlen = ip_len - (ihl * 4 + th->doff * 4);
			acc += TCPCalcChecksum((uint16_t *)th, (th->doff << 2) + payloadlen, iph->saddr, iph->daddr);
		}
	}
	acc += GetRSSHash(ntohl(iph->saddr), ntohl(iph->daddr), sp, dp);
	acc += (uint32_t)GetRSSCPUCore(ntohl(iph->saddr), ntohl(iph->daddr), sp, dp, nq);
	return acc;
}

static double now_s(void)
{
	struct timespec ts;
	clock_gettime(CLOCK_MONOTONIC, &ts);
	return ts.tv_sec + ts.tv_nsec * 1e-9;
}

struct slice {
	const uint32_t *off;
	const uint16_t *len;
	const uint8_t *frames;
	uint32_t lo, hi;
	int nq;
	double seconds, el;
	uint64_t passes;
	uint32_t sink;
	pthread_barrier_t *go;
};

static void *slice_run(void *arg)
{
	struct slice *s = arg;
	uint32_t i, sink = 0;
	uint64_t passes = 0;
	double t0, el;
	pthread_barrier_wait(s->go);
	t0 = now_s();
	do {
		for (i = s->lo; i < s->hi; i++)
			sink += ref_frame(s->frames + s->off[i], s->len[i], s->nq);
		passes++;
		el = now_s() - t0;
	} while (el < s->seconds);
	s->el = el;
	s->passes = passes;
	s->sink = sink;
	return NULL;
}

static int time_mode(uint32_t n, const uint32_t *off, const uint16_t *len, const uint8_t *frames, int nq,
                     double seconds, int threads)
{
	struct slice *sl;
	pthread_t *th;
	pthread_barrier_t go;
	uint64_t frames_done = 0, bytes_done = 0, passes = 0;
	uint32_t i, sink = 0;
	double el = 0;
	int t;
	if (threads < 1 || (uint32_t)threads > n)
		threads = 1;
	sl = calloc((size_t)threads, sizeof(*sl));
	th = calloc((size_t)threads, sizeof(*th));
	if (!sl || !th || pthread_barrier_init(&go, NULL, (unsigned)threads))
		return 1;
	for (t = 0; t < threads; t++) {
		sl[t] = (struct slice){off, len, frames, (uint32_t)((uint64_t)n * t / threads),
		                       (uint32_t)((uint64_t)n * (t + 1) / threads), nq, seconds, 0, 0, 0, &go};
		if (t && pthread_create(&th[t], NULL, slice_run, &sl[t]))
			return 1;
	}
	slice_run(&sl[0]);
	for (t = 1; t < threads; t++)
		pthread_join(th[t], NULL);
	for (t = 0; t < threads; t++) {
		uint64_t b = 0;
		for (i = sl[t].lo; i < sl[t].hi; i++)
			b += len[i];
		frames_done += (uint64_t)(sl[t].hi - sl[t].lo) * sl[t].passes;
		bytes_done += b * sl[t].passes;
		passes += sl[t].passes;
		sink += sl[t].sink;
		el = sl[t].el > el ? sl[t].el : el;
	}
	printf("{\"frames\": %u, \"threads\": %d, \"passes\": %llu, \"seconds\": %.3f, \"mpkts\": %.4f, "
	       "\"caplen_gbps\": %.4f, \"sink\": %u}\n",
	       n, threads, (unsigned long long)passes, el, (double)frames_done / el / 1e6, (double)bytes_done / el / 1e9,
	       sink);
	pthread_barrier_destroy(&go);
	free(sl);
	free(th);
	return 0;
}

int main(int argc, char **argv)
{
	FILE *in, *out;
	char magic[4];
	uint32_t ver, n, i;
	uint64_t fb;
	uint32_t num_msp, num_esp, nlocal = 0, local_ip[16];
	int32_t forward, nq, qmode;
	uint32_t *off;
	uint16_t *len;
	uint8_t *frames;
	static struct mtcp_manager m;
	static struct mtcp_thread_context tctx;
	static struct mos_conf mc;
	static struct netdev_conf nd;
	static struct netdev_entry nde[16];
	static struct route_conf rt;
	static io_module_func null_iom;
	static log_thread_context lg;

	int timing = (argc == 4 || argc == 5) && !strcmp(argv[1], "--time");
	const int threads = timing && argc == 5 ? atoi(argv[4]) : 1;
	const int timing_pp = argc == 4 && !strcmp(argv[1], "--time-pp");
	if (argc != 3 && !timing && !timing_pp) {
		fprintf(stderr, "usage: %s trace.in results.out | %s --time trace.in seconds [threads] | "
		        "%s --time-pp trace.in seconds\n", argv[0], argv[0], argv[0]);
		return 2;
	}
	if (timing_pp)
		argv++;
	if (timing)
		argv++;
	in = fopen(argv[1], "rb");
	if (!in || rd(in, magic, 4) || memcmp(magic, "MRXT", 4) || rd(in, &ver, 4) || (ver != 1 && ver != 2) ||
	    rd(in, &n, 4) || rd(in, &fb, 8) || rd(in, &num_msp, 4) || rd(in, &num_esp, 4) ||
	    rd(in, &forward, 4) || rd(in, &nq, 4) || rd(in, &qmode, 4) ||
	    (ver == 2 && (rd(in, &nlocal, 4) || nlocal > 16 || rd(in, local_ip, sizeof(local_ip))))) {
		fprintf(stderr, "bad trace header\n");
		return 1;
	}
	if ((forward != 0 && forward != 1) || nq < 1) {
		fprintf(stderr, "forward must be 0 or 1 and num_queues >= 1\n");
		return 1;
	}
	off = malloc((size_t)n * 4 + 1);
	len = malloc((size_t)n * 2 + 1);
	frames = calloc(fb + 64, 1); /* +64: the masked odd-tail read may touch one byte past a frame */
	if (!off || !len || !frames || rd(in, off, (size_t)n * 4) || rd(in, len, (size_t)n * 2) ||
	    rd(in, frames, fb)) {
		fprintf(stderr, "short trace\n");
		return 1;
	}
	fclose(in);
	g_qmode = qmode;
	if (timing)
		return time_mode(n, off, len, frames, nq, atof(argv[2]), threads);

	/* stack state: core.c:1079-1110 InitializeMTCPManager, reduced */
	nd.num = (int)nlocal;
	for (i = 0; i < nlocal; i++) {
		nde[i].ip_addr = local_ip[i];
		nd.ent[i] = &nde[i];
	}
	rt.num = 0;
	mc.forward = forward;
	mc.netdev_table = &nd;
	mc.route_table = &rt;
	g_config.mos = &mc;
	tctx.cpu = 0;
	tctx.mtcp_manager = &m;
	TAILQ_INIT(&m.monitors);
	m.num_msp = num_msp;
	m.num_esp = num_esp;
	m.tcp_flow_table = CreateHashtable();
	m.iom = &null_iom;
	m.ctx = &tctx;
	InitLogThreadContext(&lg, 0);
	m.logger = &lg;
	m.log_fp = fopen("/dev/null", "w");
	if (getenv("MOSREF_LISTENER")) {
		static struct tcp_listener lst;
		static struct socket_map lsock;
		lsock.socktype = MOS_SOCK_STREAM_LISTEN;
		lsock.saddr.sin_family = AF_INET;
		lsock.saddr.sin_addr.s_addr = INADDR_ANY;
		lsock.saddr.sin_port = htons((uint16_t)atoi(getenv("MOSREF_LISTENER")));
		lst.socket = &lsock;
		m.listener = &lst;
	}

	if (timing_pp) {   /* every frame through ProcessPacket, as the rx loop calls it (core.c:906) */
		uint64_t passes = 0, bytes = 0;
		uint32_t sink = 0;
		const double seconds = atof(argv[2]);
		double t0, el;
		for (i = 0; i < n; i++)
			bytes += len[i];
		t0 = now_s();
		do {
			for (i = 0; i < n; i++)
				sink += (uint32_t)ProcessPacket(&m, 0, (int)i, 0, frames + off[i], (int)len[i]);
			passes++;
			el = now_s() - t0;
		} while (el < seconds);
		printf("{\"frames\": %u, \"passes\": %llu, \"seconds\": %.3f, \"mpkts\": %.4f, "
		       "\"caplen_gbps\": %.4f, \"sink\": %u}\n",
		       n, (unsigned long long)passes, el, (double)n * passes / el / 1e6, (double)bytes * passes / el / 1e9,
		       sink);
		return 0;
	}
	out = fopen(argv[2], "wb");
	if (!out)
		return 1;
	for (i = 0; i < n; i++) {
		uint8_t *f = frames + off[i];
		uint32_t cap = len[i];
		struct rec r;
		memset(&r, 0, sizeof(r));
		if (cap < 14) {
			r.have = 8;
		} else if (f[12] == 0x08 && f[13] == 0x00) {
			struct iphdr *iph = (struct iphdr *)(f + 14);
			if (cap < 34) {
				r.have = 8;
			} else {
				unsigned ihl = iph->ihl, ip_len = ntohs(iph->tot_len), proto = iph->protocol;
				if (14 + ihl * 4 > cap || 14 + ip_len > cap || (proto == 6 && 14 + ihl * 4 + 20 > cap)) {
					r.have = 8;
				} else {
					struct tcphdr *th = (struct tcphdr *)((uint8_t *)iph + ihl * 4);
					uint16_t sp = proto == 6 ? ntohs(th->source) : 0;
					uint16_t dp = proto == 6 ? ntohs(th->dest) : 0;
					r.ip_csum = ip_fast_csum(iph, ihl);
					r.have |= 1;
					if (proto == 6 && ip_len >= (ihl + th->doff) * 4) {
						uint16_t payloadlen = ip_len - (ihl * 4 + th->doff * 4);
						r.tcp_csum = TCPCalcChecksum((uint16_t *)th, (th->doff << 2) + payloadlen,
						                             iph->saddr, iph->daddr);
						r.have |= 2;
					}
					r.rss = GetRSSHash(ntohl(iph->saddr), ntohl(iph->daddr), sp, dp);
					r.queue = GetRSSCPUCore(ntohl(iph->saddr), ntohl(iph->daddr), sp, dp, nq);
					r.have |= 4;
					if (proto == 6) {   /* FindStream's temp stream, tcp.c:185-190 */
						static tcp_stream ts;
						struct pkt_ctx pctx;
						ts.saddr = iph->daddr;
						ts.sport = th->dest;
						ts.daddr = iph->saddr;
						ts.dport = th->source;
						r.fbucket = HashFlow(&ts);
						r.have |= 16;
						/* ProcessInIPv4Packet -> ProcessInTCPPacket's context fill */
						memset(&pctx, 0, sizeof(pctx));
						pctx.p.ethh = (struct ethhdr *)f;
						FillInPacketIPContext(&pctx, iph, (int)ip_len);
						FillPacketContextTCPInfo(&pctx, th);
						r.payloadlen = pctx.p.payloadlen;
						r.payload_off = (uint16_t)(pctx.p.payload - (uint8_t *)pctx.p.ethh);
						r.seq = pctx.p.seq;
						r.ack_seq = pctx.p.ack_seq;
						r.window = pctx.p.window;
						r.tcp_flags = ((uint8_t *)th)[13];
						r.ihl_doff = (uint8_t)((iph->ihl << 4) | th->doff);
						r.ip_len = pctx.p.ip_len;
						r.have |= 32;
					}
				}
			}
		}
		if (!(r.have & 8)) {
			g_fwd = 0;
			r.verdict = (int8_t)ProcessPacket(&m, 0, (int)i, 0, f, (int)cap);
			r.fwd = g_fwd > 0;
		}
		fwrite(&r, sizeof(r), 1, out);
	}
	fwrite(&m.nstat.rx_packets[0], 8, 1, out);
	fwrite(&m.nstat.rx_bytes[0], 8, 1, out);
	fwrite(&m.nstat.rx_errors[0], 8, 1, out);
	fclose(out);
	return 0;
}
