/*
 * mos_gpu_loop.c — TEST INFRASTRUCTURE ONLY (tests/test_backend_gpu.py).
 *
 * gpu_module_func inside an mOS build, checked by mOS itself: this program is
 * linked from mOS's own compiled core/src objects (oracle/_ref/obj, built from
 * /root/reference by `make -C oracle ref`), csrc/gpu_module.c compiled against
 * mOS's io_module.h / config.h (-DMOSRX_HAVE_MOS_IO_MODULE) and libmosrx.so.
 * It registers the backend as core.c:1725-1736 would (current_iomodule_func,
 * load_module_upper_half, init_handle), receives a trace through it from an
 * in-memory source, and runs RunMainLoop's rx section (core.c:897-909) with
 * mOS's own ProcessPacket on every frame get_rptr hands out.  For each frame
 * the backend's GPU verdict must equal ProcessPacket's return value, and the
 * RSS hash behind dev_ioctl(PKT_RX_RSS) (mOS's own RssInfo) must equal
 * GetRSSHash; mOS's NETSTAT counters must equal the census of the GPU records.
 *
 * The stack state comes from the trace header (oracle/ref_harness.c format):
 * num_msp / num_esp into the mtcp_manager, the netdevs' addresses into
 * g_config.mos->netdev_table and `forward` into g_config.mos (both read back
 * by load_module_upper_half), num_queues and the queue map into the module's
 * configuration.  With forward set, mOS's own ForwardIPPacket /
 * ForwardEthernetFrame are wrapped (-Wl,--wrap: they would need route and ARP
 * tables and TX buffers) to record which frames ProcessPacket forwards; that
 * set must equal mosrx_mos_forwards() over the GPU records, the rule the rx
 * loop's forwarding consumer applies.  Frames whose headers claim bytes past
 * the capture (the reference reads past its buffer there) are passed over.
 *
 * With a period P (third argument) the application changes the stack state
 * every P batches -- mOS's num_msp toggles between the trace's value and 0, as
 * a monitor socket being created and closed would (socket.c:77-78) -- and the
 * backend must follow on its own: the thread context points at the
 * mtcp_manager (mtcp.h:304-312), and a batch classified in flight under the old
 * state is classified again before it is handed out.
 *
 * Usage: mos_gpu_loop <trace.in> <batch> [period [group]]   -- prints one JSON
 * line, exit 0 when every compared value is equal.  `group`: batches per launch
 * (cfg.group, the rx ring serviced at once).
 */
#include <arpa/inet.h>
#include <execinfo.h>
#include <signal.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "mtcp.h"
#include "config.h"
#include "io_module.h"
#include "fhash.h"
#include "logger.h"
#include "mtcp_util.h"
#include "socket.h"
#include "mosrx_io_module.h"

int ProcessPacket(mtcp_manager_t mtcp, const int ifidx, const int index,
                  uint32_t cur_ts, unsigned char *pkt_data, int len);
uint32_t GetRSSHash(in_addr_t sip, in_addr_t dip, in_port_t sp, in_port_t dp);   /* util.c:61-62, no header declares it */

static int g_qmode = 1;
int __wrap_FetchEndianType(void) { return g_qmode; }

/* mOS's forwarding calls, recorded instead of transmitted */
static int g_fwd;
void __wrap_ForwardIPPacket(mtcp_manager_t mtcp, struct pkt_ctx *pctx) { (void)mtcp; (void)pctx; g_fwd++; }
void __wrap_ForwardEthernetFrame(struct mtcp_manager *mtcp, struct pkt_ctx *pctx) { (void)mtcp; (void)pctx; g_fwd++; }

static int rd(FILE *f, void *p, size_t n) { return fread(p, 1, n, f) == n ? 0 : -1; }

/* a crash names where it happened (the test prints stderr) */
static const char *g_stage = "start";
static void on_segv(int sig)
{
	void *bt[32];
	const int k = backtrace(bt, 32);
	fprintf(stderr, "signal %d at stage %s\n", sig, g_stage);
	backtrace_symbols_fd(bt, k, 2);
	_exit(3);
}

/* ref_harness.c's rule: would the reference read past the capture? */
static int past_capture(const uint8_t *f, uint32_t cap)
{
	const struct iphdr *iph = (const struct iphdr *)(f + 14);
	unsigned ihl, ip_len;
	if (cap < 14)
		return 1;
	if (f[12] != 0x08 || f[13] != 0x00)
		return 0;
	if (cap < 34)
		return 1;
	ihl = iph->ihl;
	ip_len = ntohs(iph->tot_len);
	return 14 + ihl * 4 > cap || 14 + ip_len > cap || (iph->protocol == 6 && 14 + ihl * 4 + 20 > cap);
}

int main(int argc, char **argv)
{
	FILE *in;
	char magic[4];
	uint32_t ver, n, i, nlocal = 0, local_ip[16], num_msp, num_esp;
	uint64_t fb;
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
	mosrx_gpu_module_cfg cfg;
	mosrx_gpu_module_stats st;
	mosrx_source *src;
	uint64_t frames_seen = 0, compared = 0, skipped = 0, verdict_diff = 0, rss_checked = 0, rss_diff = 0;
	uint64_t fwd_mos = 0, fwd_diff = 0;
	uint64_t batches = 0, census[MOSRX_R_COUNT], neg = 0, bytes = 0;
	int64_t first_bad = -1;

	signal(SIGSEGV, on_segv);
	if (argc < 3 || argc > 5) {
		fprintf(stderr, "usage: %s trace.in batch [period [group]]\n", argv[0]);
		return 2;
	}
	in = fopen(argv[1], "rb");
	if (!in || rd(in, magic, 4) || memcmp(magic, "MRXT", 4) || rd(in, &ver, 4) || (ver != 1 && ver != 2) ||
	    rd(in, &n, 4) || rd(in, &fb, 8) || rd(in, &num_msp, 4) || rd(in, &num_esp, 4) ||
	    rd(in, &forward, 4) || rd(in, &nq, 4) || rd(in, &qmode, 4) ||
	    (ver == 2 && (rd(in, &nlocal, 4) || nlocal > 16 || rd(in, local_ip, sizeof(local_ip))))) {
		fprintf(stderr, "bad trace header\n");
		return 2;
	}
	if ((forward != 0 && forward != 1) || nq < 1) {
		fprintf(stderr, "forward must be 0 or 1 and num_queues >= 1\n");
		return 2;
	}
	off = malloc((size_t)n * 4 + 4);
	len = malloc((size_t)n * 2 + 2);
	frames = calloc(fb + 64, 1);
	if (!off || !len || !frames || rd(in, off, (size_t)n * 4) || rd(in, len, (size_t)n * 2) || rd(in, frames, fb)) {
		fprintf(stderr, "short trace\n");
		return 2;
	}
	fclose(in);
	g_qmode = qmode;
	memset(census, 0, sizeof(census));

	/* mOS's stack state (core.c:1079-1110 reduced, as ref_harness.c) */
	nd.num = (int)nlocal;       /* exactly ref_harness.c's table (ARP/ICMP walk it) */
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
	tctx.mtcp_manager = &m;     /* the backend reads num_msp / num_esp through it */
	TAILQ_INIT(&m.monitors);
	m.num_msp = num_msp;
	m.num_esp = num_esp;
	m.tcp_flow_table = CreateHashtable();
	m.iom = &null_iom;          /* nothing is sent: forward 0, empty route table */
	m.ctx = &tctx;
	InitLogThreadContext(&lg, 0);
	m.logger = &lg;
	m.log_fp = fopen("/dev/null", "w");
	if (getenv("MOSREF_LISTENER")) {   /* an end-host socket listening on that port (as ref_harness.c) */
		static struct tcp_listener lst;
		static struct socket_map lsock;
		lsock.socktype = MOS_SOCK_STREAM_LISTEN;
		lsock.saddr.sin_family = AF_INET;
		lsock.saddr.sin_addr.s_addr = INADDR_ANY;
		lsock.saddr.sin_port = htons((uint16_t)atoi(getenv("MOSREF_LISTENER")));
		lst.socket = &lsock;
		m.listener = &lst;
	}

	/* the backend, registered and loaded as core.c:1725-1736 does */
	src = mosrx_source_mem(frames, off, len, n, 1);
	if (!src)
		return 2;
	mosrx_gpu_module_cfg_default(&cfg);
	cfg.num_ifs = 1;
	cfg.src[0] = src;
	cfg.batch = (uint32_t)atoi(argv[2]);
	if (argc == 5)
		cfg.group = (uint32_t)atoi(argv[4]);
	cfg.params.num_msp = num_msp;
	cfg.params.num_esp = num_esp;
	cfg.params.num_queues = nq;
	cfg.params.queue_mode = qmode;
	if (mosrx_gpu_module_configure(&cfg))
		return 2;
	g_stage = "load_module_upper_half";
	current_iomodule_func = &gpu_module_func;
	current_iomodule_func->load_module_upper_half();    /* forward and netdev addresses from g_config */
	if (num_queues != nq) {
		fprintf(stderr, "load_module_upper_half left num_queues %d\n", num_queues);
		return 1;
	}
	g_stage = "init_handle";
	mosrx_gpu_module_bind(&tctx, 0);
	current_iomodule_func->init_handle(&tctx);

	/* RunMainLoop's rx section, core.c:897-909, with the GPU verdicts beside it */
	for (;;) {
		const mosrx_result *res = NULL;
		int32_t cnt;
		g_stage = "recv_pkts";
		cnt = current_iomodule_func->recv_pkts(&tctx, 0);
		int32_t k;
		if (cnt <= 0)
			break;
		batches++;
		if (current_iomodule_func->dev_ioctl(&tctx, 0, MOSRX_PKT_RX_RESULTS, &res) || !res)
			return 1;
		for (k = 0; k < cnt; k++, frames_seen++) {
			uint16_t l = 0;
			uint8_t *pkt = current_iomodule_func->get_rptr(&tctx, 0, k, &l);
			if (!pkt)
				return 1;
			if (res[k].reason < MOSRX_R_COUNT)
				census[res[k].reason]++;
			neg += res[k].verdict < 0;
			bytes += (uint64_t)l + 24;
			if (k < 127) {              /* the existing per-packet hook, int8 pktidx (io_module.h:81-84) */
				RssInfo ri = {(int8_t)k, 0};
				if (current_iomodule_func->dev_ioctl(&tctx, 0, PKT_RX_RSS, &ri) == 0 && res[k].payload_off) {
					const struct iphdr *iph = (const struct iphdr *)(pkt + 14);
					const struct tcphdr *th = (const struct tcphdr *)((const uint8_t *)iph + iph->ihl * 4);
					rss_checked++;
					rss_diff += ri.hash_value != GetRSSHash(ntohl(iph->saddr), ntohl(iph->daddr), ntohs(th->source),
					                                        ntohs(th->dest));
				}
			}
			if (past_capture(pkt, l)) {
				skipped++;
				continue;
			}
			compared++;
			g_stage = "ProcessPacket";
			g_fwd = 0;
			if ((int)res[k].verdict != ProcessPacket(&m, 0, k, 0, pkt, (int)l)) {
				verdict_diff++;
				if (first_bad < 0)
					first_bad = (int64_t)frames_seen;
			}
			fwd_mos += g_fwd > 0;
			if ((g_fwd > 0) != (mosrx_mos_forwards(&res[k], forward, m.num_msp, m.listener != NULL) != 0)) {
				fwd_diff++;
				if (first_bad < 0)
					first_bad = (int64_t)frames_seen;
			}
		}
		if (argc >= 4 && atoi(argv[3]) > 0 && batches % (uint64_t)atoi(argv[3]) == 0)
			m.num_msp = m.num_msp ? 0 : (num_msp ? num_msp : 1);   /* a monitor socket comes or goes */
	}
	g_stage = "destroy_handle";
	mosrx_gpu_module_stats_of(&tctx, &st);
	current_iomodule_func->destroy_handle(&tctx);
	mosrx_source_close(src);
	{
		/* mOS's NETSTAT over the compared frames vs the GPU census over all of them:
		 * equal when nothing was passed over */
		const int nstat_ok = skipped || (m.nstat.rx_packets[0] == frames_seen && m.nstat.rx_errors[0] == neg &&
		                                 m.nstat.rx_bytes[0] == bytes);
		printf("{\"frames\": %llu, \"batches\": %llu, \"compared\": %llu, \"skipped\": %llu, \"verdict_diff\": %llu, "
		       "\"first_bad\": %lld, \"rss_checked\": %llu, \"rss_diff\": %llu, \"num_queues\": %d, "
		       "\"nstat_rx_packets\": %llu, \"nstat_rx_errors\": %llu, \"nstat_ok\": %d, \"tcp_ok\": %llu, "
		       "\"reclassified\": %llu, \"forwarded_by_mos\": %llu, \"forward_diff\": %llu}\n",
		       (unsigned long long)frames_seen, (unsigned long long)batches, (unsigned long long)compared,
		       (unsigned long long)skipped, (unsigned long long)verdict_diff, (long long)first_bad,
		       (unsigned long long)rss_checked, (unsigned long long)rss_diff, num_queues,
		       (unsigned long long)m.nstat.rx_packets[0], (unsigned long long)m.nstat.rx_errors[0], nstat_ok,
		       (unsigned long long)census[MOSRX_R_TCP_OK], (unsigned long long)st.rx_reclassified,
		       (unsigned long long)fwd_mos, (unsigned long long)fwd_diff);
		return (frames_seen == n && !verdict_diff && !rss_diff && !fwd_diff && nstat_ok) ? 0 : 1;
	}
}
