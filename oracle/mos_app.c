/*
 * mos_app.c — TEST INFRASTRUCTURE ONLY (tests/test_mos_consumer.py).
 *
 * mOS itself, running: mtcp_init from a mos.conf, one mTCP thread
 * (mtcp_create_context -> MTCPRunThread -> RunMainLoop, core.c:1282-1349,
 * 851-1047), monitor sockets with callbacks and BPF filters, an optional
 * end-host listener -- with gpu_module_func as its I/O module (set before
 * mtcp_init: core.c is compiled without an ENABLE_* backend, so
 * core.c:1725-1733 leaves the choice alone, exactly what the ENABLE_GPU
 * branch of INTEGRATION.md §2 does).  The frames of a trace come in through
 * the backend from an in-memory source; everything mOS sends (forwarded
 * frames, RSTs, ICMP replies) goes out through the backend's TX into a pcap
 * dump.
 *
 * RunMainLoop's per-frame call (core.c:906) is routed, at link time
 * (-Wl,--wrap=ProcessPacket), to
 *   mode "pp":  mOS's own ProcessPacket (eth_in.c:27-87), checks on the CPU;
 *   mode "gpu": mosrx_mos_process_packet (csrc/mos_rx.c), the checks' outcome
 *               taken from the GPU records.
 * Everything observable is written out for the test to compare between the
 * two modes: each frame's return value, NETSTAT, every callback with the
 * packet it saw (mtcp_getlastpkt), the streams in the flow table after the
 * last frame, and the TX dump.  Per-frame CPU time of the rx loop is timed
 * per batch (index 0 .. n-1 of RunMainLoop's loop).
 *
 * Usage: mos_app <mode> <mos.conf> <trace.mrxt> <outdir>
 *   env MOSAPP_MONITORS=k        stream monitor sockets (default 1)
 *   env MOSAPP_RAW="bpf expr"    a raw monitor socket with this filter
 *   env MOSAPP_RAW_NOFILTER=1    a raw monitor socket without a filter
 *   env MOSAPP_SYN="bpf expr"    stream SYN filter of the first stream monitor
 *   env MOSAPP_ORPHAN="bpf expr" its orphan filter
 *   env MOSAPP_LISTEN=port       an end-host socket listening on that port
 *   env MOSAPP_BATCH=n           frames per recv_pkts (default 4096)
 *   env MOSAPP_GROUP=g           batches per launch (default 0 = auto)
 *   env MOSAPP_FLOWHASH=0        no flow-table hashes from the GPU (the consumer hashes on the CPU)
 *   env MOSAPP_LATE_RAW_AT=k     create the raw monitor (MOSAPP_RAW's filter) just before
 *                                frame k, on the mTCP thread (a filter bound mid-batch)
 *   env MOSAPP_LATE_MON_AT=k     create one more stream monitor just before frame k (the
 *                                checksum gate of ip_in.c:67 turning on mid-batch when
 *                                MOSAPP_MONITORS=0)
 *   env MOSAPP_LOOPS=l           replay the trace l times (timing runs)
 *   env MOSAPP_QUIET=1           no callback log (timing runs)
 *   env MOSAPP_NO_TX=1           no TX dump: what mOS sends is dropped at the source (counted as
 *                                TX errors), so timing runs do not time pcap writes
 *   env MOSAPP_REOPEN_RAW_AT=k   just before frame k, the raw monitor's program is replaced by
 *                                MOSAPP_RAW2's (same length) at the same address: what a freed
 *                                program (FreeMonListener, socket.c:33-36) reallocated for the
 *                                next monitor's filter looks like.  (mOS's mtcp_close cannot
 *                                close a monitor socket -- it looks the id up in smap, monitors
 *                                live in msmap -- and the allocator need not hand the address
 *                                back, so the harness writes the new program in place.)
 *   env MOSAPP_FAIL_RECLASSIFY=k the k-th MOSRX_PKT_RX_RECLASSIFY request fails (a GPU error
 *                                in the middle of a batch: the consumer drops the rest of it)
 * The per-frame time is reported as measured and without the time spent in
 * get_wptr (which flushes the TX buffer to the source every tx_batch frames).
 */
#define _GNU_SOURCE
#include <arpa/inet.h>
#include <errno.h>
#include <execinfo.h>
#include <pthread.h>
#include <signal.h>
#include <stdatomic.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/time.h>
#include <time.h>
#include <unistd.h>

#include "mtcp_api.h"
#include "mos_api.h"
#include "mtcp.h"
#include "config.h"
#include "fhash.h"
#include "tcp_stream.h"
#include "io_module.h"
#include "mosrx_io_module.h"
#include "mosrx_mos_rx.h"
#include "socket.h"
#include "sfbpf.h"

int __real_ProcessPacket(mtcp_manager_t mtcp, const int ifidx, const int index, uint32_t cur_ts,
                         unsigned char *pkt_data, int len);
extern mtcp_manager_t g_mtcp[];

static int g_mode_gpu;
static uint64_t g_total;                 /* frames the run will process */
static _Atomic uint64_t g_done;          /* frames processed so far */
static int8_t *g_ret;
static uint32_t g_batch_n;               /* frames of the batch being walked */
static struct timespec g_t0;
static double g_rx_ns;                   /* CPU time of the per-frame loop, summed per batch */
static uint64_t g_rx_frames;
static FILE *g_cb;
static int g_quiet;
static int g_frozen_clock;

/* MOSAPP_FROZEN_CLOCK: the frames mOS builds itself come out the same in both
 * runs, so they can be compared byte for byte: mOS's clock (RunMainLoop's
 * gettimeofday, core.c:887) stands still -- the same TCP timestamp option, and
 * no timer fires -- and the initial sequence numbers of its streams
 * (posix_seq_rand, tcp_stream.c:526) start from a fixed seed instead of the
 * mTCP thread's pthread_self (core.c:1085), which ASLR moves from run to run. */
void __real_posix_seq_srand(unsigned seed);
void __wrap_posix_seq_srand(unsigned seed)
{
	__real_posix_seq_srand(g_frozen_clock ? 1u : seed);
}
int __real_gettimeofday(struct timeval *tv, void *tz);
int __wrap_gettimeofday(struct timeval *tv, void *tz)
{
	if (g_frozen_clock) {
		tv->tv_sec = 1700000000;
		tv->tv_usec = 0;
		return 0;
	}
	return __real_gettimeofday(tv, tz);
}
static unsigned long g_arp_sent;         /* ARP frames in the TX dump */
static char g_snap[1 << 20];             /* flow table + NETSTAT after the last frame */
static size_t g_snap_len;
static mctx_t g_mctx;
static _Atomic int g_go;                  /* the application's sockets are set up */
static io_module_func g_gated;           /* gpu_module_func, receiving nothing before g_go */

static uint64_t g_late_raw, g_late_mon, g_reopen_raw;
static int g_raw_sock = -1;
static int g_reopen_same_addr;           /* the rebound program took the freed one's address */
static int raw_monitor(void);
static int raw_monitor_filter(const char *expr);
static void die(const char *m);
static int stream_monitor(int with_filters);
static int g_in_window;                  /* inside a batch's timed per-frame loop */
static double g_tx_ns;                   /* of the timed loop, the time spent in get_wptr (TX flushes) */
static uint64_t g_fail_reclassify, g_reclassify_calls;

/* get_wptr timed inside the rx window: a full TX buffer is flushed to the
 * source there (the pcap dump), which is the harness's sink, not mOS's work */
static uint8_t *timed_get_wptr(struct mtcp_thread_context *ctx, int ifidx, uint16_t len)
{
	struct timespec a, b;
	uint8_t *r;
	if (!g_in_window)
		return gpu_module_func.get_wptr(ctx, ifidx, len);
	clock_gettime(CLOCK_MONOTONIC, &a);
	r = gpu_module_func.get_wptr(ctx, ifidx, len);
	clock_gettime(CLOCK_MONOTONIC, &b);
	g_tx_ns += (b.tv_sec - a.tv_sec) * 1e9 + (b.tv_nsec - a.tv_nsec);
	return r;
}

/* a GPU error on the k-th reclassification (MOSAPP_FAIL_RECLASSIFY) */
static int32_t failing_dev_ioctl(struct mtcp_thread_context *ctx, int nif, int cmd, void *argp)
{
	if (cmd == MOSRX_PKT_RX_RECLASSIFY && ++g_reclassify_calls == g_fail_reclassify)
		return -1;
	return gpu_module_func.dev_ioctl(ctx, nif, cmd, argp);
}

static int32_t gated_recv_pkts(struct mtcp_thread_context *ctx, int ifidx)
{
	return atomic_load(&g_go) ? gpu_module_func.recv_pkts(ctx, ifidx) : 0;
}

/* the backend's TX counters after each send_pkts (the context's stats go with
 * destroy_handle) */
static mosrx_gpu_module_stats g_tx_stats;
static int32_t counted_send_pkts(struct mtcp_thread_context *ctx, int nif)
{
	const int32_t r = gpu_module_func.send_pkts(ctx, nif);
	mosrx_gpu_module_stats_of(ctx, &g_tx_stats);
	return r;
}

static double ns_between(const struct timespec *a, const struct timespec *b)
{
	return (b->tv_sec - a->tv_sec) * 1e9 + (b->tv_nsec - a->tv_nsec);
}

int __wrap_GetNumCPUs(void)   /* core.c sizes per-cpu arrays of MAX_CPUS by it (core.c:1711-1716) */
{
	long n = sysconf(_SC_NPROCESSORS_ONLN);
	return n < MAX_CPUS ? (int)n : MAX_CPUS;
}

static int stream_cmp(const void *a, const void *b)
{
	return memcmp(a, b, 16);
}

/* The flow table as the test compares it: each stream's tuple, type, state,
 * side and whether it has a pair, sorted; then NETSTAT. */
static void snapshot(mtcp_manager_t mtcp)
{
	struct hashtable *ht = mtcp->tcp_flow_table;
	uint8_t (*rows)[16] = calloc(200000, 16);
	size_t nrow = 0, i;
	int b;
	for (b = 0; rows && b < NUM_BINS; b++) {
		tcp_stream *w;
		TAILQ_FOREACH(w, &ht->ht_table[b], rcvvar->he_link) {
			if (nrow == 200000)
				break;
			memcpy(rows[nrow], &w->saddr, 4);
			memcpy(rows[nrow] + 4, &w->daddr, 4);
			memcpy(rows[nrow] + 8, &w->sport, 2);
			memcpy(rows[nrow] + 10, &w->dport, 2);
			rows[nrow][12] = (uint8_t)w->stream_type;
			rows[nrow][13] = (uint8_t)w->state;
			rows[nrow][14] = (uint8_t)w->side;
			rows[nrow][15] = w->pair_stream != NULL;
			nrow++;
		}
	}
	if (rows)
		qsort(rows, nrow, 16, stream_cmp);
	g_snap_len = (size_t)snprintf(g_snap, sizeof(g_snap), "streams %zu flow_cnt %u\n", nrow, mtcp->flow_cnt);
	for (i = 0; i < nrow && g_snap_len < sizeof(g_snap) - 64; i++) {
		int k;
		for (k = 0; k < 16; k++)
			g_snap_len += (size_t)snprintf(g_snap + g_snap_len, sizeof(g_snap) - g_snap_len, "%02x", rows[i][k]);
		g_snap[g_snap_len++] = '\n';
	}
	g_snap_len += (size_t)snprintf(g_snap + g_snap_len, sizeof(g_snap) - g_snap_len,
	                               "nstat rx_packets %lu rx_bytes %lu rx_errors %lu\n",
	                               (unsigned long)mtcp->nstat.rx_packets[0], (unsigned long)mtcp->nstat.rx_bytes[0],
	                               (unsigned long)mtcp->nstat.rx_errors[0]);
	free(rows);
}

/* core.c:906's call, routed to the mode's receive step. */
int __wrap_ProcessPacket(mtcp_manager_t mtcp, const int ifidx, const int index, uint32_t cur_ts,
                         unsigned char *pkt_data, int len)
{
	int ret;
	uint64_t k = atomic_load(&g_done);
	/* sockets that appear in the middle of a batch, at a fixed frame (on the
	 * mTCP thread, so both modes see them at the same point) */
	if (g_late_raw && k + 1 == g_late_raw)
		raw_monitor();
	if (g_late_mon && k + 1 == g_late_mon)
		stream_monitor(0);
	if (g_reopen_raw && k + 1 == g_reopen_raw && g_raw_sock >= 0) {
		struct sfbpf_program *fc = &mtcp->msmap[g_raw_sock].monitor_listener->raw_pkt_fcode, nf;
		memset(&nf, 0, sizeof(nf));
		if (SET_BPFFILTER(&nf, getenv("MOSAPP_RAW2")) < 0 || nf.bf_len != fc->bf_len)
			die("MOSAPP_RAW2: a filter of the same length");
		memcpy(fc->bf_insns, nf.bf_insns, nf.bf_len * sizeof(*nf.bf_insns));
		sfbpf_freecode(&nf);
		g_reopen_same_addr = 1;
	}
	if (index == 0) {
		mosrx_rx_state st;
		g_batch_n = mtcp->iom->dev_ioctl(mtcp->ctx, ifidx, MOSRX_PKT_RX_STATE, &st) ? 0 : st.n;
		g_in_window = 1;
		clock_gettime(CLOCK_MONOTONIC, &g_t0);
	}
	ret = g_mode_gpu ? mosrx_mos_process_packet(mtcp, ifidx, index, cur_ts, pkt_data, len)
	                 : __real_ProcessPacket(mtcp, ifidx, index, cur_ts, pkt_data, len);
	if ((uint32_t)index + 1 == g_batch_n) {
		struct timespec t1;
		clock_gettime(CLOCK_MONOTONIC, &t1);
		g_rx_ns += ns_between(&g_t0, &t1);
		g_rx_frames += g_batch_n;
		g_in_window = 0;
	}
	if (g_ret && k < g_total)
		g_ret[k] = (int8_t)ret;
	if (k + 1 == g_total)
		snapshot(mtcp);
	atomic_store(&g_done, k + 1);
	return ret;
}

/* Every callback with the packet it was raised for. */
static void on_event(mctx_t mctx, int sock, int side, event_t ev, filter_arg_t *arg)
{
	struct pkt_info p;
	(void)arg;
	if (g_quiet)
		return;
	memset(&p, 0, sizeof(p));
	if (mtcp_getlastpkt(mctx, sock, side, &p) != 0)
		memset(&p, 0, sizeof(p));
	fprintf(g_cb, "f %lu ev %lx sock %d side %d eth %u ip %u plen %u seq %u ack %u win %u off %lu\n",
	        (unsigned long)atomic_load(&g_done), (unsigned long)ev, sock, side, p.eth_len, p.ip_len, p.payloadlen,
	        p.seq, p.ack_seq, p.window, (unsigned long)p.offset);
}

static int rd(FILE *f, void *p, size_t n) { return fread(p, 1, n, f) == n ? 0 : -1; }

static void die(const char *m)
{
	fprintf(stderr, "mos_app: %s (errno %d)\n", m, errno);
	exit(2);
}

static int raw_monitor_filter(const char *expr)
{
	int s = mtcp_socket(g_mctx, AF_INET, MOS_SOCK_MONITOR_RAW, 0);
	if (s < 0)
		die("raw monitor socket");
	if (expr) {
		union monitor_filter ft = {.raw_pkt_filter = (char *)expr};
		if (mtcp_bind_monitor_filter(g_mctx, s, &ft))
			die("raw filter");
	}
	if (mtcp_register_callback(g_mctx, s, MOS_ON_PKT_IN, MOS_NULL, on_event))
		die("raw callback");
	return s;
}

static int raw_monitor(void)
{
	return g_raw_sock = raw_monitor_filter(getenv("MOSAPP_RAW"));
}

/* ARP frames (ethertype 0x0806) in a classic pcap file: mOS's ARP requests */
static unsigned long pcap_arp_frames(const char *path)
{
	FILE *f = fopen(path, "rb");
	unsigned char h[24], rec[16], eth[14];
	unsigned long n = 0;
	if (!f || fread(h, 1, 24, f) != 24) {
		if (f)
			fclose(f);
		return 0;
	}
	while (fread(rec, 1, 16, f) == 16) {
		uint32_t incl;
		memcpy(&incl, rec + 8, 4);
		if (incl >= 14 && fread(eth, 1, 14, f) == 14) {
			n += eth[12] == 0x08 && eth[13] == 0x06;
			incl -= 14;
		}
		if (fseek(f, incl, SEEK_CUR))
			break;
	}
	fclose(f);
	return n;
}

/* A MOS_SOCK_MONITOR_STREAM socket (num_msp++, socket.c:77-78) with every
 * stream event's callback; the first one takes MOSAPP_SYN / MOSAPP_ORPHAN. */
static int stream_monitor(int with_filters)
{
	int s = mtcp_socket(g_mctx, AF_INET, MOS_SOCK_MONITOR_STREAM, 0);
	if (s < 0)
		die("monitor socket");
	if (with_filters && (getenv("MOSAPP_SYN") || getenv("MOSAPP_ORPHAN"))) {
		union monitor_filter ft;
		memset(&ft, 0, sizeof(ft));
		ft.stream_syn_filter = getenv("MOSAPP_SYN");
		ft.stream_orphan_filter = getenv("MOSAPP_ORPHAN");
		if (mtcp_bind_monitor_filter(g_mctx, s, &ft))
			die("stream filters");
	}
	if (mtcp_register_callback(g_mctx, s, MOS_ON_PKT_IN, MOS_HK_SND, on_event) ||
	    mtcp_register_callback(g_mctx, s, MOS_ON_PKT_IN, MOS_HK_RCV, on_event) ||
	    mtcp_register_callback(g_mctx, s, MOS_ON_CONN_START, MOS_HK_SND, on_event) ||
	    mtcp_register_callback(g_mctx, s, MOS_ON_TCP_STATE_CHANGE, MOS_HK_RCV, on_event) ||
	    mtcp_register_callback(g_mctx, s, MOS_ON_CONN_END, MOS_HK_RCV, on_event) ||
	    mtcp_register_callback(g_mctx, s, MOS_ON_ORPHAN, MOS_NULL, on_event))
		die("stream callbacks");
	return s;
}

/* An abort (a fortified copy, an assert in mOS) prints where it came from:
 * the harness links with -rdynamic, so the frames have names. */
static void on_abort(int sig)
{
	void *fr[48];
	int n = backtrace(fr, 48);
	(void)sig;
	backtrace_symbols_fd(fr, n, 2);
	signal(SIGABRT, SIG_DFL);
	abort();
}

int main(int argc, char **argv)
{
	FILE *in;
	char magic[4], path[4096];
	uint32_t ver, n, nlocal = 0, local_ip[16], num_msp, num_esp, i;
	uint64_t fb;
	int32_t forward, nq, qmode;
	uint32_t *off;
	uint16_t *len;
	uint8_t *frames;
	mosrx_source *src;
	mosrx_gpu_module_cfg cfg;
	struct mtcp_conf mcfg;
	int monitors = getenv("MOSAPP_MONITORS") ? atoi(getenv("MOSAPP_MONITORS")) : 1;
	uint32_t loops = getenv("MOSAPP_LOOPS") ? (uint32_t)atoi(getenv("MOSAPP_LOOPS")) : 1;
	uint64_t late_raw = getenv("MOSAPP_LATE_RAW_AT") ? strtoull(getenv("MOSAPP_LATE_RAW_AT"), NULL, 10) : 0;
	int mon0 = -1, m;
	FILE *f;
	signal(SIGABRT, on_abort);

	if (argc != 5 || (strcmp(argv[1], "pp") && strcmp(argv[1], "gpu"))) {
		fprintf(stderr, "usage: %s pp|gpu mos.conf trace.mrxt outdir\n", argv[0]);
		return 2;
	}
	g_mode_gpu = !strcmp(argv[1], "gpu");
	g_quiet = getenv("MOSAPP_QUIET") != NULL;
	g_frozen_clock = getenv("MOSAPP_FROZEN_CLOCK") != NULL;
	in = fopen(argv[3], "rb");
	if (!in || rd(in, magic, 4) || memcmp(magic, "MRXT", 4) || rd(in, &ver, 4) || (ver != 1 && ver != 2) ||
	    rd(in, &n, 4) || rd(in, &fb, 8) || rd(in, &num_msp, 4) || rd(in, &num_esp, 4) ||
	    rd(in, &forward, 4) || rd(in, &nq, 4) || rd(in, &qmode, 4) ||
	    (ver == 2 && (rd(in, &nlocal, 4) || nlocal > 16 || rd(in, local_ip, sizeof(local_ip)))))
		die("bad trace header");
	off = malloc((size_t)n * 4 + 4);
	len = malloc((size_t)n * 2 + 2);
	frames = calloc(fb + 64, 1);
	if (!off || !len || !frames || rd(in, off, (size_t)n * 4) || rd(in, len, (size_t)n * 2) || rd(in, frames, fb))
		die("short trace");
	fclose(in);
	g_total = (uint64_t)n * loops;
	g_ret = calloc(g_total, 1);
	snprintf(path, sizeof(path), "%s/callbacks.txt", argv[4]);
	g_cb = fopen(path, "w");
	if (!g_cb)
		die("callbacks file");

	/* the backend: frames from memory, TX into a pcap dump, mOS's I/O module */
	src = mosrx_source_mem(frames, off, len, n, loops);
	if (!src)
		die("source");
	mosrx_source_mem_set_mode(src, 1);   /* copied in runs: frames stay writable for mOS (forward rewrites) */
	snprintf(path, sizeof(path), "%s/tx.pcap", argv[4]);
	if (!getenv("MOSAPP_NO_TX") && mosrx_source_tx_pcap(src, path))
		die("tx dump");
	mosrx_gpu_module_cfg_default(&cfg);
	cfg.num_ifs = 1;
	strncpy(cfg.if_names[0], "lo", IFNAMSIZ - 1);
	cfg.src[0] = src;
	cfg.batch = getenv("MOSAPP_BATCH") ? (uint32_t)atoi(getenv("MOSAPP_BATCH")) : 4096;
	cfg.group = getenv("MOSAPP_GROUP") ? (uint32_t)atoi(getenv("MOSAPP_GROUP")) : MOSRX_GROUP_AUTO;
	cfg.flowhash = getenv("MOSAPP_FLOWHASH") ? atoi(getenv("MOSAPP_FLOWHASH")) : 1;   /* FindStream's bucket too */
	/* mOS's TX checksums on the GPU (dev_ioctl PKT_TX_*_CSUM, as with DPDK's offload) */
	cfg.tx_csum = getenv("MOSAPP_TX_CSUM") ? atoi(getenv("MOSAPP_TX_CSUM")) : 0;
	/* 8-byte records (what an unconfigured mOS build of the module uses), or 16-byte ones */
	cfg.compact = getenv("MOSAPP_COMPACT") ? atoi(getenv("MOSAPP_COMPACT")) : 1;
	/* the harness's traces are small: 64 MiB auto groups (pinned twice) instead of the default */
	cfg.group_bytes = getenv("MOSAPP_GROUP_BYTES") ? strtoull(getenv("MOSAPP_GROUP_BYTES"), NULL, 10) : 64ull << 20;
	cfg.params.num_queues = nq;
	cfg.params.queue_mode = qmode;
	cfg.params.num_msp = 0;                       /* followed from mOS's manager (mos_state) */
	cfg.params.num_esp = 0;
	if (mosrx_gpu_module_configure(&cfg))
		die("configure");
	/* the ENABLE_GPU branch of core.c:1725-1733; frames are held back until the
	 * application's sockets exist, so both modes see the same stack state */
	g_gated = gpu_module_func;
	g_gated.recv_pkts = gated_recv_pkts;
	g_gated.send_pkts = counted_send_pkts;
	g_gated.get_wptr = timed_get_wptr;
	g_fail_reclassify = getenv("MOSAPP_FAIL_RECLASSIFY") ? strtoull(getenv("MOSAPP_FAIL_RECLASSIFY"), NULL, 10) : 0;
	if (g_fail_reclassify)
		g_gated.dev_ioctl = failing_dev_ioctl;
	current_iomodule_func = &g_gated;

	if (mtcp_init(argv[2]))
		die("mtcp_init");
	mtcp_getconf(&mcfg);
	mcfg.num_cores = 1;
	mtcp_setconf(&mcfg);
	g_mctx = mtcp_create_context(0);
	if (!g_mctx)
		die("mtcp_create_context");

	/* the application's sockets (simple_firewall.c:383-395 and friends) */
	for (m = 0; m < monitors; m++) {
		int s = stream_monitor(m == 0);
		if (m == 0)
			mon0 = s;
	}
	if ((getenv("MOSAPP_RAW") || getenv("MOSAPP_RAW_NOFILTER")) && !late_raw)
		raw_monitor();
	g_late_raw = late_raw;
	g_reopen_raw = getenv("MOSAPP_REOPEN_RAW_AT") ? strtoull(getenv("MOSAPP_REOPEN_RAW_AT"), NULL, 10) : 0;
	g_late_mon = getenv("MOSAPP_LATE_MON_AT") ? strtoull(getenv("MOSAPP_LATE_MON_AT"), NULL, 10) : 0;
	if (getenv("MOSAPP_LISTEN")) {
		struct sockaddr_in a;
		int s = mtcp_socket(g_mctx, AF_INET, SOCK_STREAM, 0);   /* num_esp++ (socket.c:96) */
		memset(&a, 0, sizeof(a));
		a.sin_family = AF_INET;
		a.sin_addr.s_addr = INADDR_ANY;
		a.sin_port = htons((uint16_t)atoi(getenv("MOSAPP_LISTEN")));
		if (s < 0)
			die("listener socket");
		if (mtcp_bind(g_mctx, s, (struct sockaddr *)&a, sizeof(a)))
			die("listener bind");
		if (mtcp_listen(g_mctx, s, 128))
			die("listener listen");
	}
	atomic_store(&g_go, 1);
	(void)mon0;
	(void)num_msp;
	(void)num_esp;
	(void)forward;
	(void)nlocal;

	/* the frames go through; a late raw monitor appears mid-trace (the app
	 * thread creating a socket while the mTCP thread receives, as
	 * simple_firewall's threads do) */
	while (atomic_load(&g_done) < g_total)
		usleep(200);
	usleep(100000);                       /* the last round's send_pkts */
	mtcp_destroy_context(g_mctx);
	mosrx_source_tx_flush(src);
	mosrx_source_tx_pcap(src, NULL);
	snprintf(path, sizeof(path), "%s/tx.pcap", argv[4]);
	{
		const unsigned long arp = getenv("MOSAPP_NO_TX") ? 0 : pcap_arp_frames(path);
		g_arp_sent = arp;
	}

	snprintf(path, sizeof(path), "%s/returns.bin", argv[4]);
	f = fopen(path, "wb");
	if (!f || fwrite(g_ret, 1, g_total, f) != g_total)
		die("returns");
	fclose(f);
	snprintf(path, sizeof(path), "%s/state.txt", argv[4]);
	f = fopen(path, "w");
	if (!f || fwrite(g_snap, 1, g_snap_len, f) != g_snap_len)
		die("state");
	fclose(f);
	fclose(g_cb);
	{
		mosrx_mos_rx_stats cs;
		mosrx_mos_rx_stats_of(0, &cs);
		printf("{\"mode\": \"%s\", \"frames\": %lu, \"rx_frames_timed\": %lu, \"rx_ns_per_frame\": %.2f, "
		       "\"rx_ns_per_frame_excl_tx\": %.2f, "
		       "\"consumer_frames\": %lu, \"stream_step\": %lu, \"gpu_flow_hash\": %lu, \"reclassified\": %lu, "
		       "\"filter_installs\": %lu, \"max_filter_sync_ns\": %lu, \"gpu_errors\": %lu, \"gpu_dropped\": %lu, "
		       "\"filters_gpu\": %lu, \"filters_cpu\": %lu, \"tx_packets\": %lu, \"tx_csum_offloaded\": %lu, "
		       "\"tx_errors\": %lu, \"arp_sent\": %lu, \"reopen_same_addr\": %d, \"batches_c8\": %lu}\n",
		       argv[1], (unsigned long)g_total, (unsigned long)g_rx_frames,
		       g_rx_frames ? g_rx_ns / (double)g_rx_frames : 0.0,
		       g_rx_frames ? (g_rx_ns - g_tx_ns) / (double)g_rx_frames : 0.0, (unsigned long)cs.frames,
		       (unsigned long)cs.stream_step, (unsigned long)cs.gpu_flow_hash, (unsigned long)cs.reclassified,
		       (unsigned long)cs.filter_installs, (unsigned long)cs.max_filter_sync_ns, (unsigned long)cs.gpu_errors,
		       (unsigned long)cs.gpu_dropped,
		       (unsigned long)cs.filters_gpu, (unsigned long)cs.filters_cpu, (unsigned long)g_tx_stats.tx_packets,
		       (unsigned long)g_tx_stats.tx_csum_offloaded, (unsigned long)g_tx_stats.tx_errors, g_arp_sent,
		       g_reopen_same_addr, (unsigned long)cs.batches_c8);
	}
	mosrx_source_close(src);
	return 0;
}
