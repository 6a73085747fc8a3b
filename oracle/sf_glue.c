/*
 * sf_glue.c — TEST INFRASTRUCTURE ONLY (tests/test_simple_firewall.py).
 *
 * Linked, with -Wl,--wrap, into mOS's own samples/simple_firewall compiled
 * unmodified (oracle/Makefile _ref/simple_firewall*), so that BASELINE config
 * #1 runs through the reference's application itself: its mtcp_init, its
 * monitor socket and SYN event, its FWRLookup / MOS_DROP / MOS_STOP_MON
 * actions (simple_firewall.c:332-410) and its rule table printout, over the
 * ENABLE_GPU build of mOS (core.c through core_enable_gpu.py) with
 * gpu_module_func replaying a pcap file (MOSRX_PCAP_<netdev>).  The glue only
 * observes and routes; it changes nothing the application does:
 *
 *   - RunMainLoop's per-frame call (core.c:906) goes to mOS's ProcessPacket
 *     (SFGLUE_MODE=pp) or to the consumer of the GPU records,
 *     mosrx_mos_process_packet (SFGLUE_MODE=gpu); every return is recorded;
 *   - receiving starts once the application registered its callback (the
 *     sample's last socket step, simple_firewall.c:392-396), so both modes
 *     see the same stack state from the first frame;
 *   - after the last of SFGLUE_FRAMES frames and SFGLUE_LINGER_MS more (the
 *     sample's 1 s table timer fires at least once), the mTCP thread is told to
 *     exit as mOS's own SIGINT path does (ctx->exit, core.c:103-119), so the
 *     sample's mtcp_app_join returns and it tears down as it would;
 *   - at exit: SFGLUE_OUT/returns.bin (one int8 per frame), state.txt (NETSTAT,
 *     flow_cnt after the last frame) and result.json (the rx loop's per-frame
 *     CPU time, timed per batch as oracle/mos_app.c does).
 */
#define _GNU_SOURCE
#include <pthread.h>
#include <stdatomic.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <unistd.h>

#include "mtcp_api.h"
#include "mos_api.h"
#include "mtcp.h"
#include "io_module.h"
#include "mosrx_io_module.h"
#include "mosrx_mos_rx.h"

int __real_ProcessPacket(mtcp_manager_t mtcp, const int ifidx, const int index, uint32_t cur_ts,
                         unsigned char *pkt_data, int len);
int __real_mtcp_register_callback(mctx_t mctx, int sockid, event_t event, int hook_point, callback_t callback);
extern struct mtcp_thread_context *g_pctx[];

static int g_gpu;
static uint64_t g_total;
static _Atomic uint64_t g_done;
static _Atomic int g_go;
static int8_t *g_ret;
static uint32_t g_batch_n;
static struct timespec g_t0, g_first, g_last;
static double g_rx_ns;
static uint64_t g_rx_frames;
static char g_state[256];
static int32_t (*g_recv)(struct mtcp_thread_context *ctx, int ifidx);

static double ns_between(const struct timespec *a, const struct timespec *b)
{
	return (b->tv_sec - a->tv_sec) * 1e9 + (b->tv_nsec - a->tv_nsec);
}

int __wrap_GetNumCPUs(void)   /* core.c sizes per-cpu arrays of MAX_CPUS by it (core.c:1711-1716) */
{
	long n = sysconf(_SC_NPROCESSORS_ONLN);
	return n < MAX_CPUS ? (int)n : MAX_CPUS;
}

static int32_t gated_recv_pkts(struct mtcp_thread_context *ctx, int ifidx)
{
	return atomic_load(&g_go) ? g_recv(ctx, ifidx) : 0;
}

int __wrap_mtcp_register_callback(mctx_t mctx, int sockid, event_t event, int hook_point, callback_t callback)
{
	const int r = __real_mtcp_register_callback(mctx, sockid, event, hook_point, callback);
	atomic_store(&g_go, 1);
	return r;
}

int __wrap_ProcessPacket(mtcp_manager_t mtcp, const int ifidx, const int index, uint32_t cur_ts,
                         unsigned char *pkt_data, int len)
{
	const uint64_t k = atomic_load(&g_done);
	int ret;
	if (index == 0) {
		mosrx_rx_state st;
		g_batch_n = mtcp->iom->dev_ioctl(mtcp->ctx, ifidx, MOSRX_PKT_RX_STATE, &st) ? 0 : st.n;
		clock_gettime(CLOCK_MONOTONIC, &g_t0);
		if (k == 0)
			g_first = g_t0;
	}
	ret = g_gpu ? mosrx_mos_process_packet(mtcp, ifidx, index, cur_ts, pkt_data, len)
	            : __real_ProcessPacket(mtcp, ifidx, index, cur_ts, pkt_data, len);
	if ((uint32_t)index + 1 == g_batch_n) {
		struct timespec t1;
		clock_gettime(CLOCK_MONOTONIC, &t1);
		g_rx_ns += ns_between(&g_t0, &t1);
		g_rx_frames += g_batch_n;
		g_last = t1;
	}
	if (k < g_total)
		g_ret[k] = (int8_t)ret;
	if (k + 1 == g_total)
		snprintf(g_state, sizeof(g_state), "nstat rx_packets %lu rx_bytes %lu rx_errors %lu flow_cnt %u\n",
		         (unsigned long)mtcp->nstat.rx_packets[0], (unsigned long)mtcp->nstat.rx_bytes[0],
		         (unsigned long)mtcp->nstat.rx_errors[0], mtcp->flow_cnt);
	atomic_store(&g_done, k + 1);
	return ret;
}

static void *watcher(void *arg)
{
	const char *l = getenv("SFGLUE_LINGER_MS");
	const long linger = l ? atol(l) : 1200;
	(void)arg;
	while (atomic_load(&g_done) < g_total)
		usleep(500);
	usleep((useconds_t)linger * 1000);
	if (g_pctx[0])
		g_pctx[0]->exit = 1;       /* as HandleSignal does for a running thread (core.c:103-119) */
	return NULL;
}

static void write_out(void)
{
	const char *dir = getenv("SFGLUE_OUT");
	char path[4096];
	FILE *f;
	mosrx_mos_rx_stats cs;
	if (!dir)
		return;
	snprintf(path, sizeof(path), "%s/returns.bin", dir);
	if ((f = fopen(path, "wb"))) {
		fwrite(g_ret, 1, g_total, f);
		fclose(f);
	}
	snprintf(path, sizeof(path), "%s/state.txt", dir);
	if ((f = fopen(path, "w"))) {
		fputs(g_state, f);
		fclose(f);
	}
	memset(&cs, 0, sizeof(cs));
	mosrx_mos_rx_stats_of(0, &cs);
	snprintf(path, sizeof(path), "%s/result.json", dir);
	if ((f = fopen(path, "w"))) {
		fprintf(f, "{\"mode\": \"%s\", \"frames\": %lu, \"done\": %lu, \"rx_frames_timed\": %lu, "
		        "\"rx_ns_per_frame\": %.2f, \"wall_first_to_last_s\": %.6f, \"consumer_frames\": %lu, "
		        "\"gpu_errors\": %lu}\n",
		        g_gpu ? "gpu" : "pp", (unsigned long)g_total, (unsigned long)atomic_load(&g_done),
		        (unsigned long)g_rx_frames, g_rx_frames ? g_rx_ns / (double)g_rx_frames : 0.0,
		        ns_between(&g_first, &g_last) * 1e-9, (unsigned long)cs.frames, (unsigned long)cs.gpu_errors);
		fclose(f);
	}
}

__attribute__((constructor)) static void sfglue_init(void)
{
	const char *m = getenv("SFGLUE_MODE"), *n = getenv("SFGLUE_FRAMES");
	pthread_t t;
	g_gpu = m && !strcmp(m, "gpu");
	g_total = n ? strtoull(n, NULL, 10) : 0;
	g_ret = calloc(g_total ? g_total : 1, 1);
	g_recv = gpu_module_func.recv_pkts;
	gpu_module_func.recv_pkts = gated_recv_pkts;
	atexit(write_out);
	if (g_total && !pthread_create(&t, NULL, watcher, NULL))
		pthread_detach(t);
}
