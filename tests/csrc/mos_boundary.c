/*
 * mos_boundary.c — TEST INFRASTRUCTURE ONLY (tests/test_boundary.py).
 *
 * Built twice by the test: once against mOS's own io_module.h / config.h
 * (-DMOSRX_HAVE_MOS_IO_MODULE -I<reference>/core/src/include) and linked with
 * csrc/gpu_module.c compiled the same way plus mOS's compiled core/src objects
 * (oracle/_ref/obj), and once standalone against include/mosrx_io_module.h.
 * Each build prints the layout of io_module_func and RssInfo; the mOS build
 * also loads the backend's upper half as mtcp_init would (core.c:1735) and
 * prints the globals it set.  The test compares the two layouts line by line.
 * With an interface name as argument the mOS build skips the configure call
 * and lets load_module_upper_half open that netdev itself.
 */
#include <stddef.h>
#include <stdio.h>
#include <string.h>

#include "mosrx_io_module.h"
#ifdef MOSRX_HAVE_MOS_IO_MODULE
#include <pthread.h>
#include <stdlib.h>
#include "config.h"
#include "mtcp.h"

/* --map mode: the module's calls into libmosrx are wrapped (-Wl,--wrap) so
 * init_handle runs without a GPU on a pretended device count; only the
 * device choice is observed. */
static int g_fake_ndev = 1;
int __wrap_mosrx_device_count(void) { return g_fake_ndev; }
int __wrap_mosrx_open(int device, const mosrx_params *p, mosrx_ctx **out)
{
	(void)p;
	if (device < 0 || device >= g_fake_ndev)
		return -19;
	*out = (mosrx_ctx *)calloc(1, 64);
	return *out ? 0 : -12;
}
void __wrap_mosrx_close(mosrx_ctx *c) { free(c); }
int __wrap_mosrx_host_alloc(mosrx_ctx *c, size_t bytes, void **p) { (void)c; *p = calloc(1, bytes); return *p ? 0 : -12; }
int __wrap_mosrx_host_free(mosrx_ctx *c, void *p) { (void)c; free(p); return 0; }
int __wrap_mosrx_set_counters(mosrx_ctx *c, int on) { (void)c; (void)on; return 0; }
int __wrap_mosrx_set_direct(mosrx_ctx *c, uint64_t b, uint32_t f) { (void)c; (void)b; (void)f; return 0; }
int __wrap_mosrx_classify_host_reserve(mosrx_ctx *c, uint64_t fb, uint32_t n) { (void)c; (void)fb; (void)n; return 0; }

static void *init_thread(void *arg)
{
	current_iomodule_func->init_handle((struct mtcp_thread_context *)arg);   /* core.c:1313 */
	return NULL;
}

/* mTCP threads created for cores in a scrambled order, each calling
 * init_handle concurrently (as MTCPRunThread does): print cpu -> device. */
static int map_mode(int ndev, int base, int ngpu)
{
	enum { NT = 12 };
	static const int cores[NT] = {5, 2, 11, 0, 7, 3, 9, 1, 10, 4, 8, 6};
	static struct mtcp_thread_context tc[NT];
	pthread_t th[NT];
	mosrx_gpu_module_cfg cfg;
	int i;
	g_fake_ndev = ndev;
	mosrx_gpu_module_cfg_default(&cfg);
	cfg.num_ifs = 1;
	cfg.batch = 64;
	cfg.gpu_base = base;
	cfg.ngpu = ngpu;
	if (mosrx_gpu_module_configure(&cfg))
		return 1;
	current_iomodule_func = &gpu_module_func;
	for (i = 0; i < NT; i++) {
		tc[i].cpu = cores[i];
		if (pthread_create(&th[i], NULL, init_thread, &tc[i]))
			return 1;
	}
	for (i = 0; i < NT; i++)
		pthread_join(th[i], NULL);
	for (i = 0; i < NT; i++) {
		mosrx_gpu_module_stats st;
		if (mosrx_gpu_module_stats_of(&tc[i], &st))
			return 1;
		printf("map %d %d %d\n", tc[i].cpu, st.cpu, st.device);
	}
	for (i = 0; i < NT; i++)
		current_iomodule_func->destroy_handle(&tc[i]);
	return 0;
}
#endif

#define OFF(m) printf("io_module_func.%s %zu\n", #m, offsetof(io_module_func, m))

int main(int argc, char **argv)
{
#ifdef MOSRX_HAVE_MOS_IO_MODULE
	if (argc == 5 && !strcmp(argv[1], "--map"))
		return map_mode(atoi(argv[2]), atoi(argv[3]), atoi(argv[4]));
#endif
	OFF(load_module_upper_half); OFF(load_module_lower_half); OFF(init_handle); OFF(link_devices);
	OFF(release_pkt); OFF(get_wptr); OFF(set_wptr); OFF(send_pkts); OFF(get_rptr); OFF(get_nif);
	OFF(recv_pkts); OFF(select); OFF(destroy_handle); OFF(dev_ioctl);
	printf("io_module_func.size %zu align %zu\n", sizeof(io_module_func), _Alignof(io_module_func));
	printf("RssInfo.pktidx %zu RssInfo.hash_value %zu RssInfo.size %zu\n", offsetof(RssInfo, pktidx),
	       offsetof(RssInfo, hash_value), sizeof(RssInfo));
	printf("ioctl %d %d %d %d\n", PKT_TX_IP_CSUM, PKT_TX_TCP_CSUM, PKT_RX_RSS, DRV_NAME);
#ifdef MOSRX_HAVE_MOS_IO_MODULE
	{
		int GetRSSCPUCore(uint32_t sip, uint32_t dip, uint16_t sp, uint16_t dp, int num_queues);
		/* mOS's configuration as LoadConfigurationUpperHalf leaves it (config.c:1175) */
		static struct mos_conf mc;
		static struct netdev_conf nd;
		static struct netdev_entry e[2];
		mosrx_gpu_module_cfg cfg;
		e[0].ip_addr = 0x0200000A;   /* 10.0.0.2 */
		e[1].ip_addr = 0x0101A8C0;   /* 192.168.1.1 */
		nd.num = 2;
		nd.ent[0] = &e[0];
		nd.ent[1] = &e[1];
		mc.forward = 1;
		mc.netdev_table = &nd;
		g_config.mos = &mc;
		num_queues = 0;
		if (argc > 1) {
			/* no mosrx_gpu_module_configure: the upper half opens the netdevs
			 * itself, as pcap_load_module_upper_half does */
			snprintf(e[0].dev_name, sizeof(e[0].dev_name), "%s", argv[1]);
			nd.num = 1;
			current_iomodule_func = &gpu_module_func;
			current_iomodule_func->load_module_upper_half();
			mosrx_gpu_module_get_cfg(&cfg);
			printf("auto num_ifs %u if %s src %d num_queues %d forward %d\n", cfg.num_ifs, cfg.if_names[0],
			       cfg.src[0] != NULL, num_queues, cfg.params.forward);
			return 0;
		}
		mosrx_gpu_module_cfg_default(&cfg);
		cfg.num_ifs = 1;
		cfg.params.num_queues = 3;
		cfg.params.forward = 0;
		if (mosrx_gpu_module_configure(&cfg))
			return 1;
		current_iomodule_func = &gpu_module_func;          /* core.c:1725-1733 */
		current_iomodule_func->load_module_upper_half();   /* core.c:1735 */
		mosrx_gpu_module_get_cfg(&cfg);
		printf("num_queues %d\n", num_queues);
		printf("forward %d num_local %u local %08x %08x\n", cfg.params.forward, cfg.params.num_local,
		       cfg.params.local_ip[0], cfg.params.local_ip[1]);
		printf("queue %d\n", GetRSSCPUCore(0x0A000001, 0x0A000002, 1234, 80, num_queues));   /* util.c:114 */
	}
#endif
	return 0;
}
