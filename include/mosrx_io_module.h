/*
 * mosrx_io_module.h — the GPU batch-consumer backend behind mOS's packet-I/O
 * plugin surface.
 *
 * `io_module_func` below is layout-identical to mOS's own vtable
 * (core/src/include/io_module.h:63-78); inside an mOS tree the maintainer
 * includes io_module.h instead (define MOSRX_HAVE_MOS_IO_MODULE) and registers
 * `gpu_module_func` exactly like pcap/dpdk/netmap (io_module.h:100-111,
 * core.c:1725-1733).  The backend never dereferences `struct
 * mtcp_thread_context`, so it compiles against either definition.
 *
 * Semantics kept from the reference:
 *   - recv_pkts returns the batch size (0 when idle, -1 on a bad ifidx,
 *     pcap_module.c:37-38) and get_rptr pointers stay valid until the next
 *     recv_pkts on that ifidx (dpdk_module.c:379-382, pcap_module.c:41);
 *   - dev_ioctl(PKT_RX_RSS) fills RssInfo{int8 pktidx, u32 hash_value}
 *     (io_module.h:81-84, dpdk_module.c:568-571); -1 for unsupported commands;
 *   - NULL members are "not provided" (select, link_devices, set_wptr).
 * New: dev_ioctl(MOSRX_PKT_RX_RESULTS) returns the batch's mosrx_result array,
 * whose verdicts the rx loop consumes instead of re-running ProcessPacket's checks;
 * with monitor filters configured, dev_ioctl(MOSRX_PKT_RX_MATCH) returns their
 * per-frame match masks, computed in the same pass (EVAL_BPFFILTER, ip_in.c:56-63).
 */
#ifndef MOSRX_IO_MODULE_H
#define MOSRX_IO_MODULE_H

#include <stdint.h>
#include <net/if.h>

#include "mosrx.h"

#ifdef __cplusplus
extern "C" {
#endif

struct mtcp_thread_context;

#ifdef MOSRX_HAVE_MOS_IO_MODULE
#include "io_module.h"
#else
typedef struct io_module_func {
	void      (*load_module_upper_half)(void);
	void      (*load_module_lower_half)(void);
	void      (*init_handle)(struct mtcp_thread_context *ctx);
	int32_t   (*link_devices)(struct mtcp_thread_context *ctx);
	void      (*release_pkt)(struct mtcp_thread_context *ctx, int ifidx, unsigned char *pkt_data, int len);
	uint8_t * (*get_wptr)(struct mtcp_thread_context *ctx, int ifidx, uint16_t len);
	void      (*set_wptr)(struct mtcp_thread_context *ctx, int out_ifidx, int in_ifidx, int idx);
	int32_t   (*send_pkts)(struct mtcp_thread_context *ctx, int nif);
	uint8_t * (*get_rptr)(struct mtcp_thread_context *ctx, int ifidx, int index, uint16_t *len);
	int       (*get_nif)(struct ifreq *ifr);
	int32_t   (*recv_pkts)(struct mtcp_thread_context *ctx, int ifidx);
	int32_t   (*select)(struct mtcp_thread_context *ctx);
	void      (*destroy_handle)(struct mtcp_thread_context *ctx);
	int32_t   (*dev_ioctl)(struct mtcp_thread_context *ctx, int nif, int cmd, void *argp);
} io_module_func __attribute__((aligned(__WORDSIZE)));

typedef struct {
	int8_t   pktidx;
	uint32_t hash_value;
} RssInfo;

#define PKT_TX_IP_CSUM   0x01
#define PKT_TX_TCP_CSUM  0x02
#define PKT_RX_RSS       0x03
#define DRV_NAME         0x08
#endif

#define MOSRX_PKT_RX_RESULTS 0x10   /* argp: const mosrx_result ** (whole batch) */
#define MOSRX_PKT_RX_MATCH   0x11   /* argp: const uint32_t ** (whole batch's BPF match masks, bit j = program j) */
#define MOSRX_MAX_DEVICES    16     /* MAX_DEVICES, io_module.h:87 */

extern io_module_func gpu_module_func;

/* ---- frame sources: the raw-socket / loopback side the GPU path sits behind ---- */
typedef struct mosrx_source mosrx_source;

/* Replay `n` frames from memory, `loops` times (0 = forever). Frames are copied. */
mosrx_source *mosrx_source_mem(const uint8_t *frames, const uint32_t *off, const uint16_t *len,
                               uint32_t n, uint32_t loops);
/* Classic libpcap file (magic a1b2c3d4 / d4c3b2a1, usec or nsec), LINKTYPE_ETHERNET.
 * Native reader: libpcap is absent (pcap_module.c:13). */
mosrx_source *mosrx_source_pcap(const char *path, uint32_t loops);
/* AF_PACKET raw socket on an interface (e.g. "lo"); needs CAP_NET_RAW. */
mosrx_source *mosrx_source_afpacket(const char *ifname);
/* Pull the next frame into dst (at most cap bytes); returns its caplen, 0 when none. */
int           mosrx_source_next(mosrx_source *s, uint8_t *dst, uint32_t cap);
/* How gpu_module_func takes batches from an in-memory source: 0 = best (the
 * replay buffer lent zero-copy when it is pinned, else copied in runs), 1 =
 * copied in runs, 2 = copied frame by frame (what a recvfrom-style source
 * does).  Results never depend on it.  0 or -EINVAL (not a memory source). */
int           mosrx_source_mem_set_mode(mosrx_source *s, int mode);
void          mosrx_source_close(mosrx_source *s);

/* ---- backend configuration (before load_module_upper_half) ---- */
typedef struct mosrx_gpu_module_cfg {
	uint32_t      num_ifs;                          /* netdevs (netdev_table->num) */
	char          if_names[MOSRX_MAX_DEVICES][IFNAMSIZ];
	mosrx_source *src[MOSRX_MAX_DEVICES];           /* one source per netdev (caller closes after destroy_handle) */
	uint32_t      batch;                            /* frames per recv_pkts (default 32768) */
	uint32_t      max_frame;                        /* largest frame accepted (default 2048) */
	int32_t       gpu_base;                         /* GPU for cpu c = gpu_base + c % ngpu */
	int32_t       ngpu;                             /* 0 = all visible */
	int32_t       pipeline;                         /* 1: classify batch k+1 while k is consumed */
	mosrx_params  params;                           /* stack state (num_msp, forward, key, ...) */
	const mosrx_bpf_prog *bpf_progs;                /* monitor filters (SET_BPFFILTER output), evaluated in the */
	uint32_t      bpf_nprog;                        /*   classify pass; kept by the caller until init_handle */
} mosrx_gpu_module_cfg;

void mosrx_gpu_module_cfg_default(mosrx_gpu_module_cfg *cfg);
int  mosrx_gpu_module_configure(const mosrx_gpu_module_cfg *cfg);
/* Bind a thread context pointer to a cpu index before init_handle (standalone use;
 * inside mOS the module reads nothing from ctx and uses the registration order). */
int  mosrx_gpu_module_bind(struct mtcp_thread_context *ctx, int cpu);

/* ---- RunMainLoop-shaped driver (core.c:897-909) ---- */
typedef struct mosrx_rx_stats {
	uint64_t rx_packets, rx_bytes, rx_errors;        /* NETSTAT, eth_in.c:42-45,80-84 (bytes + ETHER_OVR) */
	uint64_t rounds, batches;
	uint64_t by_reason[MOSRX_R_COUNT];
} mosrx_rx_stats;

/* Per-frame consumer: the part of ProcessPacket after the checks (flow lookup,
 * callbacks).  Gets the frame and its precomputed record; may be NULL. */
typedef void (*mosrx_pkt_fn)(void *arg, int ifidx, int index, const uint8_t *pkt, uint16_t len,
                             const mosrx_result *res);

/* Run rounds over `nif` netdevs until `max_pkts` frames were received or every
 * source is exhausted (recv_pkts == 0 on all netdevs for a whole round). */
int mosrx_rx_loop(const io_module_func *iom, struct mtcp_thread_context *ctx, int nif,
                  uint64_t max_pkts, mosrx_pkt_fn fn, void *arg, mosrx_rx_stats *st);

#ifdef __cplusplus
}
#endif
#endif
