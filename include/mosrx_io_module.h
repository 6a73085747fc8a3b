/*
 * mosrx_io_module.h — the GPU batch-consumer backend behind mOS's packet-I/O
 * plugin surface.
 *
 * `io_module_func` below is layout-identical to mOS's own vtable
 * (core/src/include/io_module.h:63-78); inside an mOS tree the maintainer
 * includes io_module.h instead (define MOSRX_HAVE_MOS_IO_MODULE) and registers
 * `gpu_module_func` exactly like pcap/dpdk/netmap (io_module.h:100-111,
 * core.c:1725-1733).  Standalone the backend never dereferences `struct
 * mtcp_thread_context`, so it compiles against either definition; built
 * inside mOS it reads the context's `cpu` and `mtcp_manager` (mtcp.h:304-312).
 *
 * Semantics kept from the reference:
 *   - recv_pkts returns the batch size (0 when idle, -1 on a bad ifidx,
 *     pcap_module.c:37-38) and get_rptr pointers stay valid until the next
 *     recv_pkts on that ifidx (dpdk_module.c:379-382, pcap_module.c:41);
 *   - dev_ioctl(PKT_RX_RSS) fills RssInfo{int8 pktidx, u32 hash_value}
 *     (io_module.h:81-84, dpdk_module.c:568-571); PKT_TX_IP_CSUM /
 *     PKT_TX_TCP_CSUM are taken as a NIC offload when cfg.tx_csum is set
 *     (dpdk_module.c:556-566); -1 for unsupported commands;
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
#define MOSRX_PKT_RX_TCPINFO 0x12   /* argp: const mosrx_tcpinfo ** (whole batch; cfg.tcpinfo set) */
#define MOSRX_PKT_SET_PARAMS 0x13   /* argp: const mosrx_params * -- the stack state changed (a monitor
                                     * socket was created: num_msp++, socket.c:77-78); batches not yet
                                     * handed out on that netdev are classified again under it */
#define MOSRX_PKT_RX_STATE   0x14   /* argp: mosrx_rx_state * -- what the exposed batch was classified under */
#define MOSRX_PKT_RX_RECLASSIFY 0x15 /* argp: unused (non-NULL) -- classify the exposed batch again now,
                                     * under mOS's current state and BPF set (blocking) */
#define MOSRX_PKT_RX_FHASH   0x17   /* argp: const uint32_t ** (whole batch): HashFlow of FindStream's tuple
                                     * before the NUM_BINS mask (cfg.flowhash set; -1 for a batch
                                     * classified with BPF filters) */
#define MOSRX_PKT_SET_BPF    0x16   /* argp: const mosrx_bpf_set_arg * -- the monitor filters to evaluate in
                                     * the classify pass from now on (nprog 0: none); batches not yet
                                     * handed out are classified again with them */
#define MOSRX_PKT_RX_RESULTS8 0x18  /* argp: const mosrx_result8 ** (whole batch): the records of a batch
                                     * classified in compact form (cfg.compact); RX_RESULTS is -1 for it */
typedef struct mosrx_rx_state {
	uint32_t num_msp, num_esp;   /* the stack state of the batch's verdicts */
	uint32_t gen;                /* the netdev's parameter / filter generation they were made with */
	uint32_t bpf_nprog;          /* programs in its match masks (0: no masks) */
	uint32_t n;                  /* frames in the batch */
	uint32_t rec_bytes;          /* its records: 16 (mosrx_result, RX_RESULTS) or 8 (mosrx_result8, RX_RESULTS8) */
} mosrx_rx_state;
typedef struct mosrx_bpf_set_arg {
	const mosrx_bpf_prog *progs;
	uint32_t nprog;
} mosrx_bpf_set_arg;
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
/* AF_PACKET raw socket on an interface (e.g. "lo") with a TPACKET_V3 PACKET_MMAP
 * receive ring; needs CAP_NET_RAW.  Frames the host sends (PACKET_OUTGOING) are
 * not received, as with libpcap's default direction.  When the ring can be
 * registered with the HIP runtime, batches are lent zero-copy to the backend. */
mosrx_source *mosrx_source_afpacket(const char *ifname);
typedef struct mosrx_afpacket_opts {
	uint32_t ring_blocks;    /* 4 MiB ring blocks (default 8, at most 64) */
	uint32_t retire_ms;      /* a partly filled block is handed over after this long (default 1) */
	uint32_t fanout_group;   /* != 0: join this PACKET_FANOUT_HASH group (one socket per mTCP
	                          * thread; flows split by hash, as RSS splits them over NIC queues) */
	int32_t  copy;           /* 1: never lend the ring (frames are copied into the stage) */
} mosrx_afpacket_opts;
mosrx_source *mosrx_source_afpacket_ex(const char *ifname, const mosrx_afpacket_opts *opts);
typedef struct mosrx_afpacket_info {
	int32_t  zero_copy;        /* the ring is registered: batches are lent, not copied */
	uint64_t ring_bytes;
	uint64_t dropped_outgoing; /* outgoing frames skipped (kernels without PACKET_IGNORE_OUTGOING) */
	uint64_t ring_packets;     /* PACKET_STATISTICS since the socket opened (pcap_stats' ps_recv) */
	uint64_t ring_drops;       /* frames the kernel dropped with every ring block owned by us (ps_drop) */
} mosrx_afpacket_info;
int           mosrx_source_afpacket_info(mosrx_source *s, mosrx_afpacket_info *info);
/* A TPACKET_V3 receive ring (linux/if_packet.h block layout: tpacket_block_desc,
 * tpacket3_hdr + sockaddr_ll per frame) at `ring`, `nblocks` blocks of
 * `block_size` bytes (a power of two), mapped by the caller and filled by
 * someone else -- another process's capture in shared memory, a driver with
 * the same layout.  Read and lent exactly like the AF_PACKET socket's ring:
 * blocks whose status has TP_STATUS_USER are taken in order and handed back
 * with TP_STATUS_KERNEL once their frames are no longer exposed.  The caller
 * keeps the mapping until mosrx_source_close.  NULL on bad arguments. */
mosrx_source *mosrx_source_tpacket_v3(void *ring, uint32_t nblocks, uint32_t block_size);
/* Pull the next frame into dst (at most cap bytes); returns its caplen, 0 when none. */
int           mosrx_source_next(mosrx_source *s, uint8_t *dst, uint32_t cap);
/* Receive up to max_n frames (at most max_frame bytes each) into dst[0, cap)
 * in gpu_module_func's staging layout: the first frame at byte 2, a frame of
 * up to 128 bytes right after the previous one, a longer one at the next
 * 16-byte boundary + 2; off[]/len[] written, *end = the bytes used.  What
 * the backend does for every batch it copies (the batch form of the source,
 * or mosrx_source_next per frame).  Returns the count or -EINVAL. */
int           mosrx_source_fill(mosrx_source *s, uint8_t *dst, uint64_t cap, uint32_t *off, uint16_t *len,
                                uint32_t max_n, uint32_t max_frame, uint64_t *end);
/* Zero-copy runs (what gpu_module_func lends to the GPU copy): up to max_n
 * frames that sit in the source's own memory, as one run from *frames in
 * buffer order -- off[]/len[] relative to it, len clamped to max_frame --
 * valid until mosrx_source_give_back releases the run (oldest first; for the
 * AF_PACKET ring that returns its blocks to the kernel).  Returns the count
 * (0: nothing ready) or -EOPNOTSUPP for sources that cannot lend. */
int           mosrx_source_borrow(mosrx_source *s, uint32_t max_n, uint32_t max_frame, const uint8_t **frames,
                                  uint64_t *frames_bytes, uint32_t *off, uint16_t *len);
int           mosrx_source_give_back(mosrx_source *s);
/* How gpu_module_func takes batches from an in-memory source: 0 = best (the
 * replay buffer lent zero-copy when it is pinned, else copied in runs), 1 =
 * copied in runs, 2 = copied frame by frame (what a recvfrom-style source
 * does).  Results never depend on it.  0 or -EINVAL (not a memory source). */
int           mosrx_source_mem_set_mode(mosrx_source *s, int mode);
void          mosrx_source_close(mosrx_source *s);

/* Transmit one frame through the source (pcap_inject, pcap_module.c:67-79): the
 * AF_PACKET socket; -EOPNOTSUPP for sources that cannot send (a trace file)
 * unless a TX dump is set.  0 or -errno. */
int           mosrx_source_send(mosrx_source *s, const uint8_t *frame, uint32_t len);
/* Divert the source's transmit into a classic pcap file (path NULL: back to
 * the native transmit).  Works for every source. */
int           mosrx_source_tx_pcap(mosrx_source *s, const char *path);
int           mosrx_source_tx_flush(mosrx_source *s);
int           mosrx_source_tx_stats(const mosrx_source *s, uint64_t *packets, uint64_t *bytes, uint64_t *errors);

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
	uint32_t      tx_batch;                         /* frames get_wptr buffers per netdev before send_pkts
	                                                 * flushes them (default 64, MAX_PKT_BURST of dpdk_module.c:61) */
	int32_t       tcpinfo;                          /* 1: also compute pkt_info's TCP fields per batch
	                                                 * (dev_ioctl(MOSRX_PKT_RX_TCPINFO)) */
	uint32_t      group;                            /* batches received per kernel launch: 1..MOSRX_MAX_GROUP,
	                                                 * or MOSRX_GROUP_AUTO (0, the default): as many batches
	                                                 * as the source has ready, up to `group_bytes` of frames.
	                                                 * A group is classified by one launch and handed out one
	                                                 * batch per recv_pkts.  With BPF filters installed a
	                                                 * launch classifies one batch. */
	uint64_t      group_bytes;                      /* MOSRX_GROUP_AUTO: frame bytes per launch aimed at
	                                                 * (0 = MOSRX_GROUP_AUTO_BYTES) */
	int32_t       flowhash;                         /* 1: also the flow-table hash of every frame
	                                                 * (dev_ioctl(MOSRX_PKT_RX_FHASH)); not with BPF filters */
	int32_t       tx_csum;                          /* 1: take mOS's TX checksum offload requests
	                                                 * (dev_ioctl PKT_TX_IP_CSUM / PKT_TX_TCP_CSUM on the frame
	                                                 * get_wptr returned last, as dpdk_dev_ioctl does,
	                                                 * dpdk_module.c:556-566) and fill those checks on the GPU
	                                                 * when send_pkts sends the frames; 0 (default): -1, mOS
	                                                 * computes them (ip_out.c:169-174, tcp_out.c:207-218) */
	int32_t       numa;                             /* 1 (default): core c drives a GPU on c's NUMA node
	                                                 * (mosrx_numa_pick); 0: gpu_base + c % ngpu */
	int32_t       compact;                          /* 1: 8-byte records (mosrx_result8: rss, reason, queue,
	                                                 * verdict, tcp_flags; dev_ioctl(MOSRX_PKT_RX_RESULTS8)),
	                                                 * written and copied back at half the bytes; the consumer
	                                                 * takes pkt_info's lengths from the header as
	                                                 * FillPacketContextTCPInfo does (tcp.c:258-270); with BPF
	                                                 * filters too (the fused kernels' 8-byte forms).  A batch's
	                                                 * mosrx_rx_state.rec_bytes says which form it has.  Not
	                                                 * with tcpinfo.  Default 0 standalone, 1 in an mOS build
	                                                 * left unconfigured (its consumer, mos_rx.c, reads both). */
	uint32_t      group_max_us;                     /* latency budget of a group (0: none): it takes no more
	                                                 * frames than, at this netdev's measured rates, cross PCIe
	                                                 * and are classified within the budget, or than the rx
	                                                 * loop walks within it (never under 4096 frames); any
	                                                 * group mode.  A group is never waited for: a receive
	                                                 * takes what has arrived.  DESIGN.md §5 (latency) */
	uint32_t      direct_kb;                        /* groups of at most this many KiB of frames + descriptors
	                                                 * launch with no copies: the kernel reads the pinned
	                                                 * staging / the source's pinned buffers and writes the
	                                                 * pinned records in place over PCIe (mosrx_set_direct).
	                                                 * 0: every group is copied.  Default
	                                                 * MOSRX_DIRECT_DEFAULT_KB */
	uint32_t      direct_frames;                    /* ... and of at most this many frames (default
	                                                 * MOSRX_DIRECT_DEFAULT_FRAMES) */
} mosrx_gpu_module_cfg;
#define MOSRX_GROUP_AUTO        0
#define MOSRX_DIRECT_DEFAULT_FRAMES 0xFFFFFFFFu   /* no frame limit: a 16K limit made the 64 B 90 % points
                                                   * worse (one batch per launch p50 / p99 58 / 84 -> 209 /
                                                   * 303 us) and did not stop the auto groups' 90 % point
                                                   * from overloading now and then, which it also does
                                                   * with every group copied (1 run in 3 either way:
                                                   * profiles/r06/direct/lat90_frames16k.txt) */
#define MOSRX_DIRECT_DEFAULT_KB 16384   /* measured (profiles/r06/direct): copy-free groups cut the
                                          * light-load p50 ~3x (64 B auto at 25 %: 108 -> 34 us) and
                                          * lift 64 B one-batch launches 257 -> 297 Mpkt/s; at 90 %
                                          * load 16 MiB was best for 64 B auto groups (p99 500 us
                                          * against 573 at 4 MiB and 4325 at 64 MiB), while 1500 B
                                          * one-batch groups of ~100 MB stay copied (direct 33.3
                                          * against 34.8 Mpkt/s) */
#define MOSRX_GROUP_AUTO_BYTES  (1ull << 30)     /* per pipeline slot; 64 B frames: ~500 batches of 32K
                                                   * per launch, 1500 B: 10 of 64K.  Measured (round 5-6,
                                                   * profiles/r06/groups): 256 MiB groups of 64 B frames ran
                                                   * 0.43 us per batch on the device, 512 MiB 0.40-0.42, 1 GiB
                                                   * 0.41 (a launch's ramp and drain spread over more batches);
                                                   * inside mOS scaled down to the pinned budget (auto_bytes) */

void mosrx_gpu_module_cfg_default(mosrx_gpu_module_cfg *cfg);
int  mosrx_gpu_module_configure(const mosrx_gpu_module_cfg *cfg);
/* The configuration in effect (after load_module_upper_half took mOS's own
 * state into it, when built inside mOS). */
int  mosrx_gpu_module_get_cfg(mosrx_gpu_module_cfg *cfg);
/* Bind a thread context pointer to a cpu index before init_handle.  Unbound
 * contexts get their cpu from ctx->cpu inside an mOS build (the mTCP core,
 * mtcp.h:306, set by MTCPRunThread before init_handle, core.c:1302-1313) and
 * from registration order standalone. */
int  mosrx_gpu_module_bind(struct mtcp_thread_context *ctx, int cpu);
/* Give mTCP thread `cpu` its own source for netdev `ifidx` (e.g. one
 * PACKET_FANOUT_HASH socket per thread), instead of cfg.src[ifidx]. */
int  mosrx_gpu_module_bind_source(int cpu, int ifidx, mosrx_source *src);
/* The GPU mTCP thread `cpu` runs on, among gpu_base .. gpu_base + ngpu - 1
 * (ngpu 0: all visible devices, `ndev`), the per-core sharding of SURVEY.md
 * §8e: with cfg.numa one on cpu's NUMA node (mosrx_numa_pick), else -- or
 * when the topology does not say -- gpu_base + cpu % ngpu.  -EINVAL if none. */
int  mosrx_gpu_module_device_of(int cpu, int ndev);

/* ---- NUMA topology (csrc/topology.c; sysfs, like mOS's cpu.c / numa(3)) ---- */
/* Node of a PCI device ("0000:c1:00.0", /sys/bus/pci/devices/<bdf>/numa_node),
 * of a core (/sys/devices/system/cpu/cpu<c>/node<n>), of HIP device `device`
 * (its PCI address from hipDeviceGetPCIBusId); -1 when unknown. */
int  mosrx_pci_numa_node(const char *bdf);
int  mosrx_cpu_numa_node(int cpu);
int  mosrx_gpu_numa_node(int device);
/* Of `ngpu` candidate GPUs on nodes gpu_node[0..ngpu-1], the one core `cpu`
 * drives: one on cpu's node, round robin by cpu's rank among the node's cores
 * (/sys/devices/system/node/node<n>/cpulist); -1 when a node is unknown or
 * cpu's node has no GPU. */
int  mosrx_numa_pick(int cpu, const int *gpu_node, int ngpu);
/* Read sysfs under `root` instead of "/" (tests: a fake tree; NULL or "/": the real one). */
int  mosrx_topology_set_root(const char *root);
/* Frames a context sent, received and dropped on TX (per netdev summed). */
typedef struct mosrx_gpu_module_stats {
	uint64_t rx_batches, rx_frames, tx_packets, tx_bytes, tx_errors;
	uint64_t kernel_launches;   /* timed launches (mosrx_set_timing on the thread's contexts) */
	double   kernel_ms;         /* their summed device time (HIP events around each kernel) */
	uint64_t rx_drops;          /* frames received but never handed out: their group's launch failed */
	uint64_t rx_reclassified;   /* batches classified again because mOS's stack state (num_msp /
	                               num_esp) changed after they were classified (mOS builds) */
	int32_t  cpu;               /* the mTCP core the context runs as (bind, or ctx->cpu in mOS builds) */
	int32_t  device;            /* the GPU it drives: gpu_base + cpu % ngpu */
	uint64_t tx_csum_offloaded; /* TX frames whose requested checks the GPU filled (cfg.tx_csum); frames
	                               whose pass failed are dropped and counted in tx_errors */
	int32_t  cpu_node;          /* the core's NUMA node, -1 unknown */
	int32_t  gpu_node;          /* its GPU's, -1 unknown */
	uint64_t rx_groups;         /* groups handed out (one launch each) */
	uint64_t max_group_frames;  /* frames of the largest of them */
	uint64_t group_cap_frames;  /* the frame cap cfg.group_max_us gave the last group filled (0: none) */
	double   ns_per_frame_host; /* the latency cap's rates: the host's time per frame of a group */
	double   ns_per_byte_dev;   /*   and a group's submit -> records ready per frame byte (0: not measured) */
	uint64_t rx_direct_groups;  /* groups of rx_groups that launched with no copies (cfg.direct_kb) */
} mosrx_gpu_module_stats;
/* Time every kernel this thread's contexts launch (for the stats above). */
int  mosrx_gpu_module_set_timing(struct mtcp_thread_context *ctx, int on);
int  mosrx_gpu_module_stats_of(struct mtcp_thread_context *ctx, mosrx_gpu_module_stats *st);

/* ---- RunMainLoop-shaped driver (core.c:897-909) ---- */
typedef struct mosrx_rx_stats {
	uint64_t rx_packets, rx_bytes, rx_errors;        /* NETSTAT, eth_in.c:42-45,80-84 (bytes + ETHER_OVR) */
	uint64_t rounds, batches;
	uint64_t by_reason[MOSRX_R_COUNT];
	uint64_t recv_errors;                            /* recv_pkts calls that returned < 0: skipped, as core.c:899-902
	                                                    (a round whose receives all failed counts as idle) */
} mosrx_rx_stats;

/* Per-frame consumer: the part of ProcessPacket after the checks (flow lookup,
 * callbacks).  Gets the frame and its precomputed record; may be NULL.  For a
 * compact batch the record carries the mosrx_result8 fields (rss, reason,
 * queue, verdict, tcp_flags) and zero elsewhere. */
typedef void (*mosrx_pkt_fn)(void *arg, int ifidx, int index, const uint8_t *pkt, uint16_t len,
                             const mosrx_result *res);

/* Run rounds over `nif` netdevs until `max_pkts` frames were received or every
 * source is exhausted (recv_pkts == 0 on all netdevs for a whole round). */
int mosrx_rx_loop(const io_module_func *iom, struct mtcp_thread_context *ctx, int nif,
                  uint64_t max_pkts, mosrx_pkt_fn fn, void *arg, mosrx_rx_stats *st);

/* The same loop for live sources: a round that receives nothing sleeps
 * `idle_us` and the loop ends after `idle_rounds` such rounds in a row (0:
 * only at max_pkts / max_us), or after `max_us` microseconds (0: no limit).
 * Every round ends with send_pkts on each netdev (core.c:999-1007), so frames
 * a consumer wrote with get_wptr leave in the same round. */
struct mosrx_latency_probe;
typedef struct mosrx_rx_loop_opts {
	uint64_t max_pkts;
	uint32_t idle_rounds;
	uint32_t idle_us;
	uint64_t max_us;
	struct mosrx_latency_probe *probe;   /* NULL, or the residency of a paced source's frames (below) */
} mosrx_rx_loop_opts;
int mosrx_rx_loop_ex(const io_module_func *iom, struct mtcp_thread_context *ctx, int nif,
                     const mosrx_rx_loop_opts *opts, mosrx_pkt_fn fn, void *arg, mosrx_rx_stats *st);

/* A consumer for mosrx_rx_loop*: the frames mOS forwards with `forward` set,
 * decided from the verdict reason and the stack state as ProcessPacket's paths
 * do (mosrx_mos_forwards), each copied with ForwardEthernetFrame's steps
 * (eth_out.c:105-129: out_if[in_ifidx] from the nic_forward_table, get_wptr,
 * copy; -1 in out_if drops).  `arg` points at a mosrx_forwarder.  The round's
 * send_pkts sends what it wrote. */
typedef struct mosrx_forwarder {
	const io_module_func *iom;
	struct mtcp_thread_context *ctx;
	int32_t out_if[MOSRX_MAX_DEVICES];
	uint64_t forwarded;          /* frames copied into a TX buffer of the output netdev */
	uint64_t dropped;            /* every other frame: not forwarded by the rule, or no output
	                                netdev (out_if -1) / no TX buffer (get_wptr NULL) */
	int32_t forward;             /* mos.conf `forward` (pctx->forward) */
	uint32_t num_msp;            /* monitor sockets of the stack the records were made under */
	uint32_t listener;           /* 1 when an end-host socket listens (mtcp->listener, mtcp_listen) */
} mosrx_forwarder;
/* 1 when mOS forwards a frame with this record, 0 when it consumes or drops it,
 * for a frame of a flow the stack holds no stream for (the standalone rx loop
 * keeps no flow table; pinned to ProcessPacket with the forwarding calls
 * recorded, tests/golden/forward.npz):
 *   NON_IPV4, ARP            forward && num_msp: ForwardEthernetFrame, eth_in.c:60-77 (ARP
 *                            is processed locally only when forwarding is off)
 *   NOVERIFY_PASS            forward: ForwardIPPacket before the transport layer, ip_in.c:66-70
 *   NOT_TCP (not to me)      forward && num_msp: ip_in.c:86-91
 *   TCP_BADCSUM              forward && num_msp: tcp.c:438-442 (the verdict stays -1)
 *   TCP_OK / TCP_LEN_OK      forward && num_msp && !listener: no stream is found, so
 *                            CreateStream makes a monitor stream (SYN, HandleMonitorStream
 *                            forwards, tcp.c:386-390) or none (the orphan path forwards,
 *                            :507-510); with a listener the orphan gets a RST instead
 *                            (:497-506); with no monitor socket the segment is consumed
 *                            (:453-457).  Frames of end-host streams are the flow engine's.
 *   ICMP_LOCAL               consumed locally; the rest are dropped. */
int  mosrx_mos_forwards(const mosrx_result *res, int forward, uint32_t num_msp, uint32_t listener);
void mosrx_forward_frame(void *arg, int ifidx, int index, const uint8_t *pkt, uint16_t len,
                         const mosrx_result *res);

/* ---- residency of frames from a paced source (latency of the drop-in path) ----
 * mosrx_source_paced: `inner`'s frames released at `rate_pps` -- frame k
 * arrives at t0 + k * 1e9 / rate_pps, t0 being the first receive call -- and
 * none before it arrives, as a NIC ring fills at line rate.  It takes `inner`
 * over (closing it closes both).  Not for AF_PACKET sources (a live wire has its
 * own pace).  mosrx_source_paced_info: t0 (CLOCK_MONOTONIC ns, 0 before the first
 * receive), ns between arrivals, frames handed out. */
mosrx_source *mosrx_source_paced(mosrx_source *inner, double rate_pps);
int           mosrx_source_paced_info(const mosrx_source *s, uint64_t *t0_ns, double *ns_per_frame,
                                      uint64_t *released);

/* Residency of a paced source's frames through the rx loop
 * (mosrx_rx_loop_opts.probe; one netdev): the k-th frame the loop receives is
 * arrival k.  Per frame after the first `skip`: recv -> verdict available (the
 * clock when recv_pkts returned its batch with the records) into avail_hist,
 * and recv -> consumed (that clock plus the frame's share of the batch's walk,
 * the walk taken as even over the batch) into done_hist.  Two clock reads per
 * batch, nothing per frame.  Histogram bin of v ns: v below 16, else
 * 16 * floor(log2 v) + the next 4 bits of v (6 % wide). */
#define MOSRX_LAT_BINS 1024
typedef struct mosrx_latency_probe {
	const mosrx_source *src;      /* the paced source of the netdev (t0 and pace read at the first batch) */
	uint64_t t0_ns;
	double   ns_per_frame;
	uint64_t skip;                /* warm-up frames not recorded */
	uint64_t seen, recorded, batches;
	uint64_t avail_max_ns, done_max_ns;
	uint64_t avail_hist[MOSRX_LAT_BINS];
	uint64_t done_hist[MOSRX_LAT_BINS];
} mosrx_latency_probe;

#ifdef __cplusplus
}
#endif
#endif
