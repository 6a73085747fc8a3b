/*
 * mosrx.h — C ABI of the MI355X receive-path classifier for mOS.
 *
 * One call classifies a batch of received Ethernet frames on a gfx950 GPU and
 * emits one 16-byte result record per frame.  The per-frame transform is the
 * part of mOS's software receive path that runs before the stateful flow
 * engine:
 *
 *   ProcessPacket          core/src/eth_in.c:27-87      (ethertype dispatch)
 *   ProcessInIPv4Packet    core/src/ip_in.c:30-101      (IPv4 checks)
 *   ip_fast_csum           core/src/include/ip_in.h:10-38
 *   ProcessInTCPPacket     core/src/tcp.c:408-445       (prefix up to FindStream)
 *   FillPacketContextTCPInfo core/src/tcp.c:258-270
 *   TCPCalcChecksum        core/src/tcp_util.c:157-190
 *   GetRSSHash/BuildKeyCache core/src/util.c:27-99     (Toeplitz RSS)
 *   GetRSSCPUCore          core/src/util.c:114-131     (queue map)
 *
 * The verdict in each record is bit-identical to ProcessPacket()'s return value
 * (1 / 0 / -1) for the same frame and the same stack state (num_msp, num_esp,
 * forward); `reason` distinguishes the causes that share a return value.
 *
 * Conventions (mirroring the reference's io_module_func, io_module.h:63-78):
 *   - every function returns 0 on success or a negative errno value;
 *   - the caller owns every buffer; the library never frees caller memory;
 *   - one mosrx_ctx per host thread (mOS runs one mTCP thread per core, and
 *     all io_module calls for a context come from that thread, core.c:1282-1349).
 *
 * No HIP, torch or C++ types appear in this header: streams are passed as
 * `void *` (a hipStream_t), device buffers as plain pointers.
 */
#ifndef MOSRX_H
#define MOSRX_H

#ifndef __HIPCC_RTC__
#include <stddef.h>
#include <stdint.h>
#else   /* compiled by hipRTC for a fused BPF kernel (csrc/bpf_jit.c): no libc headers there */
typedef unsigned char uint8_t;
typedef signed char int8_t;
typedef unsigned short uint16_t;
typedef unsigned int uint32_t;
typedef int int32_t;
typedef unsigned long long uint64_t;
typedef long long int64_t;
typedef unsigned long size_t;
#endif

#ifdef __cplusplus
extern "C" {
#endif

#define MOSRX_ABI_VERSION 3

/* ---- per-frame result record (16 bytes) -------------------- */

/* reason codes */
enum {
	MOSRX_R_TCP_OK        = 0,  /* TCP segment passed every check        -> 1  (tcp.c:445)      */
	MOSRX_R_ARP           = 1,  /* ARP ethertype (RUN_ARP) or forwarded  -> 1  (eth_in.c:63-66) */
	MOSRX_R_NON_IPV4      = 2,  /* other ethertype: -1, or 1 if forward && num_msp (eth_in.c:62-77) */
	MOSRX_R_IP_SHORT      = 3,  /* tot_len < 20                          -> -1 (ip_in.c:42-45)  */
	MOSRX_R_IP_BADVER     = 4,  /* version != 4                          -> 0  (ip_in.c:47-51)  */
	MOSRX_R_NOVERIFY_PASS = 5,  /* num_msp == 0 && num_esp == 0          -> 1  (ip_in.c:67-72)  */
	MOSRX_R_IP_BADCSUM    = 6,  /* ip_fast_csum != 0                     -> -1 (ip_in.c:74-77)  */
	MOSRX_R_NOT_TCP       = 7,  /* protocol != TCP                       -> 0  (ip_in.c:82-93)  */
	MOSRX_R_TCP_SHORT     = 8,  /* ip_len < (ihl + doff) * 4             -> -1 (tcp.c:429-430)  */
	MOSRX_R_TCP_BADCSUM   = 9,  /* TCPCalcChecksum != 0                  -> -1 (tcp.c:432-444)  */
	MOSRX_R_TRUNCATED     = 10, /* build-only: a byte the reference reads lies past caplen -> -1 */
	MOSRX_R_TCP_LEN_OK    = 11, /* skip_tcp_csum mode: length check passed -> 1                 */
	MOSRX_R_ICMP_LOCAL    = 12, /* ICMP to a local address: ProcessICMPPacket -> 1 (ip_in.c:83-85, icmp.c:193-227) */
	MOSRX_R_COUNT         = 13
};

typedef struct mosrx_result {
	uint32_t rss;         /* GetRSSHash(ntohl(saddr), ntohl(daddr), ntohs(sport), ntohs(dport)); ports 0 if not TCP */
	uint16_t ip_csum;     /* raw ip_fast_csum() value (0 == valid); 0 if not computed */
	uint16_t tcp_csum;    /* raw TCPCalcChecksum() value (0 == valid); 0 if not computed */
	uint16_t payloadlen;  /* pkt_info.payloadlen (tcp.c:262, u16 arithmetic, may wrap) */
	uint8_t  payload_off; /* 14 + ihl*4 + doff*4 (<= 134); 0 if not TCP */
	int8_t   verdict;     /* ProcessPacket() return value: 1, 0 or -1 */
	uint8_t  reason;      /* MOSRX_R_* */
	uint8_t  queue;       /* GetRSSCPUCore() queue for rss */
	uint8_t  tcp_flags;   /* TCP flags byte (header byte 13); 0 if not TCP */
	uint8_t  ihl_doff;    /* (ihl << 4) | doff; doff 0 if not TCP */
} mosrx_result;

/* Compact 8-byte record (opt-in, mosrx_classify_dev_compact / MOSRX_QUEUE_COMPACT):
 * what an rx loop that keeps no per-frame checksum values reads of a record --
 * the hash and queue (GetRSSHash / GetRSSCPUCore), the reason code and verdict
 * (ProcessPacket's return), the TCP flags byte.  Field for field equal to the
 * same fields of the 16-byte record; half the bytes written per frame, which
 * is a tenth of the HBM traffic of a 64 B frame (BASELINE config #2). */
typedef struct mosrx_result8 {
	uint32_t rss;
	uint8_t  reason;
	uint8_t  queue;
	int8_t   verdict;
	uint8_t  tcp_flags;
} mosrx_result8;

/* pkt_info's TCP fields (mos_api.h:122-152) as FillPacketContextTCPInfo
 * (tcp.c:258-270) fills them, for FindStream and the flow engine after it
 * (tcp.c:448): host order.  12 bytes per frame, an optional side array of the
 * classify calls (_ex); all zero where the record's payload_off is 0. */
typedef struct mosrx_tcpinfo {
	uint32_t seq;         /* ntohl(tcph->seq) */
	uint32_t ack_seq;     /* ntohl(tcph->ack_seq) */
	uint16_t window;      /* ntohs(tcph->window) */
	uint16_t ip_len;      /* pkt_info.ip_len = ntohs(iph->tot_len) (ip_in.c:36, :53) */
} mosrx_tcpinfo;

/* ---- parameters: the reference stack state the verdict depends on --------- */

enum { MOSRX_QMAP_I40E = 1, MOSRX_QMAP_IXGBE = 0 };  /* FetchEndianType() values, config.c:1261-1278 */

#define MOSRX_RSS_KEY_MAX 52   /* the DPDK backend programs a 52-byte key (dpdk_module.c:652-662) */
#define MOSRX_MAX_LOCAL   16   /* netdev entries, MAX_ETH_ENTRY = MAX_DEVICES (config.h:15, io_module.h:87) */

typedef struct mosrx_params {
	uint32_t num_msp;        /* # MOS_SOCK_MONITOR_STREAM sockets (mtcp.h:243); simple_firewall: 1 */
	uint32_t num_esp;        /* # MOS_SOCK_STREAM sockets (mtcp.h:244) */
	int32_t  forward;        /* mos.conf `forward` (config.c:608); setup.sh writes 1 */
	int32_t  num_queues;     /* GetRSSCPUCore num_queues, 1..256 (pcap: 1, pcap_module.c:159) */
	int32_t  queue_mode;     /* MOSRX_QMAP_I40E (non-DPDK default) or MOSRX_QMAP_IXGBE */
	int32_t  skip_tcp_csum;  /* 1: header parse + IP checksum + RSS only (BASELINE config #2) */
	uint32_t rss_key_len;    /* >= 16; only key bytes 0..15 affect a 12-byte input (util.c:47-57) */
	uint8_t  rss_key[MOSRX_RSS_KEY_MAX];
	/* the netdevs' IPv4 addresses (netdev_table->ent[i]->ip_addr, network order as
	 * stored, config.h:54-60): ProcessICMPPacket takes ICMP frames to one of them
	 * (icmp.c:193-200) and ProcessPacket then returns 1 instead of 0 */
	uint32_t num_local;      /* 0..MOSRX_MAX_LOCAL */
	uint32_t local_ip[MOSRX_MAX_LOCAL];
} mosrx_params;

/* simple_firewall's state: num_msp=1, num_esp=0, forward=1, num_queues=1,
 * i40e map, the all-0x05 40-byte key of util.c:36-42. */
void mosrx_params_default(mosrx_params *p);
/* The Microsoft reference Toeplitz key (util/rss.c:75-81), for the MSDN vectors. */
void mosrx_params_set_ms_key(mosrx_params *p);

/* ---- a batch of frames ---------------------------------------------------- */

/* Frame i occupies frames[off[i] .. off[i]+len[i]).  The fast layout puts each
 * frame at a 16-byte boundary + 2 (IP header 16-byte aligned); any offset is
 * accepted.  Offsets are relative to `frames`; frames_bytes bounds every read
 * (the kernel never touches memory outside [frames, frames+frames_bytes)). */
/* Largest batch buffer: its 16-byte-rounded range stays below the offset the
 * kernels use for "no load" (0xFFFFFFF0), so no rounding can wrap. */
#define MOSRX_MAX_FRAMES_BYTES 0xFFFFFFE0ull

typedef struct mosrx_batch {
	const uint8_t  *frames;       /* device pointer (classify_dev) or host pointer (classify_host) */
	uint64_t        frames_bytes; /* <= MOSRX_MAX_FRAMES_BYTES, else -E2BIG */
	const uint32_t *off;          /* n frame offsets */
	const uint16_t *len;          /* n capture lengths (pcap caplen / get_rptr *len, core.c:903-905) */
	uint32_t        n;            /* frames in the batch */
	uint32_t        max_len;      /* max(len[]) if known, else 0 (selects the kernel variant) */
	/* Layout hint (ABI 3).  MOSRX_BATCH_UNIFORM: the producer packed the frames
	 * at a fixed stride, frame i at off0 + i * stride (an rx ring of fixed-size
	 * buffers, a stage of equal-size frames).  The kernel then issues each
	 * frame's header loads from that address together with its descriptor
	 * loads instead of behind them; off[] still decides: a frame whose off[i]
	 * differs is re-read from off[i], so a wrong hint costs time, never a
	 * result.  Used when off0 and stride fit 16 bits; 0 = no hint. */
	uint32_t        layout;       /* MOSRX_BATCH_* */
	uint32_t        off0;
	uint32_t        stride;
	uint32_t        reserved;     /* 0 */
} mosrx_batch;
enum { MOSRX_BATCH_UNIFORM = 1 };

typedef struct mosrx_ctx mosrx_ctx;

/* Open a context on HIP device `device`.  Fails with -ENODEV when no GPU or
 * the HIP kernels are unavailable: there is no CPU fallback. */
int  mosrx_open(int device, const mosrx_params *p, mosrx_ctx **out);
/* Visible HIP devices (0 without a GPU or runtime). */
int  mosrx_device_count(void);
int  mosrx_set_params(mosrx_ctx *c, const mosrx_params *p);
/* Tuning knob (0..127; results never depend on it): bit 1 = non-temporal tail
 * stream (bit 0, non-temporal header windows, measured slower and folded onto
 * bit 1's setting); bits 2-6 = force a kernel shape (value - 1; 0 = automatic).
 * Default from measurements; env MOSRX_KVARIANT overrides at open. */
int  mosrx_set_variant(mosrx_ctx *c, int variant);
void mosrx_close(mosrx_ctx *c);

/* Device-resident classification: `b` points at device memory, results go to
 * device memory `d_out[n]`.  Enqueued on `stream` (a hipStream_t, NULL = the
 * context's own stream); returns after enqueue.  Graph-capturable. */
int  mosrx_classify_dev(mosrx_ctx *c, const mosrx_batch *b, mosrx_result *d_out, void *stream);

/* Same, plus the flow-table hash of every frame into device memory
 * `d_fhash[n]`: SuperFastHash of FindStream's reversed tuple (tcp.c:185-190,
 * fhash.c:25-92) before the NUM_BINS mask, i.e. HashFlow() == d_fhash[i] &
 * 0x1FFFF.  0 where payload_off == 0 (no TCP header).  Replaces the per-packet
 * HashFlow call of HTSearch (fhash.c:184-203) with a precomputed bucket. */
int  mosrx_classify_dev_fh(mosrx_ctx *c, const mosrx_batch *b, mosrx_result *d_out, uint32_t *d_fhash,
                           void *stream);

/* Same, with every optional per-frame side array: d_fhash[n] (NULL: none, as
 * above) and d_tcpinfo[n] (NULL: none), the pkt_info TCP fields, computed in the
 * same pass from the header bytes the kernel already holds. */
int  mosrx_classify_dev_ex(mosrx_ctx *c, const mosrx_batch *b, mosrx_result *d_out, uint32_t *d_fhash,
                           mosrx_tcpinfo *d_tcpinfo, void *stream);

/* Same with 8-byte records into device memory d_out8[n] (8-byte aligned). */
int  mosrx_classify_dev_compact(mosrx_ctx *c, const mosrx_batch *b, mosrx_result8 *d_out8, void *stream);

/* Device-resident classification of `nb` batches in one launch sequence. */
int  mosrx_classify_dev_many(mosrx_ctx *c, const mosrx_batch *b, uint32_t nb,
                             mosrx_result *const *d_out, void *stream);

/* Batch queue: a device-resident descriptor table of `nb` resident batches
 * that ONE kernel launch classifies (a workgroup finds its batch by binary
 * search).  Amortises launch latency for small batches (64 B frames, 32K per
 * batch); every batch keeps its own frames, descriptors and result buffer. */
typedef struct mosrx_queue mosrx_queue;
int  mosrx_queue_create(mosrx_ctx *c, const mosrx_batch *b, uint32_t nb,
                        mosrx_result *const *d_out, mosrx_queue **q);
int  mosrx_queue_run(mosrx_ctx *c, const mosrx_queue *q, void *stream);
void mosrx_queue_destroy(mosrx_ctx *c, mosrx_queue *q);
/* The batch queue with its options: d_out[i] points at 16-byte records, or at
 * 8-byte ones (mosrx_result8) with MOSRX_QUEUE_COMPACT; d_fhash[i] (NULL: none)
 * the flow-table hashes; d_match[i] (NULL: none) the match masks of the BPF set
 * installed when the queue runs -- one launch of the fused classify + BPF
 * queue kernel when the set has its compiled form, else the classify launch
 * followed by the set's kernel per batch (same results).  Compact records go
 * with both side arrays (the fused kernels have 8-byte forms). */
enum { MOSRX_QUEUE_COMPACT = 1 };
int  mosrx_queue_create_ex(mosrx_ctx *c, const mosrx_batch *b, uint32_t nb, void *const *d_out,
                           uint32_t *const *d_fhash, uint32_t *const *d_match, int flags, mosrx_queue **q);
/* `iters` back-to-back launches cycling over `nq` queues; HIP events on the
 * kernel stream (total, and per launch for the average kernel duration). */
int  mosrx_time_queue(mosrx_ctx *c, mosrx_queue *const *q, uint32_t nq, uint32_t iters,
                      float *total_ms, float *avg_kernel_ms);

/* End-to-end: host frames -> pinned staging -> H2D -> kernel -> D2H -> h_out.
 * Blocks until h_out is filled.  When frames, off and len lie in ONE host
 * block (any order, not overlapping frames_bytes, frames 16-byte aligned
 * within it, gaps under an eighth of the payload + 4 KiB) the batch crosses
 * PCIe in a single copy of that span; otherwise in three (one per array). */
int  mosrx_classify_host(mosrx_ctx *c, const mosrx_batch *b, mosrx_result *h_out);
/* Same, plus the flow hashes into h_fhash[n] (see mosrx_classify_dev_fh). */
int  mosrx_classify_host_fh(mosrx_ctx *c, const mosrx_batch *b, mosrx_result *h_out, uint32_t *h_fhash);
/* Same, with the optional side arrays of mosrx_classify_dev_ex (either may be NULL). */
int  mosrx_classify_host_ex(mosrx_ctx *c, const mosrx_batch *b, mosrx_result *h_out, uint32_t *h_fhash,
                            mosrx_tcpinfo *h_tcpinfo);

/* Asynchronous end-to-end form for pipelining: two slots per context, each
 * with its own stream.  submit enqueues H2D -> kernel -> D2H and returns; wait
 * blocks until that slot's h_out is filled.  The host buffers must stay valid
 * (and unmodified) until the wait returns; pinned buffers (mosrx_host_alloc)
 * make the copies asynchronous. */
#define MOSRX_NSLOT 2
int  mosrx_classify_host_submit(mosrx_ctx *c, int slot, const mosrx_batch *b, mosrx_result *h_out);
int  mosrx_classify_host_wait(mosrx_ctx *c, int slot);
/* Size both slots' device buffers for submits of up to `frames_bytes` of frame
 * buffers (group copies included) and `n` frames, now: without it a slot grows
 * on the first submit that needs more, which synchronises and reallocates (a
 * stall of milliseconds in the middle of traffic).  -EBUSY while a slot runs. */
int  mosrx_classify_host_reserve(mosrx_ctx *c, uint64_t frames_bytes, uint32_t n);
/* 1 when the slot's last submit has completed (its wait would not block) or
 * nothing is outstanding on it, 0 while it runs, -errno on error. */
int  mosrx_classify_host_ready(mosrx_ctx *c, int slot);

/* The same with the pkt_info TCP fields into h_tcpinfo[n] (NULL: none). */
int  mosrx_classify_host_submit_ex(mosrx_ctx *c, int slot, const mosrx_batch *b, mosrx_result *h_out,
                                   mosrx_tcpinfo *h_tcpinfo);

/* A group of `nb` (1..MOSRX_MAX_GROUP) host batches through ONE kernel launch
 * on a pipeline slot (the batch queue of mosrx_queue_*, for batches that start
 * in host memory): the batches' frames and descriptors cross PCIe in as few
 * copies as their layout allows (batches staged back to back in one pinned
 * block, or runs lent one after another by a source, go in one), the kernel
 * classifies all of them, records land in h_out[i] (and pkt_info fields in
 * h_tcpinfo[i] when h_tcpinfo is not NULL).  Wait with
 * mosrx_classify_host_wait; the counters are the group's sum.  Amortises the
 * launch for small batches the way an rx ring of several batches would. */
#define MOSRX_MAX_GROUP 512
int  mosrx_classify_host_group_submit(mosrx_ctx *c, int slot, const mosrx_batch *b, uint32_t nb,
                                      mosrx_result *const *h_out, mosrx_tcpinfo *const *h_tcpinfo);
/* The same, plus the flow-table hash of every frame into h_fhash[i] (NULL: none;
 * see mosrx_classify_dev_fh): the bucket FindStream / HTSearch would compute. */
int  mosrx_classify_host_group_submit_ex(mosrx_ctx *c, int slot, const mosrx_batch *b, uint32_t nb,
                                         mosrx_result *const *h_out, mosrx_tcpinfo *const *h_tcpinfo,
                                         uint32_t *const *h_fhash);
/* The same with 8-byte records (mosrx_result8) into h_out8[i] and, when
 * h_fhash is not NULL, the flow hashes (no pkt_info fields): the group's records are written and copied back at half the bytes
 * (gpu_module_func's cfg.compact, the records an rx loop consumes when it
 * takes pkt_info's lengths from the header, tcp.c:258-270). */
int  mosrx_classify_host_group_submit_c8(mosrx_ctx *c, int slot, const mosrx_batch *b, uint32_t nb,
                                         mosrx_result8 *const *h_out8, uint32_t *const *h_fhash);
/* The same with a BPF set installed: 8-byte records, the flow hashes (NULL:
 * none) and the set's match masks, from one launch of the fused kernel's
 * 8-byte form (or the classify launch + the set per batch while the set has
 * no compiled form). */
int  mosrx_classify_host_group_submit_bpf_c8(mosrx_ctx *c, int slot, const mosrx_batch *b, uint32_t nb,
                                             mosrx_result8 *const *h_out8, uint32_t *const *h_fhash,
                                             uint32_t *const *h_match);
/* The same for a context with a BPF set installed: the records, the flow
 * hashes (h_fhash, NULL: none) and the set's match masks into h_match[i] from
 * ONE launch of the fused classify + BPF queue kernel (the set's compiled
 * form); while the set is still compiling (mosrx_bpf_set_async) or has no
 * compiled form, the classify launch and the set's interpreter kernel per
 * batch, on the slot's stream, same results.  No pkt_info fields with masks. */
int  mosrx_classify_host_group_submit_bpf(mosrx_ctx *c, int slot, const mosrx_batch *b, uint32_t nb,
                                          mosrx_result *const *h_out, uint32_t *const *h_fhash,
                                          uint32_t *const *h_match);

/* Kernel timing on the end-to-end path: with timing on, every submit's kernel
 * launch carries a start / stop event pair its dispatch stamps (the kernel's
 * own duration, as rocprofv3 reports it; events recorded around the two
 * launches of a classify + BPF pair without the fused kernel), and after the
 * wait mosrx_last_kernel_ms gives that device time (-ENODATA if the last
 * waited submit was not timed). */
int  mosrx_set_timing(mosrx_ctx *c, int on);
/* Group submits (mosrx_classify_host_group_submit*) make the per-reason
 * counters of mosrx_last_counters (on, the default) or not (off: no counter
 * atomics in the kernel and no copy back per group; mosrx_last_counters then
 * reads zeros after such a wait).  gpu_module_func turns them off: mOS counts
 * NETSTAT from the records. */
int  mosrx_set_counters(mosrx_ctx *c, int on);
/* Direct groups: a group submit of at most max_frames frames whose frames and
 * descriptors total at most max_bytes (0, the default: none), all of them in
 * pinned memory the library
 * knows (mosrx_host_alloc / mosrx_host_register, or a source's pinned
 * buffers) with 16-byte aligned frame buffers, launches with no copies: the
 * kernel reads them, and the batch table, in place over PCIe, and writes the
 * outputs in place when every output array is pinned too (else it copies
 * them back as usual).  Records are identical either way; a small group skips
 * the copy chain (a blit or SDMA dispatch and a queue handoff per copy), which
 * shortens the group cycle at light load.  mosrx_slot_direct: 1 when the
 * slot's last group submit went direct, 0 if not. */
int  mosrx_set_direct(mosrx_ctx *c, uint64_t max_bytes, uint32_t max_frames);
int  mosrx_slot_direct(mosrx_ctx *c, int slot);
int  mosrx_last_kernel_ms(mosrx_ctx *c, float *ms);

/* Per-reason counters of the last completed end-to-end batch (MOSRX_R_COUNT
 * entries), the NETSTAT rx view of eth_in.c:42-45,80-84. */
int  mosrx_last_counters(mosrx_ctx *c, uint64_t counts[MOSRX_R_COUNT]);

/* Synchronise the context's stream. */
int  mosrx_sync(mosrx_ctx *c);

/* Device memory helpers so callers need no HIP headers. */
int  mosrx_dev_alloc(mosrx_ctx *c, size_t bytes, void **dptr);
int  mosrx_dev_free(mosrx_ctx *c, void *dptr);
/* Pinned (page-locked) host memory: the staging a backend fills from the wire
 * so H2D copies run at full PCIe rate. */
int  mosrx_host_alloc(mosrx_ctx *c, size_t bytes, void **hptr);
int  mosrx_host_free(mosrx_ctx *c, void *hptr);
/* Host memory the caller owns, made known to the library: pinned here
 * (hipHostRegister), or, with MOSRX_HOST_PINNED, already pinned by the caller
 * (hipHostMalloc / hipHostRegister of its own) and only recorded.  Batches and
 * groups whose frames and descriptors lie in one known range cross PCIe in one
 * copy (mosrx_classify_host, the group submits).  Unregister before freeing. */
enum { MOSRX_HOST_PINNED = 1 };
int  mosrx_host_register(mosrx_ctx *c, void *hptr, size_t bytes, int flags);
int  mosrx_host_unregister(mosrx_ctx *c, void *hptr);
int  mosrx_memcpy_h2d(mosrx_ctx *c, void *dst, const void *src, size_t bytes);
int  mosrx_memcpy_d2h(mosrx_ctx *c, void *dst, const void *src, size_t bytes);
/* mosrx_memcpy_h2d done by the CUs instead of the SDMA engine: a kernel reads
 * the pinned host memory over PCIe and writes HBM (src: hipHostMalloc'd or
 * registered memory; -EINVAL otherwise).  Synchronous. */
int  mosrx_memcpy_h2d_pull(mosrx_ctx *c, void *dst, const void *src, size_t bytes);
void *mosrx_stream(mosrx_ctx *c);

/* ---- timing helpers (HIP events on the context stream) -------------------- */
/* Run `iters` classify_dev calls cycling over `nb` resident batches and return
 * the elapsed device time in milliseconds between events recorded on the same
 * stream the kernels run on.  Used by bench.py for the live roofline figure. */
int  mosrx_time_dev(mosrx_ctx *c, const mosrx_batch *b, uint32_t nb,
                    mosrx_result *const *d_out, uint32_t iters, float *ms);
/* Same, with batch i enqueued on stream i % nstreams (1..MOSRX_MAX_STREAMS):
 * independent batches overlap launch and drain, as several rx queues would. */
#define MOSRX_MAX_STREAMS 8
int  mosrx_time_dev_streams(mosrx_ctx *c, const mosrx_batch *b, uint32_t nb,
                            mosrx_result *const *d_out, uint32_t iters, uint32_t nstreams, float *ms);
/* Average duration of one classify kernel over `iters` launches, each bracketed
 * by its own pair of HIP events on the stream it runs on (the roofline figure). */
int  mosrx_time_dev_kernels(mosrx_ctx *c, const mosrx_batch *b, uint32_t nb,
                            mosrx_result *const *d_out, uint32_t iters, float *avg_ms);
/* The same two measurements for any row of the path: `op` over batch i % nb
 * on stream i % nstreams (total_ms), and the average single-launch duration on
 * the context stream (avg_kernel_ms); either pointer may be NULL.  out[i]:
 * records (CLASSIFY, CLASSIFY_FH, CLASSIFY_BPF), match masks (BPF), unused
 * (TX_CSUM, `arg` = its flags); aux[i]: flow hashes (CLASSIFY_FH), match masks
 * (CLASSIFY_BPF). */
enum { MOSRX_OP_CLASSIFY = 0, MOSRX_OP_CLASSIFY_FH = 1, MOSRX_OP_BPF = 2, MOSRX_OP_TX_CSUM = 3,
       MOSRX_OP_CLASSIFY_BPF = 4, MOSRX_OP_CLASSIFY_TI = 5 /* aux[i]: mosrx_tcpinfo side arrays */,
       MOSRX_OP_TX_CHECKS = 6 /* out[i]: mosrx_tx_check records, `arg` the flags */ };
int  mosrx_time_op(mosrx_ctx *c, int op, int arg, const mosrx_batch *b, uint32_t nb, void *const *out,
                   void *const *aux, uint32_t iters, uint32_t nstreams, float *total_ms, float *avg_kernel_ms);
/* The kernel's own duration, averaged over `iters` back-to-back launches on
 * the context stream: each launch carries a start / stop event pair that the
 * dispatch itself stamps (hipExtLaunchKernel), so the gap between dispatches
 * is not counted -- the duration rocprofv3's kernel trace reports.  -ENOTSUP
 * for an operation that is not one kernel launch (the BPF rows). */
int  mosrx_time_op_dispatch(mosrx_ctx *c, int op, int arg, const mosrx_batch *b, uint32_t nb, void *const *out,
                            void *const *aux, uint32_t iters, float *avg_ms);
int  mosrx_time_queue_dispatch(mosrx_ctx *c, mosrx_queue *const *q, uint32_t nq, uint32_t iters, float *avg_ms);
/* The device's streaming-read ceiling: `iters` coalesced 16-byte-load passes
 * cycling over `nbuf` buffers of `bytes` each (sized past the 256 MiB Infinity
 * Cache), in GB/s.  The roofline figure next to the 8 TB/s spec peak. */
int  mosrx_probe_read_bw(mosrx_ctx *c, uint64_t bytes, uint32_t nbuf, uint32_t iters, float *gbps);
/* The stamp's own floor: the average dispatch-stamped duration (as
 * mosrx_time_op_dispatch measures it) of an empty kernel with the grid a
 * classify launch of `b` would have.  A short launch's stamped figure is
 * stated against it (the stamp reads ~4 us for a kernel that does nothing,
 * rocprofv3's trace 1.5-2.9 us).  Diagnostic; no mOS counterpart. */
int  mosrx_probe_stamp_floor(mosrx_ctx *c, const mosrx_batch *b, uint32_t iters, float *avg_ms);
/* hipDeviceSynchronize on the context's device. */
int  mosrx_device_sync(mosrx_ctx *c);
/* Same, end-to-end from host buffers through pinned staging, double-buffered. */
int  mosrx_time_host(mosrx_ctx *c, const mosrx_batch *b, uint32_t nb,
                     mosrx_result *const *h_out, uint32_t iters, float *ms);

/* ---- batched BPF ---------------------------------------- */
/* mOS evaluates classic-BPF programs per frame: raw-monitor filters on the
 * whole frame (ip_in.c:56-63) and stream SYN / orphan filters on the IP
 * datagram (tcp.c:42-56, 486-496), each through EVAL_BPFFILTER ->
 * sfbpf_filter(insns, p, len, len) (include/bpf/sfbpf.h:84,
 * bpf/sf_bpf_filter.c:214-536).  Programs still come from mOS's own compiler
 * (SET_BPFFILTER -> sfbpf_compile, sfbpf.h:83); the GPU runs the batched
 * evaluation of up to 32 of them over a batch and returns one match bitmask
 * per frame. */
typedef struct mosrx_bpf_insn {   /* layout of struct sfbpf_insn (include/bpf/sfbpf.h:174-179) */
	uint16_t code;
	uint8_t  jt;
	uint8_t  jf;
	uint32_t k;
} mosrx_bpf_insn;

enum {
	MOSRX_BPF_LEN_FRAME = 0,  /* wirelen = buflen = caplen (raw monitor: ethh, eth_len) */
	MOSRX_BPF_LEN_IP    = 1,  /* wirelen = buflen = 14 + ip tot_len (SYN/orphan filters);
	                           * evaluated on IPv4 frames whose datagram lies inside caplen, else 0 */
};
#define MOSRX_BPF_MAX_PROGS 32
#define MOSRX_BPF_MAX_INSNS 4096   /* total over all programs of a set */

typedef struct mosrx_bpf_prog {
	const mosrx_bpf_insn *insns;   /* NULL or len 0: no filter, matches every frame (sfbpf_filter(NULL) = ~0) */
	uint32_t              len;     /* bf_len */
	int32_t               len_mode;/* MOSRX_BPF_LEN_* */
} mosrx_bpf_prog;

/* The admission check of mosrx_bpf_set for one program (no GPU needed):
 * 0 or -EINVAL.  Besides sfbpf_validate's rules it rejects the absolute word /
 * halfword loads whose offset wraps sfbpf_filter's int bounds check (k of
 * 0xFFFFFFFC.. for a word, 0xFFFFFFFE.. for a halfword: the reference reads
 * before the frame).  The indexed loads cannot be checked at set time: where
 * X + k wraps into those ranges the reference reads before the frame
 * (undefined) and the GPU returns 0, as sfbpf_filter does for every other
 * out-of-bounds offset. */
int  mosrx_bpf_check(const mosrx_bpf_insn *insns, uint32_t len);
/* Install a program set on the context (host arrays, copied).  Each program
 * must pass sfbpf_validate (sf_bpf_filter.c:548-691) and, beyond it, use only
 * opcodes sfbpf_filter executes (others abort() there) with jump targets that
 * stay forward in 64-bit pointer arithmetic; otherwise -EINVAL, as
 * SET_BPFFILTER failing makes mtcp_bind_monitor_filter return EINVAL
 * (mos_api.c:127-155).  nprog = 0 clears the set. */
int  mosrx_bpf_set(mosrx_ctx *c, const mosrx_bpf_prog *progs, uint32_t nprog);
/* The same without waiting for the compiled form: the set is admitted,
 * staged and in effect when this returns (microseconds; no device-wide
 * synchronisation), evaluated by the interpreter kernel until the context's
 * compile thread has built and loaded its kernels with hipRTC, which replace
 * it at the next launch (a set seen before is taken from the cache at once).
 * Results are the same on either engine.  mosrx_bpf_wait blocks until the
 * installed set's compiled form is in (or failed: the interpreter stays);
 * mosrx_bpf_pending is 1 while its compile is outstanding. */
int  mosrx_bpf_set_async(mosrx_ctx *c, const mosrx_bpf_prog *progs, uint32_t nprog);
int  mosrx_bpf_wait(mosrx_ctx *c);
int  mosrx_bpf_pending(mosrx_ctx *c);
/* Evaluation engine of the next mosrx_bpf_set.  JIT (default): the set is
 * translated to one straight-line gfx950 kernel and compiled with hipRTC at
 * set time (cached per context); INTERP: the uniform-pc interpreter kernel.
 * Both run on the GPU with the same results; env MOSRX_BPF_ENGINE=0 selects
 * INTERP at open.  mosrx_bpf_engine() reports the engine of the installed set
 * (INTERP when the JIT could not compile; mosrx_bpf_jit_log() says why). */
enum { MOSRX_BPF_ENGINE_INTERP = 0, MOSRX_BPF_ENGINE_JIT = 1 };
int  mosrx_bpf_set_engine(mosrx_ctx *c, int engine);
int  mosrx_bpf_engine(const mosrx_ctx *c);
const char *mosrx_bpf_jit_log(const mosrx_ctx *c);
/* The generated kernel source of a program set (no GPU needed; free() it). */
int  mosrx_bpf_jit_source(const mosrx_bpf_prog *progs, uint32_t nprog, char **src);
/* The generated hook of the fused classify + BPF kernel: the set as the
 * device function the header wave calls on its window (free() it). */
int  mosrx_bpf_jit_hook_source(const mosrx_bpf_prog *progs, uint32_t nprog, char **src);
/* Generate and compile a program set with hipRTC for gfx950 without loading
 * it (no GPU needed): 0 and the code-object size, or -errno and the log. */
int  mosrx_bpf_jit_compile(const mosrx_bpf_prog *progs, uint32_t nprog, char *log, size_t logsz,
                           size_t *code_size);
/* Same for the fused classify + BPF kernel (the set inlined into the
 * classification kernel's header wave). */
int  mosrx_bpf_jit_compile_fused(const mosrx_bpf_prog *progs, uint32_t nprog, char *log, size_t logsz,
                                 size_t *code_size);
/* Classification (as mosrx_classify_dev) and the installed BPF set (as
 * mosrx_bpf_dev) in ONE pass over the frames: with the JIT engine the set is
 * compiled into the classify kernel, whose header wave evaluates it on the
 * bytes it already holds; otherwise two launches, same results.
 * mosrx_bpf_fused() = 1 when the installed set has the fused kernel. */
int  mosrx_classify_bpf_dev(mosrx_ctx *c, const mosrx_batch *b, mosrx_result *d_out, uint32_t *d_match,
                            void *stream);
int  mosrx_bpf_fused(const mosrx_ctx *c);
/* The same from host memory: H2D, the one-pass kernel, D2H of records and
 * masks (blocking, or submit/wait on a pipeline slot like mosrx_classify_host). */
int  mosrx_classify_bpf_host(mosrx_ctx *c, const mosrx_batch *b, mosrx_result *h_out, uint32_t *h_match);
int  mosrx_classify_bpf_host_submit(mosrx_ctx *c, int slot, const mosrx_batch *b, mosrx_result *h_out,
                                    uint32_t *h_match);
/* Device-resident evaluation: d_match[i] bit j = (sfbpf_filter(prog j, frame i) != 0). */
int  mosrx_bpf_dev(mosrx_ctx *c, const mosrx_batch *b, uint32_t *d_match, void *stream);
/* End-to-end from host memory (blocking). */
int  mosrx_bpf_host(mosrx_ctx *c, const mosrx_batch *b, uint32_t *h_match);

/* ---- TX checksum generation ---------------------------- */
/* The checksum rewrite mOS applies to a frame before it goes out again:
 * mtcp_setlastpkt with MOS_UPDATE_IP_CHKSUM / MOS_UPDATE_TCP_CHKSUM
 * (mos_api.c:1177-1193): iph->check = 0, iph->check = ip_fast_csum(iph, ihl);
 * tcph->check = 0, tcph->check = TCPCalcChecksum(tcph, tot_len - ihl*4, saddr,
 * daddr) -- the same arithmetic as the S/W fallback of ip_out.c:169-174 and
 * tcp_out.c:207-218.  Flags use mos_api.h:107-108's values.  Frames are
 * rewritten IN PLACE (b->frames is written through); frames must not overlap.
 * IP check: IPv4 frames with ihl >= 5 and the datagram inside the capture.
 * TCP check: those of them with protocol 6 and tot_len >= (ihl + doff) * 4.
 * Other frames are left untouched. */
#define MOSRX_TX_IP_CSUM  (1 << 4)   /* MOS_UPDATE_IP_CHKSUM */
#define MOSRX_TX_TCP_CSUM (1 << 5)   /* MOS_UPDATE_TCP_CHKSUM */
int  mosrx_tx_csum_dev(mosrx_ctx *c, const mosrx_batch *b, int flags, void *stream);
/* The same checks without touching the frames: one 8-byte record per frame
 * into d_checks (8-byte aligned, b->n of them).  `what` bit 0: ip_check is the
 * frame's new iph->check (little-endian u16 at frame byte 24), bit 1:
 * tcp_check its new tcph->check (at frame byte 14 + 4 * ihl + 16); frames the
 * rewrite would leave untouched have what = 0.  For a consumer that writes
 * the words itself (mosrx_tx_csum_host does, on the host).  Same checks as
 * mtcp_setlastpkt's MOS_UPDATE_IP_CHKSUM / MOS_UPDATE_TCP_CHKSUM
 * (core/src/mos_api.c:1177-1193) and the S/W paths of ip_out.c:169-174,
 * tcp_out.c:207-218. */
typedef struct mosrx_tx_check {
	uint16_t ip_check;
	uint16_t tcp_check;
	uint8_t  what;
	uint8_t  ihl;
	uint16_t pad;
} mosrx_tx_check;
int  mosrx_tx_csum_dev_checks(mosrx_ctx *c, const mosrx_batch *b, int flags, mosrx_tx_check *d_checks,
                              void *stream);
/* End-to-end from host memory (blocking): the frames cross PCIe once, the
 * check records come back and are written into b->frames. */
int  mosrx_tx_csum_host(mosrx_ctx *c, const mosrx_batch *b, int flags);

/* ---- RSS helpers (host-side table build; the hash itself runs on the GPU) -- */
/* Toeplitz nibble tables: 24 tables x 16 u32 for the 12-byte tuple
 * saddr|daddr|sport|dport (wire order).  Built from the key cache of
 * BuildKeyCache (util.c:27-58). */
int  mosrx_rss_tables(const uint8_t *key, uint32_t key_len, uint32_t tables[24 * 16]);

int  mosrx_abi_version(void);
const char *mosrx_strerror(int err);

#ifdef __cplusplus
}
#endif
#endif /* MOSRX_H */
