/*
 * mosrx_internal.h — shared between the C host library (mosrx_api.c) and the
 * HIP kernels (mosrx_kernels.hip).  Plain C layout, no HIP types except the
 * launcher's stream argument.
 */
#ifndef MOSRX_INTERNAL_H
#define MOSRX_INTERNAL_H

#include "../../include/mosrx.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Device-side lookup tables, one block per context:
 *   [0, 384)   Toeplitz nibble tables, 24 x 16 u32 (mosrx_rss_tables)
 *   [384, 512) GetRSSCPUCore queue LUT, 512 x u8 indexed by (rss & 0x1FF)
 *   (the first MOSRX_TAB_WORDS are staged in LDS by every header wave)
 *   [512]      number of local addresses, [513, 529) the addresses (read with
 *              scalar loads by waves that hold an ICMP frame) */
#define MOSRX_TAB_RSS_WORDS   384
#define MOSRX_TAB_QLUT_WORDS  128
#define MOSRX_TAB_WORDS       512
#define MOSRX_TAB_LOCAL       512
#define MOSRX_TAB_ALLOC_WORDS (MOSRX_TAB_LOCAL + 1 + MOSRX_MAX_LOCAL)

enum {
	MOSRX_KF_VERIFY    = 1u << 0,  /* num_msp || num_esp: checksums verified (ip_in.c:67) */
	MOSRX_KF_FWD_NONIP = 1u << 1,  /* num_msp && forward: non-IPv4 frames forwarded (eth_in.c:62) */
	MOSRX_KF_SKIP_TCP  = 1u << 2,  /* skip TCPCalcChecksum (BASELINE config #2 mode) */
	MOSRX_KF_TX_IP     = 1u << 3,  /* TX fill: write iph->check (no records) */
	MOSRX_KF_TX_TCP    = 1u << 4,  /* TX fill: write tcph->check (no records) */
	MOSRX_KF_COMPACT   = 1u << 5,  /* host side only: 8-byte records (mosrx_result8) */
};

typedef struct mosrx_kparams {
	const uint8_t  *frames;
	const uint32_t *off;
	const uint16_t *len;
	mosrx_result   *out;
	const uint32_t *tables;     /* MOSRX_TAB_WORDS */
	uint32_t       *counters;   /* MOSRX_CNT_SHARDS x MOSRX_CNT_STRIDE u32 (reason counts, summed over shards
	                             * by the host), accumulated with atomics; may be NULL */
	uint32_t       *fhash;      /* n flow hashes (HashFlow before the NUM_BINS mask); may be NULL */
	uint32_t       *bmatch;     /* fused BPF match masks (hipRTC-built kernels only); else NULL */
	mosrx_tcpinfo  *tinfo;      /* n pkt_info TCP field records; may be NULL */
	uint32_t        frames_bytes;
	uint32_t        n;
	uint32_t        flags;      /* MOSRX_KF_* */
	uint32_t        uni;        /* layout hint (mosrx_uni_pack): frame i expected at (uni >> 16) + i * (uni & 0xFFFF);
	                             * 0 = none.  Read by the SMALL tile's VAR_UNI kernels only */
} mosrx_kparams;

/* Launches of at most this many workgroups take the SMALL tile's hinted forms
 * (VAR_UNI): one round of resident workgroups, latency-bound, where the
 * descriptor -> window round trip is the launch's critical path (config #2's
 * single 32K batch: 128 workgroups).  Larger launches keep the plain forms:
 * with every slot busy the round trip is hidden, and the hinted form measured
 * 1-2.5 % slower on the 64 B rings (profiles/r05/hint_ab). */
#define MOSRX_UNI_MAX_TILES 2048u

/* The uniform-layout hint of a batch (MOSRX_BATCH_UNIFORM, include/mosrx.h) in
 * the 32 bits a kernel argument / queue descriptor carries: 0 when the batch
 * has none or its first offset or stride does not fit 16 bits (the kernels
 * then wait for the descriptors, as without a hint). */
static inline uint32_t mosrx_uni_pack(const mosrx_batch *b)
{
	if (!(b->layout & MOSRX_BATCH_UNIFORM) || b->stride == 0 || b->stride > 0xFFFFu || b->off0 > 0xFFFFu)
		return 0;
	return (b->off0 << 16) | b->stride;
}

/* Reason counters: workgroup b adds to shard b % MOSRX_CNT_SHARDS, one 64-byte line each */
#define MOSRX_CNT_SHARDS 256
#define MOSRX_CNT_STRIDE 16
#define MOSRX_CNT_WORDS  (MOSRX_CNT_SHARDS * MOSRX_CNT_STRIDE)

/* Kernel shapes ("kinds") the library builds:
 *   SMALL  256 frames / 4 waves, lane per frame, every frame fits the header
 *          window (the 64 B configs)
 *   S13     64 frames / 1 header wave + 3 streamer waves that read the tile's
 *          tail span in buffer order with a prefix scan (frames sorted and
 *          disjoint, checked per tile; unsorted tiles stream tail by tail)
 * Tuning shapes (LARGE, MID, L12/L24/L28, S12/S14/S16, the decoupled S13xN)
 * live in scripts/probe_*
 * (DESIGN.md §4.3 has their measurements). */
enum { MOSRX_KIND_SMALL = 0, MOSRX_KIND_S13 = 1, MOSRX_KIND_COUNT = 2 };
#define MOSRX_STREAMERS 3
#ifndef MOSRX_SMALL_FRAMES
#define MOSRX_SMALL_FRAMES 256u   /* 256 x frames per lane */
#endif
#define MOSRX_KIND_FRAMES(k) ((k) == MOSRX_KIND_SMALL ? MOSRX_SMALL_FRAMES : 64u)
/* Header windows.  Frames whose IP datagram ends at or before the window end
 * are finished in the per-lane header window; longer ones stream their tail
 * cooperatively from the first 16-byte boundary at or below it (the split).
 * The SMALL tile reads 5 chunks (frame bytes [2, 78): every 64-byte frame
 * ends inside), the stream tile 4 ([2, 62): the TCP header and the first
 * payload bytes); a wave holding a frame with IP options reads the full 6
 * ([2, 94)), whatever the tile. */
#define MOSRX_WINDOW_END_SMALL  78
#define MOSRX_WINDOW_END_STREAM 62
#define MOSRX_WINDOW_END_FULL   94

/* (mosrx_tx_check, include/mosrx.h: the TX rewrite's records when kp.out is set) */

/* Batch-queue descriptor (device resident), 64 bytes. */
typedef struct mosrx_qdesc {
	const uint8_t  *frames;
	const uint32_t *off;
	const uint16_t *len;
	mosrx_result   *out;         /* 16-byte records, or 8-byte ones (mosrx_result8) for a compact queue */
	union {
		mosrx_tcpinfo *tinfo;    /* the classify kernels: NULL unless launched with pkt_info fields */
		uint32_t      *bmatch;   /* the fused classify + BPF kernels (they write no pkt_info): match masks */
	};
	uint32_t       *fhash;       /* flow-table hashes, or NULL */
	uint32_t        frames_bytes;
	uint32_t        n;
	uint32_t        tile_base;   /* first workgroup of this batch in the launch */
	uint32_t        uni;         /* the batch's layout hint (mosrx_uni_pack), 0 = none */
} mosrx_qdesc;

typedef struct mosrx_qparams {
	const mosrx_qdesc *desc;     /* nb entries */
	const uint32_t    *tables;
	uint32_t          *counters;
	uint32_t           nb;
	uint32_t           flags;
	uint32_t           tpb;      /* tiles per batch when every batch has the same tile count, else 0 */
	uint32_t           tinfo;    /* 1: the descriptors carry pkt_info TCP field buffers (VAR_TI);
	                              * 2: the records are the 8-byte compact form (VAR_C8) */
	uint32_t           uni;      /* 1: some descriptor carries a layout hint (the SMALL tile's VAR_UNI forms) */
} mosrx_qparams;

/* Batched BPF launch: the program table rides in the kernel arguments, the
 * instructions sit in one device buffer read with scalar loads. */
typedef struct mosrx_bparams {
	const uint8_t        *frames;
	const uint32_t       *off;
	const uint16_t       *len;
	uint32_t             *match;
	const mosrx_bpf_insn *insns;      /* MOSRX_BPF_MAX_INSNS */
	uint32_t              frames_bytes;
	uint32_t              n;
	uint32_t              nprog;
	uint32_t              ip_mode;    /* bit j: program j uses MOSRX_BPF_LEN_IP */
	uint16_t              prog_off[MOSRX_BPF_MAX_PROGS];
	uint16_t              prog_len[MOSRX_BPF_MAX_PROGS];   /* 0: no filter (matches) */
} mosrx_bparams;

int mosrx_launch_bpf(const mosrx_bparams *bp, void *stream);

int mosrx_launch_queue(const mosrx_qparams *qp, uint32_t total_tiles, int tile, int variant, void *stream);
int mosrx_launch_read_bw(const void *p, uint64_t bytes, uint32_t *sink, void *stream);
int mosrx_launch_empty(int kind, uint32_t tiles, void *stream);

/* Launch one classify kernel; returns 0 or -EINVAL / -EIO.  `stream` is a hipStream_t. */
int mosrx_launch_classify(const mosrx_kparams *kp, int tile, int variant, void *stream);

/* Dispatch-stamped timing hooks (mosrx_kernels.hip): the next classify / queue
 * launch of the calling thread takes this start / stop event pair; the count
 * of launches made by the thread so far. */
void mosrx__stamp_next(void *start, void *stop);
uint32_t mosrx__launch_count(void);
/* A launch made outside mosrx_kernels.hip: counted, and the pending stamp
 * pair (1) or none (0) handed over for it. */
int mosrx__stamp_take(void **start, void **stop);

#ifdef __cplusplus
}
#endif
#endif
