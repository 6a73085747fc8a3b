/*
 * mosrx_mos_rx.h — mOS's per-frame receive step driven by the GPU records.
 *
 * mosrx_mos_process_packet() has ProcessPacket's signature and return value
 * (core/src/include/eth_in.h:7, eth_in.c:27-87) and is the call RunMainLoop
 * makes per received frame (core.c:902-907) in an mOS build whose I/O module
 * is gpu_module_func.  It does not re-run the checks the GPU made for the
 * batch: ethertype / IP header checks (eth_in.c:56-78, ip_in.c:39-51),
 * ip_fast_csum (ip_in.h:10-38, ip_in.c:74-77), the TCP length check and
 * TCPCalcChecksum (tcp.c:429-444), the raw-monitor and stream SYN / orphan BPF
 * filters (ip_in.c:56-63, tcp.c:42-56, :486-496).  It takes the frame's
 * record (dev_ioctl(MOSRX_PKT_RX_RESULTS), reason code + header fields) and
 * the filters' match masks (MOSRX_PKT_RX_MATCH), and performs every side
 * effect ProcessPacket performs for that outcome, in the same order: NETSTAT
 * (eth_in.c:42-45, 80-84), ProcessARPPacket / DumpPacket / release_pkt,
 * ForwardEthernetFrame / ForwardIPPacket, ProcessICMPPacket, the raw-monitor
 * MOS_ON_PKT_IN callbacks (ip_in.c:56-63, tcp.c:424-427), and the stream
 * step after the checks (tcp.c:445-514: FindStream, CreateStream with the
 * SYN filters, HandleSockStream / HandleMonitorStream, the orphan callbacks,
 * the RST of an end host or the forward of a monitor).
 *
 * Integration: at core.c:906 the rx loop calls mosrx_mos_process_packet
 * instead of ProcessPacket (same arguments).  Compile csrc/mos_rx.c inside
 * mOS's tree with -DMOSRX_HAVE_MOS_IO_MODULE (-I core/src/include
 * -I core/src/include/bpf), next to gpu_module.c.
 *
 * Freshness: a batch's records were made under the socket counts mOS had when
 * it was classified; ProcessPacket reads them live per frame.  When a monitor
 * or end-host socket appears or goes away so that checksum verification turns
 * on or off (ip_in.c:67) in the middle of a batch, the backend classifies the
 * rest of the batch again under the new counts (MOSRX_PKT_RX_RECLASSIFY)
 * before the next frame is taken.  When a monitor binds a filter the GPU does
 * not hold yet, the monitors' filters are installed on every netdev
 * (MOSRX_PKT_SET_BPF, bit j = filter j) and the batch classified again.
 * Filters past the 32 the GPU evaluates in one pass are evaluated by mOS's
 * own EVAL_BPFFILTER.  Filters are known by their instructions (a closed
 * monitor's program can be freed and another's allocated at its address), and
 * the installed set is checked against the monitors' at every batch start.
 *
 * GPU errors: a batch whose records cannot be had (a failed reclassification,
 * no records handed out) loses its remaining frames -- counted in rx_packets
 * and rx_errors, released, -1 -- and mOS runs on (gpu_errors / gpu_dropped).
 */
#ifndef MOSRX_MOS_RX_H
#define MOSRX_MOS_RX_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

struct mtcp_manager;

int mosrx_mos_process_packet(struct mtcp_manager *mtcp, const int ifidx, const int index, uint32_t cur_ts,
                             unsigned char *pkt_data, int len);

typedef struct mosrx_mos_rx_stats {
	uint64_t frames;            /* frames taken from records */
	uint64_t stream_step;       /* of them, TCP segments that entered the stream step (tcp.c:445) */
	uint64_t gpu_flow_hash;     /* of those, flow-table lookups on the GPU's bucket (cfg.flowhash) */
	uint64_t reclassified;      /* batches classified again mid-batch (state / filter change) */
	uint64_t filter_installs;   /* BPF sets installed on the GPU */
	uint64_t filters_gpu;       /* filters in the installed set */
	uint64_t filters_cpu;       /* filters evaluated by mOS's EVAL_BPFFILTER (past the GPU's 32) */
	uint64_t max_filter_sync_ns;/* longest filter install (the rx loop's stall: set + reclassify) */
	uint64_t gpu_errors;        /* batches (or their rest) left without records: the backend failed */
	uint64_t gpu_dropped;       /* frames of those batches, dropped and counted in rx_errors */
	uint64_t batches_c8;        /* batch record sets read in the 8-byte form (cfg.compact) */
} mosrx_mos_rx_stats;

/* Counters of the mTCP thread running core `cpu` (mtcp->ctx->cpu). */
int mosrx_mos_rx_stats_of(int cpu, mosrx_mos_rx_stats *st);

#ifdef __cplusplus
}
#endif
#endif
