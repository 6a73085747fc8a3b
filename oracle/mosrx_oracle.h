/*
 * mosrx_oracle.h — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of mOS's receive-path per-packet transform, used as the
 * parity checker for the HIP path and as the CPU baseline in bench.py.  Only
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it.
 * The product library (libmosrx.so) never links or calls this code.
 *
 * Parity of this restatement is pinned against the reference itself: the
 * recipe in oracle/ref.mk compiles mOS's own core/src objects into
 * oracle/_ref/mosref, and tests/golden/ holds the vectors it produced
 * (tests/golden/make_golden.py), plus the MSDN Toeplitz KAT of util/rss.c:177-193.
 */
#ifndef MOSRX_ORACLE_H
#define MOSRX_ORACLE_H

#include <stdint.h>
#include "../include/mosrx.h"

#ifdef __cplusplus
extern "C" {
#endif

/* ip_fast_csum, core/src/include/ip_in.h:10-38 (x86 asm restated). */
uint16_t mo_ip_fast_csum(const uint8_t *iph, unsigned ihl);
/* TCPCalcChecksum, core/src/tcp_util.c:157-190.  saddr/daddr are the raw
 * network-order words as loaded on little-endian x86. */
uint16_t mo_tcp_csum(const uint8_t *seg, uint16_t len, uint32_t saddr, uint32_t daddr);
/* BuildKeyCache, core/src/util.c:27-58 (96 entries). */
void     mo_rss_key_cache(const uint8_t *key, uint32_t cache[96]);
/* GetRSSHash, core/src/util.c:61-99 (host-order arguments). */
uint32_t mo_rss_hash(const uint32_t cache[96], uint32_t sip, uint32_t dip, uint16_t sp, uint16_t dp);
/* GetRSSCPUCore, core/src/util.c:114-131, with FetchEndianType() == mode. */
int      mo_rss_queue(uint32_t hash, int mode, int num_queues);

/* SuperFastHash, core/src/fhash.c:25-69. */
uint32_t mo_superfasthash(const uint8_t *data, int len);
/* HashFlow of FindStream's reversed tuple (tcp.c:185-190, fhash.c:72-92), full
 * 32 bits; bucket = value & 0x1FFFF (NUM_BINS, fhash.h:7). */
uint32_t mo_flow_hash(const uint8_t *iph, const uint8_t *tcph);
/* mo_classify + the flow hash per frame (0 unless a TCP frame with header fields). */
int mo_classify_fh(const mosrx_params *p, const uint8_t *frames, uint64_t frames_bytes, const uint32_t *off,
                   const uint16_t *len, uint32_t n, mosrx_result *out, uint32_t *fhash);

/* mo_classify + both optional side arrays of mosrx_classify_dev_ex (either may
 * be NULL): the flow hash and pkt_info's TCP fields as FillPacketContextTCPInfo
 * (tcp.c:258-270) sets them, zero where payload_off == 0. */
int mo_classify_ex(const mosrx_params *p, const uint8_t *frames, uint64_t frames_bytes, const uint32_t *off,
                   const uint16_t *len, uint32_t n, mosrx_result *out, uint32_t *fhash, mosrx_tcpinfo *tinfo);

/* sfbpf_filter (bpf/sf_bpf_filter.c:214-536) and sfbpf_validate (:548-691). */
uint32_t mo_bpf_filter(const mosrx_bpf_insn *pc, const uint8_t *p, uint32_t wirelen, uint32_t buflen);
int      mo_bpf_validate(const mosrx_bpf_insn *f, int len);
/* One program's return value on every frame at a call-site length (0 where not evaluated). */
int      mo_bpf_returns(const mosrx_bpf_insn *insns, uint32_t ninsn, int len_mode, const uint8_t *frames,
                        uint64_t frames_bytes, const uint32_t *off, const uint16_t *len, uint32_t n, uint32_t *ret);
/* Batched: out[i] bit j = program j matched frame i (lengths per MOSRX_BPF_LEN_*). */
int      mo_bpf_eval(const mosrx_bpf_prog *progs, uint32_t nprog, const uint8_t *frames, uint64_t frames_bytes,
                     const uint32_t *off, const uint16_t *len, uint32_t n, uint32_t *out);

/* TX checksum rewrite of mosrx_tx_csum_dev (mos_api.c:1177-1193), in place. */
int mo_tx_csum(uint8_t *frames, uint64_t frames_bytes, const uint32_t *off, const uint16_t *len, uint32_t n,
               int flags);

/* ProcessPacket (eth_in.c:27-87) through the TCP prefix (tcp.c:408-445) plus
 * the RSS hash/queue, for one frame.  Fills all 16 bytes of *r. */
void mo_classify_one(const mosrx_params *p, const uint32_t cache[96],
                     const uint8_t *frame, uint32_t caplen, mosrx_result *r);

/* Batch form on host memory (frames + off/len as in mosrx_batch). */
int mo_classify(const mosrx_params *p, const uint8_t *frames, uint64_t frames_bytes,
                const uint32_t *off, const uint16_t *len, uint32_t n, mosrx_result *out);

/* Same, split over `nthreads` pthreads on disjoint slices (mirrors mOS per-core
 * sharding, core.c:1369-1466).  Used for the all-cores CPU baseline. */
int mo_classify_mt(const mosrx_params *p, const uint8_t *frames, uint64_t frames_bytes,
                   const uint32_t *off, const uint16_t *len, uint32_t n, mosrx_result *out,
                   int nthreads);

/* Defaults identical to mosrx_params_default() (simple_firewall state). */
void mo_params_default(mosrx_params *p);

#ifdef __cplusplus
}
#endif
#endif
