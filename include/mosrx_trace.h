/*
 * mosrx_trace.h — seeded synthetic TCP/IPv4 traces for the BASELINE configs.
 *
 * Host-side input tooling (not on the classify path).  Generates packed batches
 * in the layout mosrx_classify_* consumes: each frame at a 16-byte boundary + 2.
 * Content follows BASELINE.md §3: splitmix64 seeded with 0x6D4F5321 + config
 * index, valid checksums except a deterministic 1/1024 with a corrupted IP
 * checksum and 1/1024 with a corrupted TCP checksum, TTL 64, DF, IP id = index,
 * TCP seq advancing per flow, SYN on a flow's first packet, ACK otherwise.
 */
#ifndef MOSRX_TRACE_H
#define MOSRX_TRACE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum {
	MOSRX_TRACE_FW64  = 0,  /* config #1: simple_firewall, 10k x 64 B, one flow */
	MOSRX_TRACE_S64   = 1,  /* config #2: 64 B (caplen 60), one flow 10.0.0.1:1234 -> 10.0.0.2:80 */
	MOSRX_TRACE_M1500 = 2,  /* config #3: 1500 B MTU (caplen 1514, doff 8), 1M flows */
	MOSRX_TRACE_IMIX  = 3,  /* config #4/#5: 60/590/1514 in 7:4:1, shuffled, 1M flows */
};

#define MOSRX_TRACE_SEED 0x6D4F5321ull

typedef struct mosrx_trace {
	uint8_t  *frames;        /* malloc'd, frames_bytes + 64 zero bytes of padding */
	uint64_t  frames_bytes;
	uint32_t *off;
	uint16_t *len;
	uint32_t  n;
	uint32_t  max_len;
	uint64_t  caplen_sum;    /* sum of len[] (algorithmic frame bytes) */
} mosrx_trace;

/* n frames of `kind`; nflows distinct 4-tuples (ignored for the one-flow kinds);
 * seed 0 selects MOSRX_TRACE_SEED + kind.  Returns 0 or -errno. */
int  mosrx_trace_gen(int kind, uint32_t n, uint32_t nflows, uint64_t seed, mosrx_trace *out);
void mosrx_trace_free(mosrx_trace *t);

#ifdef __cplusplus
}
#endif
#endif
