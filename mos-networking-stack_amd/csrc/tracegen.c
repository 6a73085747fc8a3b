/*
 * tracegen.c — seeded synthetic traces (include/mosrx_trace.h).
 *
 * Builds frames the way a sender's stack would (checksums generated, not
 * verified), so the classifier has realistic input: the IPv4 header checksum
 * as in ip_out.c:169-174 and the TCP checksum over pseudo-header + segment as
 * in tcp_out.c:207-218.  Not on the classify path.
 */
#include <errno.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/mosrx_trace.h"

static inline uint64_t splitmix64(uint64_t *s)
{
	uint64_t z = (*s += 0x9E3779B97F4A7C15ull);
	z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
	z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
	return z ^ (z >> 31);
}

/* bijective 32-bit mixer (murmur3 finaliser): distinct flow index -> distinct saddr */
static inline uint32_t mix32(uint32_t x)
{
	x ^= x >> 16; x *= 0x85EBCA6Bu;
	x ^= x >> 13; x *= 0xC2B2AE35u;
	x ^= x >> 16;
	return x;
}

static inline void put16(uint8_t *p, uint32_t v) { p[0] = (uint8_t)(v >> 8); p[1] = (uint8_t)v; }
static inline void put32(uint8_t *p, uint32_t v)
{
	p[0] = (uint8_t)(v >> 24); p[1] = (uint8_t)(v >> 16); p[2] = (uint8_t)(v >> 8); p[3] = (uint8_t)v;
}

/* one's-complement sum of big-endian 16-bit words */
static uint32_t ocsum(const uint8_t *p, uint32_t n, uint32_t s)
{
	uint32_t i;
	for (i = 0; i + 1 < n; i += 2)
		s += ((uint32_t)p[i] << 8) | p[i + 1];
	if (n & 1)
		s += (uint32_t)p[n - 1] << 8;
	return s;
}

static uint16_t fold_not(uint32_t s)
{
	while (s >> 16)
		s = (s & 0xFFFF) + (s >> 16);
	return (uint16_t)~s;
}

struct flow { uint32_t sip, dip, seq, ack; uint16_t sp, dp; uint8_t started; };

/* size classes: caplen, tot_len, doff */
static const uint32_t cls_cap[3] = {60, 590, 1514};
static const uint32_t cls_tot[3] = {46, 576, 1500};
static const uint32_t cls_doff[3] = {5, 8, 8};

static void build_frame(uint8_t *f, int cls, struct flow *fl, uint32_t idx, uint64_t *rng)
{
	const uint32_t cap = cls_cap[cls], tot = cls_tot[cls], doff = cls_doff[cls];
	uint8_t *ip = f + 14, *tcp = ip + 20;
	const uint32_t seglen = tot - 20, paylen = seglen - doff * 4;
	uint32_t i, s;
	uint64_t r;

	/* Ethernet */
	memcpy(f, "\x02\x00\x00\x00\x00\x02\x02\x00\x00\x00\x00\x01\x08\x00", 14);
	/* IPv4 */
	ip[0] = 0x45; ip[1] = 0;
	put16(ip + 2, tot);
	put16(ip + 4, idx & 0xFFFF);
	put16(ip + 6, 0x4000);           /* DF */
	ip[8] = 64; ip[9] = 6;
	put16(ip + 10, 0);
	put32(ip + 12, fl->sip);
	put32(ip + 16, fl->dip);
	put16(ip + 10, fold_not(ocsum(ip, 20, 0)));
	/* TCP */
	put16(tcp, fl->sp);
	put16(tcp + 2, fl->dp);
	put32(tcp + 4, fl->seq);
	put32(tcp + 8, fl->ack);
	tcp[12] = (uint8_t)(doff << 4);
	tcp[13] = fl->started ? 0x10 : 0x02;   /* SYN first, then ACK */
	r = splitmix64(rng);
	put16(tcp + 14, (uint32_t)(r & 0xFFFF) | 0x0400);
	put16(tcp + 16, 0);
	put16(tcp + 18, 0);
	if (doff == 8) {                       /* NOP, NOP, timestamp */
		tcp[20] = 1; tcp[21] = 1; tcp[22] = 8; tcp[23] = 10;
		put32(tcp + 24, (uint32_t)(r >> 16));
		put32(tcp + 28, (uint32_t)(r >> 40) * 977u);
	}
	for (i = 0; i < paylen; i += 8) {
		uint64_t v = splitmix64(rng);
		uint32_t k;
		for (k = 0; k < 8 && i + k < paylen; k++)
			tcp[doff * 4 + i + k] = (uint8_t)(v >> (8 * k));
	}
	/* pseudo header: saddr, daddr, zero, proto, tcp length */
	s = ocsum(ip + 12, 8, 0) + 6 + seglen;
	put16(tcp + 16, fold_not(ocsum(tcp, seglen, s)));
	/* deterministic corruption: 1/1024 IP, 1/1024 TCP */
	if ((idx & 1023) == 511)
		ip[10] ^= 0x01;
	if ((idx & 1023) == 1023)
		tcp[17] ^= 0x01;
	/* Ethernet padding beyond tot_len stays zero */
	memset(f + 14 + tot, 0, cap - 14 - tot);
	fl->seq += paylen ? paylen : 1;
	fl->started = 1;
}

int mosrx_trace_gen(int kind, uint32_t n, uint32_t nflows, uint64_t seed, mosrx_trace *out)
{
	uint64_t rng, pos = 2, sum = 0;
	uint8_t *cls;
	struct flow *flows;
	uint32_t i, nf, maxl = 0;

	if (!out || kind < MOSRX_TRACE_FW64 || kind > MOSRX_TRACE_IMIX)
		return -EINVAL;
	memset(out, 0, sizeof(*out));
	rng = seed ? seed : MOSRX_TRACE_SEED + (uint64_t)kind;
	nf = (kind == MOSRX_TRACE_FW64 || kind == MOSRX_TRACE_S64) ? 1 : (nflows ? nflows : 1000000u);

	cls = malloc(n ? n : 1);
	out->off = malloc((size_t)(n ? n : 1) * 4);
	out->len = malloc((size_t)(n ? n : 1) * 2);
	flows = calloc(nf, sizeof(*flows));
	if (!cls || !out->off || !out->len || !flows)
		goto nomem;

	/* size classes (IMIX: each group of 12 holds 7x60, 4x590, 1x1514, shuffled) */
	for (i = 0; i < n; i++)
		cls[i] = kind == MOSRX_TRACE_M1500 ? 2 : 0;
	if (kind == MOSRX_TRACE_IMIX) {
		for (i = 0; i < n; i += 12) {
			uint8_t g[12] = {0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2};
			int k;
			for (k = 11; k > 0; k--) {
				int j = (int)(splitmix64(&rng) % (uint64_t)(k + 1));
				uint8_t tmp = g[k]; g[k] = g[j]; g[j] = tmp;
			}
			for (k = 0; k < 12 && i + k < n; k++)
				cls[i + k] = g[k];
		}
	}
	/* layout: frame i at 16-byte boundary + 2 */
	for (i = 0; i < n; i++) {
		uint32_t cap = cls_cap[cls[i]];
		out->off[i] = (uint32_t)pos;
		out->len[i] = (uint16_t)cap;
		sum += cap;
		if (cap > maxl)
			maxl = cap;
		pos = ((pos + cap - 2 + 15) & ~15ull) + 2;
	}
	out->frames_bytes = pos;
	if (pos >= (1ull << 32))
		goto toobig;
	out->frames = calloc(pos + 64, 1);
	if (!out->frames)
		goto nomem;

	/* flows */
	if (nf == 1) {
		flows[0].sip = 0x0A000001; flows[0].dip = 0x0A000002;
		flows[0].sp = 1234; flows[0].dp = 80;
		flows[0].seq = (uint32_t)splitmix64(&rng);
		flows[0].ack = (uint32_t)splitmix64(&rng);
	} else {
		uint32_t salt = (uint32_t)splitmix64(&rng);
		for (i = 0; i < nf; i++) {
			uint64_t r = splitmix64(&rng);
			flows[i].sip = mix32(i ^ salt);
			flows[i].dip = (uint32_t)r;
			flows[i].sp = (uint16_t)(r >> 32);
			flows[i].dp = (uint16_t)(r >> 48);
			flows[i].seq = (uint32_t)splitmix64(&rng);
			flows[i].ack = (uint32_t)(r >> 16);
		}
	}
	for (i = 0; i < n; i++) {
		uint32_t fi = nf == 1 ? 0 : (uint32_t)(splitmix64(&rng) % nf);
		build_frame(out->frames + out->off[i], cls[i], &flows[fi], i, &rng);
	}
	out->n = n;
	out->max_len = maxl;
	out->caplen_sum = sum;
	free(cls);
	free(flows);
	return 0;
toobig:
	free(cls);
	free(flows);
	mosrx_trace_free(out);
	return -E2BIG;
nomem:
	free(cls);
	free(flows);
	mosrx_trace_free(out);
	return -ENOMEM;
}

void mosrx_trace_free(mosrx_trace *t)
{
	if (!t)
		return;
	free(t->frames);
	free(t->off);
	free(t->len);
	memset(t, 0, sizeof(*t));
}
