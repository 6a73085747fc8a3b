/*
 * mosrx_oracle.c — TEST INFRASTRUCTURE ONLY (see mosrx_oracle.h).
 *
 * Plain-C restatement of the mOS receive path, frame at a time, written from
 * the reference's behaviour.  Every function names the reference lines it
 * restates.  Byte order: wire fields are big-endian; the reference loads
 * multi-byte words natively on little-endian x86, which this file reproduces
 * with explicit little-endian loads.
 */
#include "mosrx_oracle.h"

#include <errno.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

static inline uint32_t le32(const uint8_t *p)
{
	return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}
static inline uint16_t le16(const uint8_t *p) { return (uint16_t)(p[0] | (p[1] << 8)); }
static inline uint16_t be16(const uint8_t *p) { return (uint16_t)((p[0] << 8) | p[1]); }
static inline uint32_t be32(const uint8_t *p)
{
	return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | (uint32_t)p[3];
}

/* core/src/include/ip_in.h:10-38.  The asm keeps a 32-bit add-with-carry chain
 * over dwords 0..ihl-1 whose final carry is added once by `adcl $0` (a carry
 * out of that last add is lost), then folds with `addw` + `adcl $0` and
 * complements.  For ihl <= 4 `subl $4; jbe 2f` skips everything and the low
 * 16 bits of dword 0 come back un-complemented. */
uint16_t mo_ip_fast_csum(const uint8_t *iph, unsigned ihl)
{
	uint32_t sum = le32(iph);
	uint64_t t;
	uint32_t c;
	unsigned k;

	if (ihl <= 4)
		return (uint16_t)sum;
	t = (uint64_t)sum + le32(iph + 4);          sum = (uint32_t)t; c = (uint32_t)(t >> 32);
	t = (uint64_t)sum + le32(iph + 8) + c;      sum = (uint32_t)t; c = (uint32_t)(t >> 32);
	t = (uint64_t)sum + le32(iph + 12) + c;     sum = (uint32_t)t; c = (uint32_t)(t >> 32);
	for (k = 4; k < ihl; k++) {                 /* label 1: adcl 16(%1); dec keeps CF */
		t = (uint64_t)sum + le32(iph + 4 * k) + c;
		sum = (uint32_t)t; c = (uint32_t)(t >> 32);
	}
	sum += c;                                   /* adcl $0, %0 */
	{
		uint32_t a = (sum >> 16) + (sum & 0xFFFF); /* shrl $16; addw %w2,%w0 */
		uint32_t r = (a & 0xFFFF) + (a >> 16);     /* adcl $0, %0 */
		return (uint16_t)~r;                       /* notl; (__sum16) */
	}
}

/* core/src/tcp_util.c:157-190 */
uint16_t mo_tcp_csum(const uint8_t *seg, uint16_t len, uint32_t saddr, uint32_t daddr)
{
	uint32_t sum = 0;
	int nleft = len;
	const uint8_t *w = seg;

	while (nleft > 1) {
		sum += le16(w);
		w += 2;
		nleft -= 2;
	}
	if (nleft)                       /* *w & ntohs(0xFF00): first byte only */
		sum += w[0];
	sum += (saddr & 0x0000FFFF) + (saddr >> 16);
	sum += (daddr & 0x0000FFFF) + (daddr >> 16);
	sum += (uint16_t)((len >> 8) | (len << 8));   /* htons(len) */
	sum += 0x0600;                                /* htons(IPPROTO_TCP) */
	sum = (sum >> 16) + (sum & 0xFFFF);
	sum += (sum >> 16);
	sum = ~sum;
	return (uint16_t)sum;
}

/* core/src/util.c:27-58 with the key as a parameter (the reference hard-codes
 * 40 x 0x05; util/rss.c:73-90 holds the Microsoft key used by the KAT). */
void mo_rss_key_cache(const uint8_t *key, uint32_t cache[96])
{
	uint32_t result = ((uint32_t)key[0] << 24) | ((uint32_t)key[1] << 16) |
	                  ((uint32_t)key[2] << 8) | (uint32_t)key[3];
	uint32_t idx = 32;
	int i;

	for (i = 0; i < 96; i++, idx++) {
		uint8_t shift = idx % 8;
		uint32_t bit = ((key[idx / 8] << shift) & 0x80) ? 1 : 0;
		cache[i] = result;
		result = (result << 1) | bit;
	}
}

/* core/src/util.c:61-99 */
uint32_t mo_rss_hash(const uint32_t cache[96], uint32_t sip, uint32_t dip, uint16_t sp, uint16_t dp)
{
	uint32_t res = 0;
	int i;

	for (i = 0; i < 32; i++) {
		if (sip & 0x80000000u)
			res ^= cache[i];
		sip <<= 1;
	}
	for (i = 0; i < 32; i++) {
		if (dip & 0x80000000u)
			res ^= cache[32 + i];
		dip <<= 1;
	}
	for (i = 0; i < 16; i++) {
		if (sp & 0x8000)
			res ^= cache[64 + i];
		sp = (uint16_t)(sp << 1);
	}
	for (i = 0; i < 16; i++) {
		if (dp & 0x8000)
			res ^= cache[80 + i];
		dp = (uint16_t)(dp << 1);
	}
	return res;
}

/* core/src/util.c:114-131 */
int mo_rss_queue(uint32_t hash, int mode, int num_queues)
{
	static const uint32_t off[4] = {3, 1, (uint32_t)-1, (uint32_t)-3};
	uint32_t masked;

	if (mode) {
		masked = hash & 0x1FF;
		masked += off[masked & 0x3];
	} else {
		masked = hash & 0x7F;
	}
	return (int)(masked % (uint32_t)num_queues);
}

/* SuperFastHash, core/src/fhash.c:25-69 (get16bits = native little-endian
 * 16-bit load on x86; the tail bytes are `signed char`). */
uint32_t mo_superfasthash(const uint8_t *data, int len)
{
	uint32_t hash = (uint32_t)len, tmp;
	int rem;

	if (len <= 0 || data == NULL)
		return 0;
	rem = len & 3;
	len >>= 2;
	for (; len > 0; len--) {
		hash += le16(data);
		tmp = ((uint32_t)le16(data + 2) << 11) ^ hash;
		hash = (hash << 16) ^ tmp;
		data += 4;
		hash += hash >> 11;
	}
	switch (rem) {
	case 3:
		hash += le16(data);
		hash ^= hash << 16;
		hash ^= (uint32_t)((int32_t)(signed char)data[2] << 18);
		hash += hash >> 11;
		break;
	case 2:
		hash += le16(data);
		hash ^= hash << 11;
		hash += hash >> 17;
		break;
	case 1:
		hash += (uint32_t)(int32_t)(signed char)data[0];
		hash ^= hash << 10;
		hash += hash >> 1;
	}
	hash ^= hash << 3;
	hash += hash >> 5;
	hash ^= hash << 4;
	hash += hash >> 17;
	hash ^= hash << 25;
	hash += hash >> 6;
	return hash;
}

/* FindStream's key (tcp.c:185-190): the reversed tuple {daddr, saddr, dport,
 * sport} as stored in tcp_stream (network order, tcp_stream.h:239-242), hashed
 * by HashFlow (fhash.c:72-92); the flow-table bucket is hash & (NUM_BINS-1). */
uint32_t mo_flow_hash(const uint8_t *iph, const uint8_t *tcph)
{
	uint8_t key[12];
	memcpy(key, iph + 16, 4);      /* temp.saddr = iph->daddr */
	memcpy(key + 4, iph + 12, 4);  /* temp.daddr = iph->saddr */
	memcpy(key + 8, tcph + 2, 2);  /* temp.sport = tcph->dest */
	memcpy(key + 10, tcph, 2);     /* temp.dport = tcph->source */
	return mo_superfasthash(key, 12);
}

int mo_classify_ex(const mosrx_params *p, const uint8_t *frames, uint64_t frames_bytes, const uint32_t *off,
                   const uint16_t *len, uint32_t n, mosrx_result *out, uint32_t *fhash, mosrx_tcpinfo *tinfo)
{
	uint32_t i;
	int rc = mo_classify(p, frames, frames_bytes, off, len, n, out);
	if (rc || (!fhash && !tinfo))
		return rc;
	for (i = 0; i < n; i++) {
		/* defined for every TCP frame whose header fields are (payload_off != 0) */
		const uint8_t *iph = frames + off[i] + 14;
		const uint8_t *tcph = iph + (out[i].ihl_doff >> 4) * 4;
		if (fhash)
			fhash[i] = out[i].payload_off ? mo_flow_hash(iph, tcph) : 0;
		if (tinfo) {
			memset(&tinfo[i], 0, sizeof(tinfo[i]));
			if (out[i].payload_off) {   /* FillPacketContextTCPInfo, tcp.c:263-265 */
				tinfo[i].seq = be32(tcph + 4);
				tinfo[i].ack_seq = be32(tcph + 8);
				tinfo[i].window = be16(tcph + 14);
				tinfo[i].ip_len = be16(iph + 2);   /* FillInPacketIPContext, ip_in.c:21-27 */
			}
		}
	}
	return 0;
}

int mo_classify_fh(const mosrx_params *p, const uint8_t *frames, uint64_t frames_bytes, const uint32_t *off,
                   const uint16_t *len, uint32_t n, mosrx_result *out, uint32_t *fhash)
{
	return mo_classify_ex(p, frames, frames_bytes, off, len, n, out, fhash, NULL);
}

/* TX checksum rewrite, mtcp_setlastpkt's MOS_UPDATE_IP_CHKSUM /
 * MOS_UPDATE_TCP_CHKSUM branch (mos_api.c:1177-1193), IP first as there, on
 * the frames include/mosrx.h defines for mosrx_tx_csum_dev.  In place. */
int mo_tx_csum(uint8_t *frames, uint64_t frames_bytes, const uint32_t *off, const uint16_t *len, uint32_t n,
               int flags)
{
	uint32_t i;
	for (i = 0; i < n; i++) {
		uint8_t *f = frames + off[i], *iph = f + 14, *th;
		uint32_t cap = (off[i] >= frames_bytes) ? 0 : (uint32_t)(frames_bytes - off[i] < len[i] ? frames_bytes - off[i] : len[i]);
		unsigned ihl, ip_len, doff;
		uint32_t saddr, daddr;
		if (cap < 34 || f[12] != 0x08 || f[13] != 0x00)
			continue;
		ihl = iph[0] & 0xF;
		ip_len = be16(iph + 2);
		if (ihl < 5 || 14 + ihl * 4 > cap || 14 + ip_len > cap || (iph[9] == 6 && 14 + ihl * 4 + 20 > cap))
			continue;
		if (flags & MOSRX_TX_IP_CSUM) {
			uint16_t v;
			iph[10] = iph[11] = 0;
			v = mo_ip_fast_csum(iph, ihl);
			memcpy(iph + 10, &v, 2);
		}
		th = iph + ihl * 4;
		doff = th[12] >> 4;
		if ((flags & MOSRX_TX_TCP_CSUM) && iph[9] == 6 && ip_len >= (ihl + doff) * 4) {
			uint16_t v;
			memcpy(&saddr, iph + 12, 4);
			memcpy(&daddr, iph + 16, 4);
			th[16] = th[17] = 0;
			v = mo_tcp_csum(th, (uint16_t)(ip_len - ihl * 4), saddr, daddr);
			memcpy(th + 16, &v, 2);
		}
	}
	return 0;
}

void mo_params_default(mosrx_params *p)
{
	memset(p, 0, sizeof(*p));
	p->num_msp = 1;
	p->num_esp = 0;
	p->forward = 1;
	p->num_queues = 1;
	p->queue_mode = MOSRX_QMAP_I40E;
	p->skip_tcp_csum = 0;
	p->rss_key_len = 40;
	memset(p->rss_key, 0x05, 40);
}

#define VERDICT(rr, v, why) do { (rr)->verdict = (int8_t)(v); (rr)->reason = (uint8_t)(why); } while (0)

/* ProcessPacket, eth_in.c:27-87 -> ProcessInIPv4Packet, ip_in.c:30-101 ->
 * ProcessInTCPPacket prefix, tcp.c:408-445 (+ FillPacketContextTCPInfo,
 * tcp.c:258-270).  The stream lookup after tcp.c:445 returns TRUE for every
 * frame in the reference harness state, so a frame that reaches it is TCP_OK. */
void mo_classify_one(const mosrx_params *p, const uint32_t cache[96],
                     const uint8_t *f, uint32_t caplen, mosrx_result *r)
{
	uint16_t h_proto, ip_len;
	unsigned ver, ihl, proto, doff = 0;
	const uint8_t *iph, *tcph;
	uint32_t saddr, daddr;
	uint16_t sport = 0, dport = 0;

	memset(r, 0, sizeof(*r));
	if (caplen < 14) {                      /* ethertype unreadable */
		VERDICT(r, -1, MOSRX_R_TRUNCATED);
		return;
	}
	h_proto = be16(f + 12);                  /* eth_in.c:34 */
	if (h_proto != 0x0800) {
		if (!p->num_msp || !p->forward) {    /* eth_in.c:62 */
			if (h_proto == 0x0806)
				VERDICT(r, 1, MOSRX_R_ARP);       /* eth_in.c:63-66, RUN_ARP (arp.h:7) */
			else
				VERDICT(r, -1, MOSRX_R_NON_IPV4); /* eth_in.c:69-73 */
		} else {                                  /* eth_in.c:74-77 ForwardEthernetFrame */
			VERDICT(r, 1, h_proto == 0x0806 ? MOSRX_R_ARP : MOSRX_R_NON_IPV4);
		}
		return;
	}

	/* IPv4.  TRUNCATED (build-only) is decided first from the
	 * header fields: any byte the reference path reads past caplen. */
	if (caplen < 34) {
		VERDICT(r, -1, MOSRX_R_TRUNCATED);
		return;
	}
	iph = f + 14;
	ip_len = be16(iph + 2);
	ver = iph[0] >> 4;
	ihl = iph[0] & 0xF;
	proto = iph[9];
	if (14u + ihl * 4 > caplen || 14u + ip_len > caplen || (proto == 6 && 14u + ihl * 4 + 20 > caplen)) {
		VERDICT(r, -1, MOSRX_R_TRUNCATED);
		return;
	}
	if (ip_len < 20) {                       /* ip_in.c:42-45 */
		VERDICT(r, -1, MOSRX_R_IP_SHORT);
		return;
	}
	if (ver != 4) {                          /* ip_in.c:47-51 */
		VERDICT(r, 0, MOSRX_R_IP_BADVER);
		return;
	}

	/* Header fields and RSS: defined for every IPv4 frame past the version check. */
	saddr = le32(iph + 12);
	daddr = le32(iph + 16);
	tcph = iph + ihl * 4;
	if (proto == 6) {
		doff = tcph[12] >> 4;
		sport = be16(tcph);
		dport = be16(tcph + 2);
		r->tcp_flags = tcph[13];
		r->payloadlen = (uint16_t)(ip_len - (ihl * 4 + doff * 4));     /* tcp.c:262 */
		r->payload_off = (uint8_t)(14 + ihl * 4 + doff * 4);
	}
	r->ihl_doff = (uint8_t)((ihl << 4) | doff);
	r->rss = mo_rss_hash(cache, be32(iph + 12), be32(iph + 16), sport, dport);
	r->queue = (uint8_t)mo_rss_queue(r->rss, p->queue_mode, p->num_queues);

	if (p->num_msp == 0 && p->num_esp == 0) { /* ip_in.c:67-72: no checksums */
		VERDICT(r, 1, MOSRX_R_NOVERIFY_PASS);
		return;
	}
	r->ip_csum = mo_ip_fast_csum(iph, ihl);
	if (r->ip_csum) {                        /* ip_in.c:74-77 */
		VERDICT(r, -1, MOSRX_R_IP_BADCSUM);
		return;
	}
	if (proto != 6) {
		/* ip_in.c:82-85: ICMP to one of the netdevs' addresses is processed
		 * (ProcessICMPPacket returns TRUE whatever the type, icmp.c:193-227) */
		if (proto == 1) {
			uint32_t k;
			for (k = 0; k < p->num_local && k < MOSRX_MAX_LOCAL; k++)
				if (daddr == p->local_ip[k]) {
					VERDICT(r, 1, MOSRX_R_ICMP_LOCAL);
					return;
				}
		}
		VERDICT(r, 0, MOSRX_R_NOT_TCP);   /* ip_in.c:86-93: other protocols */
		return;
	}
	if (ip_len < (ihl + doff) * 4) {          /* tcp.c:429-430 */
		VERDICT(r, -1, MOSRX_R_TCP_SHORT);
		return;
	}
	if (p->skip_tcp_csum) {
		VERDICT(r, 1, MOSRX_R_TCP_LEN_OK);
		return;
	}
	/* tcp.c:432-434: len = (doff << 2) + payloadlen, truncated to u16 */
	r->tcp_csum = mo_tcp_csum(tcph, (uint16_t)(doff * 4 + r->payloadlen), saddr, daddr);
	if (r->tcp_csum)
		VERDICT(r, -1, MOSRX_R_TCP_BADCSUM);
	else
		VERDICT(r, 1, MOSRX_R_TCP_OK);
}

static inline uint32_t eff_caplen(uint64_t frames_bytes, uint32_t off, uint16_t len)
{
	if ((uint64_t)off >= frames_bytes)
		return 0;
	if ((uint64_t)off + len > frames_bytes)
		return (uint32_t)(frames_bytes - off);
	return len;
}

int mo_classify(const mosrx_params *p, const uint8_t *frames, uint64_t frames_bytes,
                const uint32_t *off, const uint16_t *len, uint32_t n, mosrx_result *out)
{
	uint32_t cache[96];
	uint32_t i;

	if (!p || (n && (!frames || !off || !len || !out)))
		return -EINVAL;
	if (p->rss_key_len < 16 || p->num_queues < 1 || p->num_queues > 256)
		return -EINVAL;
	mo_rss_key_cache(p->rss_key, cache);
	for (i = 0; i < n; i++)
		mo_classify_one(p, cache, frames + off[i], eff_caplen(frames_bytes, off[i], len[i]), &out[i]);
	return 0;
}

struct mt_arg {
	const mosrx_params *p;
	const uint8_t *frames;
	uint64_t frames_bytes;
	const uint32_t *off;
	const uint16_t *len;
	uint32_t lo, hi;
	mosrx_result *out;
	int ret;
};

static void *mt_main(void *a_)
{
	struct mt_arg *a = a_;
	a->ret = mo_classify(a->p, a->frames, a->frames_bytes, a->off + a->lo, a->len + a->lo,
	                     a->hi - a->lo, a->out + a->lo);
	return NULL;
}

int mo_classify_mt(const mosrx_params *p, const uint8_t *frames, uint64_t frames_bytes,
                   const uint32_t *off, const uint16_t *len, uint32_t n, mosrx_result *out,
                   int nthreads)
{
	pthread_t *th;
	struct mt_arg *args;
	int t, ret = 0;

	if (nthreads <= 1)
		return mo_classify(p, frames, frames_bytes, off, len, n, out);
	th = calloc((size_t)nthreads, sizeof(*th));
	args = calloc((size_t)nthreads, sizeof(*args));
	if (!th || !args) {
		free(th);
		free(args);
		return -ENOMEM;
	}
	for (t = 0; t < nthreads; t++) {
		args[t] = (struct mt_arg){p, frames, frames_bytes, off, len,
		                          (uint32_t)((uint64_t)n * t / nthreads),
		                          (uint32_t)((uint64_t)n * (t + 1) / nthreads), out, 0};
		if (pthread_create(&th[t], NULL, mt_main, &args[t]))
			args[t].ret = -EAGAIN, th[t] = 0;
	}
	for (t = 0; t < nthreads; t++) {
		if (th[t])
			pthread_join(th[t], NULL);
		if (args[t].ret)
			ret = args[t].ret;
	}
	free(th);
	free(args);
	return ret;
}
