/*
 * loopback.c — frame sources the GPU backend pulls from (the raw-socket /
 * loopback side of SURVEY.md §8b).
 *
 *   mem       replays an in-memory trace (the loopback trace of BASELINE config #1)
 *   pcap      native reader for classic pcap files; the reference's pcap backend
 *             links libpcap (pcap_module.c:13, pcap_next :41), which the image lacks
 *   afpacket  raw AF_PACKET socket on an interface (pcap_create + pcap_activate,
 *             pcap_module.c:140-156, without libpcap)
 *
 * Each source writes one frame straight into the caller's staging slot, so a
 * backend can receive directly into pinned memory.
 */
#define _GNU_SOURCE
#include <arpa/inet.h>
#include <errno.h>
#include <linux/if_ether.h>
#include <linux/if_packet.h>
#include <net/if.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/socket.h>
#include <unistd.h>

#include "../../include/mosrx_io_module.h"
#include "mosrx_source.h"

/* ---------------- in-memory replay ---------------- */
struct src_mem {
	struct mosrx_source base;
	uint8_t *frames;
	uint32_t *off;
	uint16_t *len;
	uint32_t n, i, loops, done_loops;
};

static int mem_next(struct mosrx_source *s_, uint8_t *dst, uint32_t cap)
{
	struct src_mem *s = (struct src_mem *)s_;
	uint32_t l;
	if (s->n == 0)
		return 0;
	if (s->i == s->n) {
		s->done_loops++;
		if (s->loops && s->done_loops >= s->loops)
			return 0;
		s->i = 0;
	}
	l = s->len[s->i];
	if (l > cap)
		l = cap;
	memcpy(dst, s->frames + s->off[s->i], l);
	s->i++;
	return (int)l;
}

static void mem_close(struct mosrx_source *s_)
{
	struct src_mem *s = (struct src_mem *)s_;
	free(s->frames);
	free(s->off);
	free(s->len);
	free(s);
}

mosrx_source *mosrx_source_mem(const uint8_t *frames, const uint32_t *off, const uint16_t *len,
                               uint32_t n, uint32_t loops)
{
	struct src_mem *s = calloc(1, sizeof(*s));
	uint64_t total = 0, pos = 0;
	uint32_t i;
	if (!s)
		return NULL;
	for (i = 0; i < n; i++)
		total += len[i];
	s->frames = malloc(total ? total : 1);
	s->off = malloc((size_t)(n ? n : 1) * 4);
	s->len = malloc((size_t)(n ? n : 1) * 2);
	if (!s->frames || !s->off || !s->len || total >= (1ull << 32)) {
		mem_close(&s->base);
		return NULL;
	}
	for (i = 0; i < n; i++) {
		memcpy(s->frames + pos, frames + off[i], len[i]);
		s->off[i] = (uint32_t)pos;
		s->len[i] = len[i];
		pos += len[i];
	}
	s->n = n;
	s->loops = loops;
	s->base.next = mem_next;
	s->base.close = mem_close;
	return &s->base;
}

/* ---------------- classic pcap file ---------------- */
struct src_pcap {
	struct mosrx_source base;
	FILE *f;
	char *path;
	int swap;
	uint32_t loops, done_loops;
};

static uint32_t sw32(uint32_t v, int swap) { return swap ? __builtin_bswap32(v) : v; }

static int pcap_open_hdr(struct src_pcap *s)
{
	uint32_t gh[6];
	if (fread(gh, 4, 6, s->f) != 6)
		return -1;
	if (gh[0] == 0xa1b2c3d4u || gh[0] == 0xa1b23c4du)
		s->swap = 0;
	else if (gh[0] == 0xd4c3b2a1u || gh[0] == 0x4d3cb2a1u)
		s->swap = 1;
	else
		return -1;
	if (sw32(gh[5], s->swap) != 1)   /* LINKTYPE_ETHERNET */
		return -1;
	return 0;
}

static int pcap_next_frame(struct mosrx_source *s_, uint8_t *dst, uint32_t cap)
{
	struct src_pcap *s = (struct src_pcap *)s_;
	uint32_t rh[4], incl, take;
	for (;;) {
		if (fread(rh, 4, 4, s->f) == 4)
			break;
		s->done_loops++;
		if (s->loops && s->done_loops >= s->loops)
			return 0;
		if (fseek(s->f, 24, SEEK_SET))
			return 0;
	}
	incl = sw32(rh[2], s->swap);
	take = incl < cap ? incl : cap;
	if (fread(dst, 1, take, s->f) != take)
		return 0;
	if (incl > take && fseek(s->f, (long)(incl - take), SEEK_CUR))
		return 0;
	return (int)take;
}

static void pcap_close_src(struct mosrx_source *s_)
{
	struct src_pcap *s = (struct src_pcap *)s_;
	if (s->f)
		fclose(s->f);
	free(s->path);
	free(s);
}

mosrx_source *mosrx_source_pcap(const char *path, uint32_t loops)
{
	struct src_pcap *s = calloc(1, sizeof(*s));
	if (!s)
		return NULL;
	s->f = fopen(path, "rb");
	if (!s->f || pcap_open_hdr(s)) {
		pcap_close_src(&s->base);
		return NULL;
	}
	s->loops = loops ? loops : 1;
	s->base.next = pcap_next_frame;
	s->base.close = pcap_close_src;
	return &s->base;
}

/* ---------------- AF_PACKET raw socket ---------------- */
struct src_afp {
	struct mosrx_source base;
	int fd;
};

static int afp_next(struct mosrx_source *s_, uint8_t *dst, uint32_t cap)
{
	struct src_afp *s = (struct src_afp *)s_;
	ssize_t r = recv(s->fd, dst, cap, MSG_DONTWAIT | MSG_TRUNC);
	if (r <= 0)
		return 0;
	return (int)(r > (ssize_t)cap ? cap : (uint32_t)r);
}

static void afp_close(struct mosrx_source *s_)
{
	struct src_afp *s = (struct src_afp *)s_;
	if (s->fd >= 0)
		close(s->fd);
	free(s);
}

mosrx_source *mosrx_source_afpacket(const char *ifname)
{
	struct src_afp *s = calloc(1, sizeof(*s));
	struct sockaddr_ll sll;
	int rcvbuf = 16 << 20;   /* PCAP_BUFFER_SIZE, pcap_module.c:26 */
	if (!s)
		return NULL;
	s->fd = socket(AF_PACKET, SOCK_RAW, htons(ETH_P_ALL));
	if (s->fd < 0) {
		free(s);
		return NULL;
	}
	memset(&sll, 0, sizeof(sll));
	sll.sll_family = AF_PACKET;
	sll.sll_protocol = htons(ETH_P_ALL);
	sll.sll_ifindex = (int)if_nametoindex(ifname);
	setsockopt(s->fd, SOL_SOCKET, SO_RCVBUF, &rcvbuf, sizeof(rcvbuf));
	if (sll.sll_ifindex == 0 || bind(s->fd, (struct sockaddr *)&sll, sizeof(sll))) {
		afp_close(&s->base);
		return NULL;
	}
	s->base.next = afp_next;
	s->base.close = afp_close;
	return &s->base;
}

int mosrx_source_next(mosrx_source *s, uint8_t *dst, uint32_t cap)
{
	if (!s || !dst || !s->next)
		return -EINVAL;
	return s->next(s, dst, cap);
}

void mosrx_source_close(mosrx_source *s)
{
	if (s && s->close)
		s->close(s);
}
