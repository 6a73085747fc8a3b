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
 * backend can receive directly into pinned memory; the memory source also
 * copies whole runs (fill) or lends its pinned replay buffer (borrow).
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
#define __HIP_PLATFORM_AMD__ 1   /* host-only C over the HIP runtime API */
#include <hip/hip_runtime_api.h>

#include "mosrx_source.h"

/* ---------------- in-memory replay ---------------- */
/* The replay buffer is kept in the staging layout (frame i at a 16-byte
 * boundary + 2, packed), so a batch is one memcpy per contiguous run with the
 * offsets rebased (mem_fill), as a NIC ring hands a DMA'd run of slots. */
struct src_mem {
	struct mosrx_source base;
	uint8_t *frames;
	uint32_t *off;
	uint16_t *len;
	uint32_t n, i, loops, done_loops, max_len;
	int pinned;   /* frames in hipHostMalloc'd memory: batches are borrowed, not copied */
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

static uint32_t mem_fill(struct mosrx_source *s_, uint8_t *dst, uint64_t cap, uint32_t *off, uint16_t *len,
                         uint32_t max_n, uint32_t max_frame, uint64_t *end)
{
	struct src_mem *s = (struct src_mem *)s_;
	uint64_t pos = 2;
	uint32_t k = 0;
	if (s->max_len > max_frame) {   /* frames to truncate: the per-frame path */
		int l;
		while (k < max_n && pos + max_frame + 16 <= cap && (l = mem_next(s_, dst + pos, max_frame)) > 0) {
			off[k] = (uint32_t)pos;
			len[k] = (uint16_t)l;
			k++;
			pos = ((pos + (uint64_t)l - 2 + 15) & ~15ull) + 2;
		}
		*end = pos;
		return k;
	}
	while (k < max_n && s->n) {
		uint32_t a, b, j;
		uint64_t base, room;
		if (s->i == s->n) {
			s->done_loops++;
			if (s->loops && s->done_loops >= s->loops)
				break;
			s->i = 0;
		}
		/* the run [a, b) of source frames that fits the count and the space left */
		a = s->i;
		base = s->off[a];
		room = cap - pos;
		b = a;
		while (b < s->n && k + (b - a) < max_n && (uint64_t)(s->off[b] - base) + max_frame + 16 <= room)
			b++;
		if (b == a)
			break;
		memcpy(dst + pos, s->frames + base, (size_t)(s->off[b - 1] - base) + s->len[b - 1]);
		for (j = a; j < b; j++, k++) {
			off[k] = (uint32_t)(pos + (s->off[j] - base));
			len[k] = s->len[j];
		}
		pos = ((pos + (s->off[b - 1] - base) + s->len[b - 1] - 2 + 15) & ~15ull) + 2;
		s->i = b;
	}
	*end = pos;
	return k;
}

/* Zero-copy: the next run of the pinned replay buffer is the batch itself (as
 * a NIC's DMA ring slots are); only the rebased descriptors are written. */
static uint32_t mem_borrow(struct mosrx_source *s_, uint32_t max_n, uint32_t max_frame, const uint8_t **frames,
                           uint64_t *frames_bytes, uint32_t *off, uint16_t *len)
{
	struct src_mem *s = (struct src_mem *)s_;
	uint32_t a, b, k, base;
	if (!s->n || !max_n)
		return 0;
	if (s->i == s->n) {
		s->done_loops++;
		if (s->loops && s->done_loops >= s->loops)
			return 0;
		s->i = 0;
	}
	a = s->i;
	b = s->n - a > max_n ? a + max_n : s->n;
	base = s->off[a] - 2;
	for (k = 0; a + k < b; k++) {
		off[k] = s->off[a + k] - base;
		len[k] = s->len[a + k] < max_frame ? s->len[a + k] : (uint16_t)max_frame;
	}
	*frames = s->frames + base;
	*frames_bytes = (uint64_t)off[k - 1] + len[k - 1];
	s->i = b;
	return k;
}

static void mem_close(struct mosrx_source *s_)
{
	struct src_mem *s = (struct src_mem *)s_;
	if (s->pinned)
		hipHostFree(s->frames);
	else
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
		total += ((uint64_t)len[i] + 15) & ~15ull;
	total += 16;
	/* pinned when a HIP device is present (zero-copy batches), else plain */
	if (hipHostMalloc((void **)&s->frames, total, hipHostMallocPortable) == hipSuccess)
		s->pinned = 1;
	else
		s->frames = malloc(total);
	s->off = malloc((size_t)(n ? n : 1) * 4);
	s->len = malloc((size_t)(n ? n : 1) * 2);
	if (!s->frames || !s->off || !s->len || total >= (1ull << 32)) {
		mem_close(&s->base);
		return NULL;
	}
	pos = 2;
	for (i = 0; i < n; i++) {
		memcpy(s->frames + pos, frames + off[i], len[i]);
		s->off[i] = (uint32_t)pos;
		s->len[i] = len[i];
		if (len[i] > s->max_len)
			s->max_len = len[i];
		pos = ((pos + len[i] - 2 + 15) & ~15ull) + 2;
	}
	s->n = n;
	s->loops = loops;
	s->base.next = mem_next;
	s->base.fill = mem_fill;
	if (s->pinned)
		s->base.borrow = mem_borrow;
	s->base.close = mem_close;
	return &s->base;
}

int mosrx_source_mem_set_mode(mosrx_source *s_, int mode)
{
	struct src_mem *s = (struct src_mem *)s_;
	if (!s_ || s_->next != mem_next || mode < 0 || mode > 2)
		return -EINVAL;
	s->base.borrow = mode == 0 && s->pinned ? mem_borrow : NULL;
	s->base.fill = mode <= 1 ? mem_fill : NULL;
	return 0;
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
