/*
 * loopback.c — frame sources the GPU backend pulls from (the raw-socket /
 * loopback side of SURVEY.md §8b).
 *
 *   mem       replays an in-memory trace (the loopback trace of BASELINE config #1)
 *   pcap      native reader for classic pcap files; the reference's pcap backend
 *             links libpcap (pcap_module.c:13, pcap_next :41), which the image lacks
 *   afpacket  raw AF_PACKET socket on an interface with a TPACKET_V3 PACKET_MMAP
 *             ring (pcap_create + pcap_activate, pcap_module.c:140-156, without
 *             libpcap)
 *
 * Each source writes one frame straight into the caller's staging slot, so a
 * backend can receive directly into pinned memory; the memory source also
 * copies whole runs (fill), and the memory and AF_PACKET sources lend their
 * pinned memory as the batch itself (borrow).  Frames sent back out
 * (send_pkts, pcap_module.c:67-89) leave through the source: the AF_PACKET
 * socket, or a pcap dump file for any source.
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
#include <sys/mman.h>
#include <sys/socket.h>
#include <time.h>
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
		while (k < max_n && pos + max_frame + 32 <= cap) {
			/* the frame's own length places it: read it into the aligned slot, move it back if it packs */
			const uint64_t al = mosrx__frame_at(pos, MOSRX_PACK_MAX + 1);
			if ((l = mem_next(s_, dst + al, max_frame)) <= 0)
				break;
			if (mosrx__frame_at(pos, (uint32_t)l) != al)
				memmove(dst + pos, dst + al, (size_t)l);
			else
				pos = al;
			off[k] = (uint32_t)pos;
			len[k] = (uint16_t)l;
			k++;
			pos += (uint64_t)l;
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
		/* the run [a, b) of source frames that fits the count and the space left,
		 * copied whole at the source's alignment mod 16 (its frames keep their
		 * places in the layout) */
		a = s->i;
		base = s->off[a];
		pos += (base - pos) & 15u;
		if (pos + 32 > cap)
			break;
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
		pos += (uint64_t)(s->off[b - 1] - base) + s->len[b - 1];
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
	base = (s->off[a] - 2) & ~15u;   /* the run handed out from a 16-byte boundary */
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
	if (s->pinned) {
		mosrx__host_range_del(s->frames);
		hipHostFree(s->frames);
	}
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
	if (hipHostMalloc((void **)&s->frames, total, hipHostMallocPortable) == hipSuccess) {
		s->pinned = 1;
		mosrx__host_range_add(s->frames, total);
	}
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
		pos = mosrx__frame_at(pos, len[i]);
		memcpy(s->frames + pos, frames + off[i], len[i]);
		s->off[i] = (uint32_t)pos;
		s->len[i] = len[i];
		if (len[i] > s->max_len)
			s->max_len = len[i];
		pos += len[i];
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
/* pcap_next (pcap_module.c:41) without libpcap.  The file is mapped and read
 * in place: per frame (next) or a batch at a time straight into the backend's
 * stage (fill: one memcpy per frame, no stdio); a file that cannot be mapped
 * is read through stdio, per frame. */
struct src_pcap {
	struct mosrx_source base;
	FILE *f;
	int swap;
	uint32_t loops, done_loops;
	const uint8_t *map;             /* the mapped file (NULL: stdio) */
	size_t map_len, pos;            /* the next record header at map + pos */
};

static uint32_t sw32(uint32_t v, int swap) { return swap ? __builtin_bswap32(v) : v; }

static int pcap_check_hdr(struct src_pcap *s, const uint32_t *gh)
{
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

/* The next record of the mapped file (wrapping for replays): its bytes and
 * captured length, or NULL at the end of the last replay. */
static const uint8_t *pcap_map_record(struct src_pcap *s, uint32_t *incl)
{
	for (;;) {
		if (s->pos + 16 <= s->map_len) {
			uint32_t rh[4];
			memcpy(rh, s->map + s->pos, 16);
			*incl = sw32(rh[2], s->swap);
			if (s->pos + 16 + (size_t)*incl <= s->map_len)
				return s->map + s->pos + 16;
		}
		s->done_loops++;             /* end of file (or a truncated last record) */
		if (s->loops && s->done_loops >= s->loops)
			return NULL;
		if (s->map_len < 24 + 16 || s->pos == 24)
			return NULL;             /* an empty file never yields a frame */
		s->pos = 24;
	}
}

static int pcap_next_frame(struct mosrx_source *s_, uint8_t *dst, uint32_t cap)
{
	struct src_pcap *s = (struct src_pcap *)s_;
	uint32_t rh[4], incl, take;
	if (s->map) {
		const uint8_t *rec = pcap_map_record(s, &incl);
		if (!rec)
			return 0;
		take = incl < cap ? incl : cap;
		memcpy(dst, rec, take);
		s->pos += 16 + (size_t)incl;
		return (int)take;
	}
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

/* A batch into the stage, in the backend's layout (mosrx__frame_at). */
static uint32_t pcap_fill(struct mosrx_source *s_, uint8_t *dst, uint64_t cap, uint32_t *off, uint16_t *len,
                          uint32_t max_n, uint32_t max_frame, uint64_t *end)
{
	struct src_pcap *s = (struct src_pcap *)s_;
	uint64_t pos = 2;
	uint32_t k = 0, incl;
	while (k < max_n && pos + max_frame + 16 <= cap) {
		const uint8_t *rec = pcap_map_record(s, &incl);
		uint32_t take;
		if (!rec)
			break;
		take = incl < max_frame ? incl : max_frame;
		pos = mosrx__frame_at(pos, take);
		memcpy(dst + pos, rec, take);
		s->pos += 16 + (size_t)incl;
		off[k] = (uint32_t)pos;
		len[k] = (uint16_t)take;
		k++;
		pos += take;
	}
	*end = pos;
	return k;
}

static void pcap_close_src(struct mosrx_source *s_)
{
	struct src_pcap *s = (struct src_pcap *)s_;
	if (s->map)
		munmap((void *)s->map, s->map_len);
	if (s->f)
		fclose(s->f);
	free(s);
}

mosrx_source *mosrx_source_pcap(const char *path, uint32_t loops)
{
	struct src_pcap *s = calloc(1, sizeof(*s));
	uint32_t gh[6];
	long sz;
	if (!s)
		return NULL;
	s->f = fopen(path, "rb");
	if (!s->f || fread(gh, 4, 6, s->f) != 6 || pcap_check_hdr(s, gh)) {
		pcap_close_src(&s->base);
		return NULL;
	}
	s->loops = loops ? loops : 1;
	s->base.next = pcap_next_frame;
	s->base.close = pcap_close_src;
	if (fseek(s->f, 0, SEEK_END) == 0 && (sz = ftell(s->f)) >= 24) {
		void *m = mmap(NULL, (size_t)sz, PROT_READ, MAP_PRIVATE, fileno(s->f), 0);
		if (m != MAP_FAILED) {
			s->map = m;
			s->map_len = (size_t)sz;
			s->pos = 24;
			s->base.fill = pcap_fill;
		}
	}
	if (!s->map && fseek(s->f, 24, SEEK_SET)) {
		pcap_close_src(&s->base);
		return NULL;
	}
	return &s->base;
}

/* ---------------- AF_PACKET raw socket: a TPACKET_V3 PACKET_MMAP ring ---------------- */
/* The kernel writes received frames straight into a ring of blocks mapped into
 * this process (what libpcap does for pcap_create + pcap_activate on Linux,
 * pcap_module.c:140-156).  TPACKET_V3 places each frame's network header on a
 * 16-byte boundary, so the Ethernet header sits at 16 B + 2: the staging layout
 * the kernels read fastest.  When the ring can be registered with the HIP
 * runtime (hipHostRegister) a run of frames is lent to the backend as the batch
 * itself (borrow), and its blocks go back to the kernel when the backend
 * releases the run (give_back); otherwise frames are copied out (fill / next)
 * and each block is returned as soon as it is drained.  Frames the host sent
 * itself (PACKET_OUTGOING) are never delivered: libpcap's default direction
 * drops them too, so a frame sent on `lo` is received once. */
#define AFP_BLOCK_SIZE (1u << 22)   /* 4 MiB blocks */
#define AFP_MAX_BLOCKS 64
#define AFP_MAX_RUNS   (2 * MOSRX_MAX_GROUP + 2)   /* borrowed runs outstanding: two groups of batches */

struct src_afp {
	struct mosrx_source base;
	int fd;
	uint8_t *ring;
	uint32_t nblocks;
	int registered;                 /* ring registered with hipHostRegister: borrow is available */
	int external;                   /* the ring is the caller's mapping (mosrx_source_tpacket_v3) */
	uint32_t bsz;                   /* block size */
	/* cursor: block `blk`, `left` frames not yet taken, next frame at `fp` */
	uint32_t blk, left;
	uint8_t *fp;
	/* blocks taken in full but not yet given back: [rel, blk) (mod nblocks), and
	 * per outstanding run the block count it completes (FIFO) */
	uint32_t rel;
	uint32_t run_upto[AFP_MAX_RUNS];
	uint32_t run_head, run_tail;
	uint64_t dropped_outgoing;
	uint64_t ring_packets, ring_drops;   /* PACKET_STATISTICS, accumulated (the kernel resets on read) */
};

static struct tpacket_block_desc *afp_block(struct src_afp *s, uint32_t b)
{
	return (struct tpacket_block_desc *)(s->ring + (size_t)(b % s->nblocks) * s->bsz);
}

static void afp_release_upto(struct src_afp *s, uint32_t upto)
{
	while (s->rel != upto) {
		struct tpacket_block_desc *bd = afp_block(s, s->rel);
		__atomic_store_n(&bd->hdr.bh1.block_status, TP_STATUS_KERNEL, __ATOMIC_RELEASE);
		s->rel++;
	}
}

/* Make the cursor point at a frame; 0 when the kernel has retired no block. */
static int afp_ready(struct src_afp *s)
{
	while (!s->left) {
		struct tpacket_block_desc *bd;
		if (s->fp) {                     /* the cursor's block is drained */
			s->blk++;
			s->fp = NULL;
		}
		if (s->blk - s->rel >= s->nblocks)
			return 0;                    /* every block held by outstanding runs */
		bd = afp_block(s, s->blk);
		if (!(__atomic_load_n(&bd->hdr.bh1.block_status, __ATOMIC_ACQUIRE) & TP_STATUS_USER))
			return 0;
		s->left = bd->hdr.bh1.num_pkts;
		s->fp = (uint8_t *)bd + bd->hdr.bh1.offset_to_first_pkt;
		if (!s->left) {                  /* an empty retired block */
			s->blk++;
			s->fp = NULL;
		}
	}
	return 1;
}

/* Blocks fully taken: those before the cursor's, and the cursor's own once drained. */
static uint32_t afp_done(const struct src_afp *s)
{
	return (s->fp && !s->left) ? s->blk + 1 : s->blk;
}

/* Take the cursor's frame: its Ethernet header and capture length, or NULL for
 * a frame to skip (outgoing). */
static const uint8_t *afp_take(struct src_afp *s, uint32_t *caplen)
{
	const struct tpacket3_hdr *h = (const struct tpacket3_hdr *)s->fp;
	const struct sockaddr_ll *sll = (const struct sockaddr_ll *)(s->fp + TPACKET_ALIGN(sizeof(*h)));
	const uint8_t *mac = s->fp + h->tp_mac;
	*caplen = h->tp_snaplen;
	s->left--;
	s->fp += h->tp_next_offset;
	if (sll->sll_pkttype == PACKET_OUTGOING) {
		s->dropped_outgoing++;
		return NULL;
	}
	return mac;
}

/* Copying forms: blocks go back as soon as they are drained (no run is lent). */
static int afp_next(struct mosrx_source *s_, uint8_t *dst, uint32_t cap)
{
	struct src_afp *s = (struct src_afp *)s_;
	for (;;) {
		uint32_t l;
		const uint8_t *mac;
		if (!afp_ready(s)) {
			if (s->run_head == s->run_tail)
				afp_release_upto(s, afp_done(s));
			return 0;
		}
		mac = afp_take(s, &l);
		if (s->run_head == s->run_tail)
			afp_release_upto(s, afp_done(s));
		if (!mac)
			continue;
		l = l < cap ? l : cap;
		memcpy(dst, mac, l);
		return (int)l;
	}
}

static void afp_give_back(struct mosrx_source *s_);

/* Zero-copy: frames of consecutive retired blocks, up to the ring's end (a run
 * never wraps, so it is one contiguous span of the registered ring). */
static uint32_t afp_borrow(struct mosrx_source *s_, uint32_t max_n, uint32_t max_frame, const uint8_t **frames,
                           uint64_t *frames_bytes, uint32_t *off, uint16_t *len)
{
	struct src_afp *s = (struct src_afp *)s_;
	const uint8_t *base = NULL;
	uint32_t k = 0, first_blk;
	uint64_t end = 0;
	if ((s->run_tail - s->run_head) >= AFP_MAX_RUNS || !afp_ready(s))
		return 0;
	first_blk = s->blk;
	base = (const uint8_t *)afp_block(s, first_blk);
	while (k < max_n) {
		uint32_t l;
		const uint8_t *mac;
		if (!s->left) {
			/* continue into the next block only if it is retired and contiguous */
			if ((s->blk + 1) % s->nblocks == 0 || !afp_ready(s))
				break;
		}
		mac = afp_take(s, &l);
		if (!mac)
			continue;
		off[k] = (uint32_t)(mac - base);
		len[k] = (uint16_t)(l < max_frame ? l : max_frame);
		end = (uint64_t)off[k] + len[k];
		k++;
	}
	/* the run completes every block before the cursor's (and the cursor's own when drained) */
	s->run_upto[s->run_tail % AFP_MAX_RUNS] = afp_done(s);
	s->run_tail++;
	if (!k) {                        /* only outgoing frames: nothing to lend, release at once */
		afp_give_back(s_);
		return 0;
	}
	*frames = base;
	*frames_bytes = end;
	return k;
}

static void afp_give_back(struct mosrx_source *s_)
{
	struct src_afp *s = (struct src_afp *)s_;
	if (s->run_head == s->run_tail)
		return;
	afp_release_upto(s, s->run_upto[s->run_head % AFP_MAX_RUNS]);
	s->run_head++;
}

static int afp_send(struct mosrx_source *s_, const uint8_t *frame, uint32_t len)
{
	struct src_afp *s = (struct src_afp *)s_;
	return send(s->fd, frame, len, 0) == (ssize_t)len ? 0 : -errno;   /* pcap_inject */
}

static void afp_close(struct mosrx_source *s_)
{
	struct src_afp *s = (struct src_afp *)s_;
	if (s->registered) {
		mosrx__host_range_del(s->ring);
		hipHostUnregister(s->ring);
	}
	if (s->ring && s->ring != MAP_FAILED && !s->external)
		munmap(s->ring, (size_t)s->nblocks * s->bsz);
	if (s->fd >= 0)
		close(s->fd);
	free(s);
}

mosrx_source *mosrx_source_afpacket_ex(const char *ifname, const mosrx_afpacket_opts *o)
{
	struct src_afp *s = calloc(1, sizeof(*s));
	struct sockaddr_ll sll;
	struct tpacket_req3 req;
	int v = TPACKET_V3, one = 1;
	const uint32_t nb = o && o->ring_blocks ? o->ring_blocks : 8;
	if (!s || !ifname || nb > AFP_MAX_BLOCKS) {
		free(s);
		return NULL;
	}
	s->base.close = afp_close;
	s->bsz = AFP_BLOCK_SIZE;
	s->fd = socket(AF_PACKET, SOCK_RAW, htons(ETH_P_ALL));
	if (s->fd < 0) {
		free(s);
		return NULL;
	}
	memset(&req, 0, sizeof(req));
	req.tp_block_size = AFP_BLOCK_SIZE;
	req.tp_block_nr = nb;
	req.tp_frame_size = 2048;
	req.tp_frame_nr = (AFP_BLOCK_SIZE / 2048) * nb;
	req.tp_retire_blk_tov = o && o->retire_ms ? o->retire_ms : 1;   /* hand partly filled blocks over after 1 ms */
	memset(&sll, 0, sizeof(sll));
	sll.sll_family = AF_PACKET;
	sll.sll_protocol = htons(ETH_P_ALL);
	sll.sll_ifindex = (int)if_nametoindex(ifname);
	if (setsockopt(s->fd, SOL_PACKET, PACKET_VERSION, &v, sizeof(v)) ||
	    setsockopt(s->fd, SOL_PACKET, PACKET_RX_RING, &req, sizeof(req))) {
		afp_close(&s->base);
		return NULL;
	}
	/* outgoing frames never reach the ring (kernels before 4.20 lack the option:
	 * afp_take still drops them by sll_pkttype) */
	setsockopt(s->fd, SOL_PACKET, PACKET_IGNORE_OUTGOING, &one, sizeof(one));
	s->nblocks = nb;
	s->ring = mmap(NULL, (size_t)nb * AFP_BLOCK_SIZE, PROT_READ | PROT_WRITE, MAP_SHARED | MAP_LOCKED, s->fd, 0);
	if (s->ring == MAP_FAILED)
		s->ring = mmap(NULL, (size_t)nb * AFP_BLOCK_SIZE, PROT_READ | PROT_WRITE, MAP_SHARED, s->fd, 0);
	if (s->ring == MAP_FAILED || sll.sll_ifindex == 0 || bind(s->fd, (struct sockaddr *)&sll, sizeof(sll))) {
		afp_close(&s->base);
		return NULL;
	}
	if (o && o->fanout_group) {      /* one socket per mTCP thread, flows split by hash (RSS-like) */
		int fo = (int)((o->fanout_group & 0xFFFF) | (PACKET_FANOUT_HASH << 16));
		if (setsockopt(s->fd, SOL_PACKET, PACKET_FANOUT, &fo, sizeof(fo))) {
			afp_close(&s->base);
			return NULL;
		}
	}
	s->base.next = afp_next;
	s->base.send = afp_send;
	if (!(o && o->copy) &&
	    hipHostRegister(s->ring, (size_t)nb * AFP_BLOCK_SIZE, hipHostRegisterDefault) == hipSuccess) {
		s->registered = 1;
		mosrx__host_range_add(s->ring, (uint64_t)nb * AFP_BLOCK_SIZE);
		s->base.borrow = afp_borrow;
		s->base.give_back = afp_give_back;
	}
	return &s->base;
}

/* A TPACKET_V3 ring the caller maps and something else fills (a shared-memory
 * capture, a driver with the same block layout): the same cursor, lending and
 * give-back as the socket's ring, registered with the HIP runtime the same way
 * (hipHostRegister of the whole mapping) so runs are lent zero-copy; copying
 * when the registration fails.  No socket: nothing to send, no statistics. */
mosrx_source *mosrx_source_tpacket_v3(void *ring, uint32_t nblocks, uint32_t block_size)
{
	struct src_afp *s;
	if (!ring || !nblocks || nblocks > AFP_MAX_BLOCKS || block_size < 4096 || (block_size & (block_size - 1)))
		return NULL;
	s = calloc(1, sizeof(*s));
	if (!s)
		return NULL;
	s->base.close = afp_close;
	s->base.next = afp_next;
	s->fd = -1;
	s->ring = ring;
	s->external = 1;
	s->nblocks = nblocks;
	s->bsz = block_size;
	if (hipHostRegister(s->ring, (size_t)nblocks * block_size, hipHostRegisterDefault) == hipSuccess) {
		s->registered = 1;
		mosrx__host_range_add(s->ring, (uint64_t)nblocks * block_size);
		s->base.borrow = afp_borrow;
		s->base.give_back = afp_give_back;
	}
	return &s->base;
}

mosrx_source *mosrx_source_afpacket(const char *ifname)
{
	return mosrx_source_afpacket_ex(ifname, NULL);
}

int mosrx_source_afpacket_info(mosrx_source *s_, mosrx_afpacket_info *info)
{
	struct src_afp *s = (struct src_afp *)s_;
	if (!s_ || !info || s_->close != afp_close)
		return -EINVAL;
	struct tpacket_stats_v3 st;
	socklen_t sl = sizeof(st);
	memset(&st, 0, sizeof(st));
	if (s->fd >= 0 && getsockopt(s->fd, SOL_PACKET, PACKET_STATISTICS, &st, &sl) == 0) {   /* pcap_stats' source */
		s->ring_packets += st.tp_packets;
		s->ring_drops += st.tp_drops;
	}
	info->zero_copy = s->registered;
	info->ring_bytes = (uint64_t)s->nblocks * s->bsz;
	info->dropped_outgoing = s->dropped_outgoing;
	info->ring_packets = s->ring_packets;
	info->ring_drops = s->ring_drops;
	return 0;
}

/* ---------------- paced arrivals ---------------- */
/* A wire at a fixed frame rate in front of another source: frame k "arrives"
 * at t0 + k / rate (t0: the first receive call) and is handed out by no
 * receive before that, as a NIC ring fills at line rate.  What the backend
 * receives per call is what has arrived by then, so group sizes follow the
 * load; the latency probe (rx_loop.c) turns frame k's arrival into its
 * residency.  The inner source keeps its receive forms (fill / borrow), capped
 * at the frames that have arrived. */
struct src_paced {
	struct mosrx_source base;
	struct mosrx_source *in;
	double ns_per_frame;
	uint64_t t0_ns, released;
};

static uint64_t mono_ns(void)
{
	struct timespec ts;
	clock_gettime(CLOCK_MONOTONIC, &ts);
	return (uint64_t)ts.tv_sec * 1000000000ull + (uint64_t)ts.tv_nsec;
}

/* frames that have arrived and were not handed out yet, at most max_n */
static uint32_t paced_ready(struct src_paced *s, uint32_t max_n)
{
	uint64_t now = mono_ns(), arrived;
	if (!s->t0_ns)
		s->t0_ns = now;
	arrived = (uint64_t)((double)(now - s->t0_ns) / s->ns_per_frame) + 1;
	arrived = arrived > s->released ? arrived - s->released : 0;
	return arrived < max_n ? (uint32_t)arrived : max_n;
}

static int paced_next(struct mosrx_source *s_, uint8_t *dst, uint32_t cap)
{
	struct src_paced *s = (struct src_paced *)s_;
	int l;
	if (!paced_ready(s, 1))
		return 0;
	l = s->in->next ? s->in->next(s->in, dst, cap) : 0;
	s->released += l > 0;
	return l;
}

static uint32_t paced_fill(struct mosrx_source *s_, uint8_t *frames, uint64_t cap, uint32_t *off, uint16_t *len,
                           uint32_t max_n, uint32_t max_frame, uint64_t *end)
{
	struct src_paced *s = (struct src_paced *)s_;
	const uint32_t n = paced_ready(s, max_n);
	int k;
	*end = 2;
	if (!n)
		return 0;
	k = mosrx_source_fill(s->in, frames, cap, off, len, n, max_frame, end);
	if (k <= 0)
		return 0;
	s->released += (uint32_t)k;
	return (uint32_t)k;
}

static uint32_t paced_borrow(struct mosrx_source *s_, uint32_t max_n, uint32_t max_frame, const uint8_t **frames,
                             uint64_t *frames_bytes, uint32_t *off, uint16_t *len)
{
	struct src_paced *s = (struct src_paced *)s_;
	const uint32_t n = paced_ready(s, max_n);
	uint32_t k;
	if (!n)
		return 0;
	k = s->in->borrow(s->in, n, max_frame, frames, frames_bytes, off, len);
	s->released += k;
	return k;
}

static void paced_give_back(struct mosrx_source *s_)
{
	struct src_paced *s = (struct src_paced *)s_;
	if (s->in->give_back)
		s->in->give_back(s->in);
}

static void paced_close(struct mosrx_source *s_)
{
	struct src_paced *s = (struct src_paced *)s_;
	mosrx_source_close(s->in);
	free(s);
}

mosrx_source *mosrx_source_paced(mosrx_source *inner, double rate_pps)
{
	struct src_paced *s;
	if (!inner || !(rate_pps > 0) || inner->close == afp_close)
		return NULL;
	s = calloc(1, sizeof(*s));
	if (!s)
		return NULL;
	s->in = inner;
	s->ns_per_frame = 1e9 / rate_pps;
	s->base.next = paced_next;
	s->base.fill = paced_fill;
	if (inner->borrow) {
		s->base.borrow = paced_borrow;
		s->base.give_back = paced_give_back;
	}
	s->base.close = paced_close;
	return &s->base;
}

int mosrx_source_paced_info(const mosrx_source *s_, uint64_t *t0_ns, double *ns_per_frame, uint64_t *released)
{
	const struct src_paced *s = (const struct src_paced *)s_;
	if (!s_ || s_->close != paced_close)
		return -EINVAL;
	if (t0_ns) *t0_ns = s->t0_ns;
	if (ns_per_frame) *ns_per_frame = s->ns_per_frame;
	if (released) *released = s->released;
	return 0;
}

/* ---------------- transmit ---------------- */
/* A frame handed to send_pkts leaves through the source it belongs to: the
 * AF_PACKET socket (pcap_inject, pcap_module.c:67-79) or, when a TX dump is
 * set, a classic pcap file (any source; the only way out of a trace file). */
int mosrx_source_send(mosrx_source *s, const uint8_t *frame, uint32_t len)
{
	int rc;
	if (!s || !frame || len > 65535)
		return -EINVAL;
	if (s->tx_dump) {
		struct timespec ts;
		uint32_t rh[4];
		clock_gettime(CLOCK_REALTIME, &ts);
		rh[0] = (uint32_t)ts.tv_sec;
		rh[1] = (uint32_t)(ts.tv_nsec / 1000);
		rh[2] = rh[3] = len;
		rc = (fwrite(rh, 4, 4, s->tx_dump) == 4 && fwrite(frame, 1, len, s->tx_dump) == len) ? 0 : -EIO;
	} else {
		rc = s->send ? s->send(s, frame, len) : -EOPNOTSUPP;
	}
	if (rc) {
		s->tx_errors++;
		return rc;
	}
	s->tx_packets++;
	s->tx_bytes += len;
	return 0;
}

int mosrx_source_tx_pcap(mosrx_source *s, const char *path)
{
	static const uint32_t gh[6] = {0xa1b2c3d4u, 2u | (4u << 16), 0, 0, 65535, 1};   /* LINKTYPE_ETHERNET */
	if (!s)
		return -EINVAL;
	if (s->tx_dump) {
		fclose(s->tx_dump);
		s->tx_dump = NULL;
	}
	if (!path)
		return 0;
	s->tx_dump = fopen(path, "wb");
	if (!s->tx_dump)
		return -errno;
	if (fwrite(gh, 4, 6, s->tx_dump) != 6)
		return -EIO;
	return 0;
}

int mosrx_source_tx_flush(mosrx_source *s)
{
	if (!s)
		return -EINVAL;
	return s->tx_dump && fflush(s->tx_dump) ? -EIO : 0;
}

int mosrx_source_tx_stats(const mosrx_source *s, uint64_t *packets, uint64_t *bytes, uint64_t *errors)
{
	if (!s)
		return -EINVAL;
	if (packets) *packets = s->tx_packets;
	if (bytes) *bytes = s->tx_bytes;
	if (errors) *errors = s->tx_errors;
	return 0;
}

/* Zero-copy runs for any consumer: the backend's path (borrow/give_back) —
 * for the AF_PACKET ring also when it is not registered with the HIP runtime
 * (a host consumer needs no registration; the backend only lends registered
 * rings to the GPU copy). */
int mosrx_source_borrow(mosrx_source *s, uint32_t max_n, uint32_t max_frame, const uint8_t **frames,
                        uint64_t *frames_bytes, uint32_t *off, uint16_t *len)
{
	if (!s || !frames || !frames_bytes || !off || !len || max_frame == 0)
		return -EINVAL;
	if (s->close == afp_close)
		return (int)afp_borrow(s, max_n, max_frame, frames, frames_bytes, off, len);
	if (!s->borrow)
		return -EOPNOTSUPP;
	return (int)s->borrow(s, max_n, max_frame, frames, frames_bytes, off, len);
}

int mosrx_source_give_back(mosrx_source *s)
{
	if (!s)
		return -EINVAL;
	if (s->close == afp_close) {
		afp_give_back(s);
		return 0;
	}
	if (!s->borrow)
		return -EOPNOTSUPP;
	if (s->give_back)
		s->give_back(s);
	return 0;
}

int mosrx_source_fill(mosrx_source *s, uint8_t *dst, uint64_t cap, uint32_t *off, uint16_t *len, uint32_t max_n,
                      uint32_t max_frame, uint64_t *end)
{
	uint64_t pos = 2;
	uint32_t k = 0;
	if (!s || !dst || !off || !len || !end || max_frame == 0 || max_frame > 65535)
		return -EINVAL;
	if (s->fill)
		return (int)s->fill(s, dst, cap, off, len, max_n, max_frame, end);
	if (!s->next)
		return -EINVAL;
	while (k < max_n && pos + max_frame + 32 <= cap) {
		/* received into the aligned slot; a frame that packs moves back (mosrx__frame_at) */
		const uint64_t al = mosrx__frame_at(pos, MOSRX_PACK_MAX + 1);
		const int l = s->next(s, dst + al, max_frame);
		if (l <= 0)
			break;
		if (mosrx__frame_at(pos, (uint32_t)l) != al)
			memmove(dst + pos, dst + al, (size_t)l);
		else
			pos = al;
		off[k] = (uint32_t)pos;
		len[k] = (uint16_t)l;
		k++;
		pos += (uint64_t)l;
	}
	*end = pos;
	return (int)k;
}

int mosrx_source_next(mosrx_source *s, uint8_t *dst, uint32_t cap)
{
	if (!s || !dst || !s->next)
		return -EINVAL;
	return s->next(s, dst, cap);
}

void mosrx_source_close(mosrx_source *s)
{
	if (s && s->tx_dump) {
		fclose(s->tx_dump);
		s->tx_dump = NULL;
	}
	if (s && s->close)
		s->close(s);
}
