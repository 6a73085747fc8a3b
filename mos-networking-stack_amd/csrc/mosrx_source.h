/* mosrx_source.h — internal: the frame-source vtable behind mosrx_source_* */
#ifndef MOSRX_SOURCE_H
#define MOSRX_SOURCE_H

#include <stdint.h>
#include <stdio.h>

/* The staging layout: frames in arrival order; a frame of up to
 * MOSRX_PACK_MAX bytes right after the previous one (the 64 B configs read 60
 * bytes per frame instead of 64: 6 % fewer bytes over PCIe and from HBM; the
 * kernels take any alignment, the S64 packed row of bench.py), a longer one
 * at the next 16-byte boundary + 2 (its IP header 16-byte aligned, its tail
 * streamed from aligned chunks).  Returns where a frame of `len` bytes goes
 * when the previous one ended at `pos`. */
#ifndef MOSRX_PACK_MAX
#define MOSRX_PACK_MAX 128u
#endif
static inline uint64_t mosrx__frame_at(uint64_t pos, uint32_t len)
{
	return len <= MOSRX_PACK_MAX ? pos : ((pos - 2 + 15) & ~15ull) + 2;
}

struct mosrx_source {
	/* write the next frame into dst (at most cap bytes); returns its caplen, 0 when none */
	int  (*next)(struct mosrx_source *s, uint8_t *dst, uint32_t cap);
	void (*close)(struct mosrx_source *s);
	/* optional batch form (NULL: the backend calls next per frame): receive up
	 * to max_n frames of at most max_frame bytes into frames[] in the staging
	 * layout (first frame at byte 2, each next one where mosrx__frame_at puts
	 * it, never past cap - 16), writing off[]/len[]; returns the count and the
	 * staging bytes used in *end */
	uint32_t (*fill)(struct mosrx_source *s, uint8_t *frames, uint64_t cap, uint32_t *off, uint16_t *len,
	                 uint32_t max_n, uint32_t max_frame, uint64_t *end);
	/* optional zero-copy form (NULL: none): hand out up to max_n frames that
	 * already sit in pinned memory the source owns, as one run starting at
	 * *frames, in buffer order, writing off[]/len[] (len clamped to max_frame)
	 * and the run's length in *frames_bytes; the bytes stay valid and
	 * unmodified until give_back releases the run (or, without give_back,
	 * until the source is closed) */
	uint32_t (*borrow)(struct mosrx_source *s, uint32_t max_n, uint32_t max_frame, const uint8_t **frames,
	                   uint64_t *frames_bytes, uint32_t *off, uint16_t *len);
	/* optional: release the OLDEST run borrow handed out that is not yet
	 * released (runs come back in the order they were borrowed), e.g. return a
	 * PACKET_MMAP ring's blocks to the kernel */
	void (*give_back)(struct mosrx_source *s);
	/* optional native transmit of one frame (pcap_inject, pcap_module.c:67-79):
	 * 0 or -errno */
	int  (*send)(struct mosrx_source *s, const uint8_t *frame, uint32_t len);
	/* generic TX sink (mosrx_source_tx_pcap): when set, sent frames are
	 * appended to this pcap file instead of the native transmit */
	FILE    *tx_dump;
	uint64_t tx_packets, tx_bytes, tx_errors;
};

/* Pinned host ranges the library knows (mosrx_host_alloc, the sources' pinned
 * replay buffers and registered rings): host regions are merged into one
 * PCIe copy only when one known range holds them all, so a copy never spans
 * two allocations or the gap between them (mosrx_api.c group_copy /
 * batch_span).  range_of: the range's id, 0 when no known range holds
 * [p, p + len). */
void     mosrx__host_range_add(const void *p, uint64_t len);
void     mosrx__host_range_del(const void *p);
uint64_t mosrx__host_range_of(const void *p, uint64_t len);

#endif
