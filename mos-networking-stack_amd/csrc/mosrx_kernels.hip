// mosrx_kernels.hip — gfx950 kernels for mOS's receive-path per-frame transform.
//
// One launch classifies a batch: Ethernet/IPv4/TCP header extraction
// (eth_in.c:27-87, ip_in.c:30-101, tcp.c:258-270, :408-445), ip_fast_csum
// (include/ip_in.h:10-38), TCPCalcChecksum over the full segment
// (tcp_util.c:157-190) and the Toeplitz RSS hash + queue map (util.c:27-131).
// Integer byte work, HBM-bound: no MFMA.
//
// Workgroup = 256 threads (4 waves) over a tile of TILE frames:
//   phase 0  lane-per-frame.  Each lane loads a 96-byte window of its frame
//            (6 x buffer_load_dwordx4 from frame byte 2, realigned with
//            v_alignbyte so the IP header sits dword-aligned in registers),
//            parses every header field, runs the ip_fast_csum carry chain, the
//            Toeplitz hash (24 nibble-table lookups in LDS) and the TCP
//            one's-complement sum of the segment bytes up to the frame's first
//            16-byte-aligned address past byte 78 ("split").  64-byte frames
//            finish here.
//   phase 1  wave-per-frame.  Frames whose IP datagram extends past the split
//            stream the rest ("tail") with coalesced, 16-byte-aligned loads,
//            1 KiB per wave instruction; each wave keeps four tails in flight
//            (8 loads) before reducing.  Lanes sum 16-bit words on the absolute
//            even grid with v_dot2_u32_u16; only the last chunk is masked.  A
//            DPP row reduction + 4 readlanes gives each tail sum.
//   phase 2  lane-per-frame: tail sum folded in (byte-swapped when the frame
//            starts at an odd address: 256 * x == bswap16(x) mod 0xFFFF), final
//            fold/complement, verdict, one 16-byte record store.
//
// All frame loads go through a buffer resource whose range is the batch
// buffer: a bad offset can never fault, out-of-range dwords read as zero.

#include <hip/hip_runtime.h>
#include <errno.h>
#include <stdint.h>

#include "mosrx_internal.h"

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));

#define WIN_RAW 24     // raw dwords per lane window (96 B)
#define WIN_DW  23     // realigned dwords: frame bytes [2, 94)
#define TAIL_G  4      // tails in flight per wave
#define TAIL_U  2      // 1 KiB loads per tail issued up front (tails <= 2 KiB finish in one pass)

static_assert(2 + 4 * WIN_DW == MOSRX_WINDOW_END, "window end");
static_assert(sizeof(mosrx_result) == 16, "record size");

__device__ __forceinline__ __amdgpu_buffer_rsrc_t frame_rsrc(const uint8_t *base, uint32_t nbytes)
{
	return __builtin_amdgcn_make_buffer_rsrc((void *)base, (short)0, (int)nbytes, 0x00020000);
}

// 16 bytes at byte offset c.  A chunk that straddles the end of the buffer is
// assembled from byte loads so that in-range bytes are never dropped by the
// range check; offsets at or past the end read zero with no memory traffic.
__device__ __forceinline__ u32x4 load16(__amdgpu_buffer_rsrc_t r, uint32_t c, uint32_t nbytes)
{
	if (__builtin_expect(c + 16u <= nbytes || c >= nbytes, 1))
		return __builtin_amdgcn_raw_buffer_load_b128(r, c, 0, 0);
	uint32_t d[4] = {0, 0, 0, 0};
	for (uint32_t b = 0; b < 16u && c + b < nbytes; b++)
		d[b >> 2] |= (uint32_t)__builtin_amdgcn_raw_buffer_load_b8(r, c + b, 0, 0) << (8 * (b & 3));
	return (u32x4){d[0], d[1], d[2], d[3]};
}

__device__ __forceinline__ uint32_t bswap16(uint32_t x) { return ((x & 0xFFu) << 8) | ((x >> 8) & 0xFFu); }
__device__ __forceinline__ uint32_t be16hi(uint32_t w) { return ((w >> 8) & 0xFF00u) | (w >> 24); } // bytes 2,3
// acc + lo16(d) + hi16(d) in one v_dot2_u32_u16
__device__ __forceinline__ uint32_t add16x2(uint32_t acc, uint32_t d)
{
	return __builtin_amdgcn_udot2(__builtin_bit_cast(u16x2, d), (u16x2){1, 1}, acc, false);
}
// mask keeping bytes [0, nb) of a little-endian dword, nb clamped to [0, 4]
__device__ __forceinline__ uint32_t keep_lo(int nb)
{
	return nb >= 4 ? 0xFFFFFFFFu : (nb <= 0 ? 0u : ((1u << (8 * nb)) - 1u));
}
__device__ __forceinline__ uint32_t fold16(uint32_t s)
{
	s = (s & 0xFFFFu) + (s >> 16);
	return (s & 0xFFFFu) + (s >> 16);
}

// sum over the 64 lanes: 4 DPP row steps, then the four row sums via readlane
__device__ __forceinline__ uint32_t wave_sum(uint32_t v)
{
	int x = (int)v;
	x += __builtin_amdgcn_update_dpp(0, x, 0xB1, 0xF, 0xF, false);   // quad_perm [1,0,3,2]
	x += __builtin_amdgcn_update_dpp(0, x, 0x4E, 0xF, 0xF, false);   // quad_perm [2,3,0,1]
	x += __builtin_amdgcn_update_dpp(0, x, 0x141, 0xF, 0xF, false);  // row_half_mirror
	x += __builtin_amdgcn_update_dpp(0, x, 0x140, 0xF, 0xF, false);  // row_mirror
	return (uint32_t)(__builtin_amdgcn_readlane(x, 0) + __builtin_amdgcn_readlane(x, 16) +
	                  __builtin_amdgcn_readlane(x, 32) + __builtin_amdgcn_readlane(x, 48));
}

// Sum of the 16-bit words (absolute even grid) of one 16-byte chunk at c, with
// bytes at or past `hi` dropped.  c is 16-aligned.
__device__ __forceinline__ uint32_t chunk_sum(u32x4 v, uint32_t c, uint32_t hi, uint32_t acc)
{
	const int e = (int)(hi - c);              // valid bytes from the chunk start
	if (e < 16) {                             // the last chunk (or past the end: e <= 0)
		v.x &= keep_lo(e);
		v.y &= keep_lo(e - 4);
		v.z &= keep_lo(e - 8);
		v.w &= keep_lo(e - 12);
	}
	acc = add16x2(acc, v.x);
	acc = add16x2(acc, v.y);
	acc = add16x2(acc, v.z);
	return add16x2(acc, v.w);
}

template <int TILE>
__device__ __forceinline__ void classify_tile(const mosrx_kparams &kp, uint32_t tile)
{
	static_assert(TILE % 64 == 0 && TILE <= 256, "tile");
	__shared__ uint32_t s_tab[MOSRX_TAB_WORDS];
	__shared__ uint32_t s_tail_lo[TILE];
	__shared__ uint32_t s_tail_hi[TILE];
	__shared__ uint32_t s_tail_sum[TILE];
	__shared__ uint32_t s_tail_pkt[TILE];
	__shared__ uint32_t s_cnt[MOSRX_R_COUNT + 1];   // [MOSRX_R_COUNT] = number of tails

	const uint32_t t = threadIdx.x;
	const uint32_t lane = t & 63u;
	const uint32_t wave = t >> 6;

	// tables: RSS nibble tables + queue LUT (2 KiB, L2-resident)
	s_tab[t] = kp.tables[t];
	s_tab[t + 256] = kp.tables[t + 256];
	if (t <= MOSRX_R_COUNT)
		s_cnt[t] = 0;

	const __amdgpu_buffer_rsrc_t rs = frame_rsrc(kp.frames, kp.frames_bytes);
	const uint32_t nbytes = kp.frames_bytes;

	// ---------------- phase 0: lane per frame ----------------
	const uint32_t p = tile * TILE + t;
	const bool active = (t < (uint32_t)TILE) && (p < kp.n);
	uint32_t o = 0, cap = 0;
	if (active) {
		o = kp.off[p];
		cap = kp.len[p];
		cap = (o >= nbytes) ? 0u : min(cap, nbytes - o);   // eff_caplen
	}
	// window: raw dwords from (o+2)&~3, realigned to frame bytes [2+4j, 6+4j)
	const uint32_t a2 = o + 2u;
	const uint32_t wbase = active ? (a2 & ~3u) : nbytes;  // inactive lanes read out of range -> 0
	const uint32_t rsh = a2 & 3u;
	uint32_t raw[WIN_RAW];
#pragma unroll
	for (int m = 0; m < WIN_RAW / 4; m++) {
		u32x4 v = load16(rs, wbase + 16u * m, nbytes);
		raw[4 * m + 0] = v.x; raw[4 * m + 1] = v.y; raw[4 * m + 2] = v.z; raw[4 * m + 3] = v.w;
	}
	uint32_t w[WIN_DW];
#pragma unroll
	for (int j = 0; j < WIN_DW; j++)
		w[j] = __builtin_amdgcn_alignbyte(raw[j + 1], raw[j], rsh);

	__syncthreads();   // s_tab, s_cnt ready

	// header fields (frame byte f sits in byte (f-2)&3 of w[(f-2)>>2])
	const uint32_t h_proto = be16hi(w[2]);            // frame bytes 12,13  (eth_in.c:34)
	const uint32_t vi = w[3] & 0xFFu;                 // frame byte 14: version/ihl
	const uint32_t ver = vi >> 4, ihl = vi & 0xFu;
	const uint32_t ip_len = be16hi(w[3]);             // frame bytes 16,17  (ip_in.c:39)
	const uint32_t proto = (w[5] >> 8) & 0xFFu;       // frame byte 23
	const uint32_t saddr = w[6], daddr = w[7];        // raw network-order words
	uint32_t th0 = 0, th3 = 0;                         // TCP header dwords 0 and 3 at iph + ihl*4
#pragma unroll
	for (int k = 0; k < 16; k++) {
		if (ihl == (uint32_t)k) {
			th0 = w[3 + k];
			th3 = w[6 + k];
		}
	}
	const bool is_tcp = (proto == 6u);
	const uint32_t doff = is_tcp ? ((th3 >> 4) & 0xFu) : 0u;
	const uint32_t fend = 14u + ip_len;                // frame byte after the IP datagram
	// split: first 16-byte-aligned buffer offset at or below o+94 (frame byte 79..94)
	const uint32_t split_abs = (o + (uint32_t)MOSRX_WINDOW_END) & ~15u;
	const uint32_t split = split_abs - o;

	// ip_fast_csum (ip_in.h:10-38): 32-bit adc chain, final carry added once, fold, not.
	uint32_t ipc;
	{
		uint32_t s = w[3];
		if (ihl <= 4u) {
			ipc = s & 0xFFFFu;
		} else {
			uint64_t tt = (uint64_t)s + w[4];
			s = (uint32_t)tt; uint32_t c = (uint32_t)(tt >> 32);
			tt = (uint64_t)s + w[5] + c; s = (uint32_t)tt; c = (uint32_t)(tt >> 32);
			tt = (uint64_t)s + w[6] + c; s = (uint32_t)tt; c = (uint32_t)(tt >> 32);
#pragma unroll
			for (int k = 4; k < 15; k++) {
				tt = (uint64_t)s + w[3 + k] + c;
				if ((uint32_t)k < ihl) { s = (uint32_t)tt; c = (uint32_t)(tt >> 32); }
			}
			s += c;
			const uint32_t a = (s >> 16) + (s & 0xFFFFu);
			const uint32_t rr = (a & 0xFFFFu) + (a >> 16);
			ipc = (~rr) & 0xFFFFu;
		}
	}

	// TCP segment sum over frame bytes [14+4*ihl, min(fend, split)) (segment grid
	// == realigned grid, dword j holds frame bytes [4j+2, 4j+6)).
	uint32_t wsum = 0;
	{
		const int wend = (int)min(fend, split);
#pragma unroll
		for (int j = 8; j < WIN_DW; j++) {
			uint32_t m = keep_lo(wend - (4 * j + 2));
			if ((uint32_t)j < 3u + ihl)
				m = 0;
			wsum = add16x2(wsum, w[j] & m);
		}
	}

	// Toeplitz over saddr|daddr|sport|dport in wire order (util.c:61-99 with host-order args)
	uint32_t rss = 0;
	{
		const uint32_t tup[3] = {saddr, daddr, is_tcp ? th0 : 0u};
#pragma unroll
		for (int k = 0; k < 12; k++) {
			const uint32_t b = (tup[k >> 2] >> (8 * (k & 3))) & 0xFFu;
			rss ^= s_tab[(2 * k) * 16 + (b >> 4)] ^ s_tab[(2 * k + 1) * 16 + (b & 0xFu)];
		}
	}
	const uint32_t queue = (s_tab[MOSRX_TAB_RSS_WORDS + ((rss & 0x1FFu) >> 2)] >> (8 * (rss & 3u))) & 0xFFu;

	// ---------------- verdict chain (eth_in.c:27 -> ip_in.c:30 -> tcp.c:408) ----------------
	const bool verify = kp.flags & MOSRX_KF_VERIFY;
	int verdict = -1;
	uint32_t reason = MOSRX_R_TRUNCATED;
	bool fields = false, need_tcp = false;
	if (cap < 14u) {
		verdict = -1; reason = MOSRX_R_TRUNCATED;
	} else if (h_proto != 0x0800u) {
		reason = (h_proto == 0x0806u) ? MOSRX_R_ARP : MOSRX_R_NON_IPV4;
		verdict = ((kp.flags & MOSRX_KF_FWD_NONIP) || h_proto == 0x0806u) ? 1 : -1;
	} else if (cap < 34u || 14u + ihl * 4u > cap || fend > cap || (is_tcp && 14u + ihl * 4u + 20u > cap)) {
		verdict = -1; reason = MOSRX_R_TRUNCATED;
	} else if (ip_len < 20u) {
		verdict = -1; reason = MOSRX_R_IP_SHORT;
	} else if (ver != 4u) {
		verdict = 0; reason = MOSRX_R_IP_BADVER;
	} else {
		fields = true;
		if (!verify) {
			verdict = 1; reason = MOSRX_R_NOVERIFY_PASS;
		} else if (ipc != 0u) {
			verdict = -1; reason = MOSRX_R_IP_BADCSUM;
		} else if (!is_tcp) {
			verdict = 0; reason = MOSRX_R_NOT_TCP;
		} else if (ip_len < (ihl + doff) * 4u) {
			verdict = -1; reason = MOSRX_R_TCP_SHORT;
		} else if (kp.flags & MOSRX_KF_SKIP_TCP) {
			verdict = 1; reason = MOSRX_R_TCP_LEN_OK;
		} else {
			need_tcp = true;   // verdict decided after the tail sum
		}
	}
	if (!active)
		need_tcp = false;
	const bool has_tail = need_tcp && fend > split;
	if (has_tail) {
		const uint32_t k = atomicAdd(&s_cnt[MOSRX_R_COUNT], 1u);
		s_tail_pkt[k] = t;
		s_tail_lo[k] = split_abs;
		s_tail_hi[k] = o + fend;
	}
	__syncthreads();

	// ---------------- phase 1: wave per tail, TAIL_G tails in flight ----------------
	{
		const uint32_t ntail = __builtin_amdgcn_readfirstlane(s_cnt[MOSRX_R_COUNT]);
#pragma unroll 1
		for (uint32_t k0 = wave * TAIL_G; k0 < ntail; k0 += 4u * TAIL_G) {
			uint32_t lo[TAIL_G], hi[TAIL_G], acc[TAIL_G];
			u32x4 v[TAIL_G][TAIL_U];
#pragma unroll
			for (int u = 0; u < TAIL_G; u++) {
				const bool ok = k0 + u < ntail;
				lo[u] = ok ? __builtin_amdgcn_readfirstlane(s_tail_lo[k0 + u]) : 0u;
				hi[u] = ok ? __builtin_amdgcn_readfirstlane(s_tail_hi[k0 + u]) : 0u;
#pragma unroll
				for (int q = 0; q < TAIL_U; q++) {
					const uint32_t c = lo[u] + 1024u * q + 16u * lane;
					v[u][q] = load16(rs, c < hi[u] ? c : nbytes, nbytes);
				}
			}
#pragma unroll
			for (int u = 0; u < TAIL_G; u++) {
				acc[u] = 0;
#pragma unroll
				for (int q = 0; q < TAIL_U; q++)
					acc[u] = chunk_sum(v[u][q], lo[u] + 1024u * q + 16u * lane, hi[u], acc[u]);
				// jumbo tails: the rest, 1 KiB per step
#pragma unroll 1
				for (uint32_t base = lo[u] + 1024u * TAIL_U; base < hi[u]; base += 1024u) {
					const uint32_t c = base + 16u * lane;
					acc[u] = chunk_sum(load16(rs, c < hi[u] ? c : nbytes, nbytes), c, hi[u], acc[u]);
				}
			}
#pragma unroll
			for (int u = 0; u < TAIL_G; u++) {
				const uint32_t s = wave_sum(acc[u]);
				if (k0 + u < ntail && lane == 0)
					s_tail_sum[__builtin_amdgcn_readfirstlane(s_tail_pkt[k0 + u])] = s;
			}
		}
	}
	__syncthreads();

	// ---------------- phase 2: finalise and store ----------------
	if (active) {
		uint32_t tcpc = 0;
		if (need_tcp) {
			const uint32_t seglen = (ip_len - ihl * 4u) & 0xFFFFu;    // (doff<<2) + payloadlen, u16
			uint32_t s = wsum + (saddr & 0xFFFFu) + (saddr >> 16) + (daddr & 0xFFFFu) + (daddr >> 16) +
			             bswap16(seglen) + 0x0600u;
			if (has_tail) {
				const uint32_t ts = fold16(s_tail_sum[t]);
				s += (o & 1u) ? bswap16(ts) : ts;
			}
			s = (s >> 16) + (s & 0xFFFFu);
			s += s >> 16;
			tcpc = (~s) & 0xFFFFu;
			verdict = tcpc ? -1 : 1;
			reason = tcpc ? MOSRX_R_TCP_BADCSUM : MOSRX_R_TCP_OK;
		}
		uint32_t r_rss = 0, r_ipc = 0, r_plen = 0, r_poff = 0, r_q = 0, r_flags = 0, r_ihld = 0;
		if (fields) {
			r_rss = rss;
			r_q = queue;
			r_ihld = (ihl << 4) | doff;
			if (verify)
				r_ipc = ipc;
			if (is_tcp) {
				r_flags = (th3 >> 8) & 0xFFu;
				r_plen = (ip_len - (ihl * 4u + doff * 4u)) & 0xFFFFu;   // tcp.c:262
				r_poff = 14u + ihl * 4u + doff * 4u;
			}
		}
		u32x4 rec;
		rec.x = r_rss;
		rec.y = r_ipc | (tcpc << 16);
		rec.z = r_plen | (r_poff << 16) | (((uint32_t)verdict & 0xFFu) << 24);
		rec.w = reason | (r_q << 8) | (r_flags << 16) | (r_ihld << 24);
		*reinterpret_cast<u32x4 *>(kp.out + p) = rec;
		if (kp.counters)
			atomicAdd(&s_cnt[reason], 1u);
	}
	if (kp.counters) {
		__syncthreads();
		if (t < MOSRX_R_COUNT && s_cnt[t])
			atomicAdd(&kp.counters[t], s_cnt[t]);
	}
}

template <int TILE>
__global__ __launch_bounds__(256) void mosrx_classify_kernel(mosrx_kparams kp)
{
	classify_tile<TILE>(kp, blockIdx.x);
}

// Batch queue: one launch over nb resident batches (descriptor table in HBM).
// Workgroup b finds its batch by a binary search of tile_base[] (scalar loads).
template <int TILE>
__global__ __launch_bounds__(256) void mosrx_classify_queue_kernel(mosrx_qparams qp)
{
	const uint32_t b = blockIdx.x;
	uint32_t lo = 0, hi = qp.nb;               // find k: tile_base[k] <= b < tile_base[k+1]
	while (hi - lo > 1) {
		const uint32_t mid = (lo + hi) >> 1;
		if (__builtin_amdgcn_readfirstlane(qp.desc[mid].tile_base) <= b)
			lo = mid;
		else
			hi = mid;
	}
	const mosrx_qdesc *d = &qp.desc[lo];
	mosrx_kparams kp;
	kp.frames = d->frames;
	kp.off = d->off;
	kp.len = d->len;
	kp.out = d->out;
	kp.tables = qp.tables;
	kp.counters = qp.counters;
	kp.frames_bytes = d->frames_bytes;
	kp.n = d->n;
	kp.flags = qp.flags;
	kp.pad = 0;
	classify_tile<TILE>(kp, b - d->tile_base);
}

extern "C" int mosrx_launch_queue(const mosrx_qparams *qp, uint32_t total_tiles, int tile, void *stream)
{
	if (!qp || qp->nb == 0 || total_tiles == 0)
		return qp ? 0 : -EINVAL;
	const hipStream_t s = (hipStream_t)stream;
	if (tile == MOSRX_TILE_SMALL)
		hipLaunchKernelGGL(mosrx_classify_queue_kernel<MOSRX_TILE_SMALL>, dim3(total_tiles), dim3(256), 0, s, *qp);
	else
		hipLaunchKernelGGL(mosrx_classify_queue_kernel<MOSRX_TILE_LARGE>, dim3(total_tiles), dim3(256), 0, s, *qp);
	return hipGetLastError() == hipSuccess ? 0 : -EIO;
}

extern "C" int mosrx_launch_classify(const mosrx_kparams *kp, int tile, void *stream)
{
	if (!kp || kp->n == 0)
		return kp ? 0 : -EINVAL;
	const hipStream_t s = (hipStream_t)stream;
	if (tile == MOSRX_TILE_SMALL) {
		const dim3 grid((kp->n + MOSRX_TILE_SMALL - 1) / MOSRX_TILE_SMALL);
		hipLaunchKernelGGL(mosrx_classify_kernel<MOSRX_TILE_SMALL>, grid, dim3(256), 0, s, *kp);
	} else {
		const dim3 grid((kp->n + MOSRX_TILE_LARGE - 1) / MOSRX_TILE_LARGE);
		hipLaunchKernelGGL(mosrx_classify_kernel<MOSRX_TILE_LARGE>, grid, dim3(256), 0, s, *kp);
	}
	return hipGetLastError() == hipSuccess ? 0 : -EIO;
}
