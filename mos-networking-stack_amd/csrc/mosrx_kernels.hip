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
//            (6 x buffer_load_dwordx4 starting at frame byte 2, so the IP header
//            sits dword-aligned in registers), parses every header field, runs
//            the ip_fast_csum carry chain, the Toeplitz hash (24 nibble-table
//            lookups in LDS) and the TCP one's-complement sum of the segment
//            bytes inside the window.  64-byte frames finish here.
//   phase 1  wave-per-frame.  Frames whose IP datagram extends past the window
//            stream the rest ("tail") with coalesced 16-byte loads, 1 KiB per
//            wave instruction, lanes summing 16-bit words on the absolute even
//            address grid; a wave reduction gives the tail sum.
//   phase 2  lane-per-frame finalisation: tail sum folded in (byte-swapped when
//            the frame starts at an odd address: 256 * x == bswap16(x) mod
//            0xFFFF), final fold/complement, verdict, one 16-byte record store.
//
// Every frame byte the reference reads is read from HBM once; the window and
// the first tail chunk overlap by at most 16 bytes (served from L1/L2).
// All loads go through a buffer resource whose range is the batch buffer, so a
// bad offset can never fault: out-of-range dwords read as zero.

#include <hip/hip_runtime.h>
#include <errno.h>
#include <stdint.h>

#include "mosrx_internal.h"

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

#define WIN_RAW 24     // raw dwords per lane window (96 B)
#define WIN_DW  23     // realigned dwords: frame bytes [2, 94)

static_assert(2 + 4 * WIN_DW == MOSRX_WINDOW_END, "window end");
static_assert(sizeof(mosrx_result) == 16, "record size");

__device__ __forceinline__ __amdgpu_buffer_rsrc_t frame_rsrc(const uint8_t *base, uint32_t nbytes)
{
	return __builtin_amdgcn_make_buffer_rsrc((void *)base, (short)0, (int)nbytes, 0x00020000);
}

// 16 bytes at byte offset c (16-aligned in the streaming phase, 4-aligned in the
// window).  A chunk that straddles the end of the buffer is assembled from byte
// loads so that in-range bytes are never dropped by the range check.
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
__device__ __forceinline__ uint32_t sum16(uint32_t d) { return (d & 0xFFFFu) + (d >> 16); }
// mask keeping bytes [0, nb) of a little-endian dword, nb in [0, 4]
__device__ __forceinline__ uint32_t keep_lo(int nb) { return nb >= 4 ? 0xFFFFFFFFu : ((1u << (8 * nb)) - 1u); }

__device__ __forceinline__ uint32_t wave_sum(uint32_t v)
{
#pragma unroll
	for (int o = 32; o >= 1; o >>= 1)
		v += __shfl_xor(v, o, 64);
	return v;
}

template <int TILE>
__global__ __launch_bounds__(256) void mosrx_classify_kernel(mosrx_kparams kp)
{
	static_assert(TILE % 64 == 0 && TILE <= 256, "tile");
	__shared__ uint32_t s_tab[MOSRX_TAB_WORDS];
	__shared__ uint32_t s_tail_lo[TILE];
	__shared__ uint32_t s_tail_hi[TILE];
	__shared__ uint32_t s_tail_sum[TILE];
	__shared__ uint64_t s_mask[TILE / 64];
	__shared__ uint32_t s_cnt[MOSRX_R_COUNT];

	const uint32_t t = threadIdx.x;
	const uint32_t lane = t & 63u;
	const uint32_t wave = t >> 6;

	// tables: RSS nibble tables + queue LUT (2 KiB, L2-resident)
	s_tab[t] = kp.tables[t];
	s_tab[t + 256] = kp.tables[t + 256];
	if (t < MOSRX_R_COUNT)
		s_cnt[t] = 0;

	const __amdgpu_buffer_rsrc_t rs = frame_rsrc(kp.frames, kp.frames_bytes);
	const uint32_t nbytes = kp.frames_bytes;

	// ---------------- phase 0: lane per frame ----------------
	const uint32_t p = blockIdx.x * TILE + t;
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

	__syncthreads();   // s_tab ready

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

	// TCP segment sum inside the window (segment grid == realigned grid).
	uint32_t wsum = 0;
#pragma unroll
	for (int j = 8; j < WIN_DW; j++) {
		int vb = (int)fend - (4 * j + 2);
		vb = vb < 0 ? 0 : (vb > 4 ? 4 : vb);
		uint32_t m = keep_lo(vb);
		if ((uint32_t)j < 3u + ihl)
			m = 0;
		wsum += sum16(w[j] & m);
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
	const bool has_tail = need_tcp && fend > (uint32_t)MOSRX_WINDOW_END;

	if (t < (uint32_t)TILE) {
		s_tail_lo[t] = o + MOSRX_WINDOW_END;
		s_tail_hi[t] = o + fend;
	}
	const uint64_t tail_mask = __ballot(has_tail);
	if (t < (uint32_t)TILE && lane == 0)
		s_mask[wave] = tail_mask;
	__syncthreads();

	// ---------------- phase 1: wave per tail ----------------
	{
		uint32_t rank = 0;
#pragma unroll 1
		for (int mw = 0; mw < TILE / 64; mw++) {
			uint64_t m = s_mask[mw];
			m = ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(m >> 32)) << 32) |
			    (uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)m);
			while (m) {
				const int b = __builtin_ctzll(m);
				m &= m - 1;
				if ((rank++ & 3u) != wave)
					continue;
				const uint32_t i = (uint32_t)(mw * 64 + b);
				const uint32_t lo = __builtin_amdgcn_readfirstlane(s_tail_lo[i]);
				const uint32_t hi = __builtin_amdgcn_readfirstlane(s_tail_hi[i]);
				uint32_t acc = 0;
#pragma unroll 1
				for (uint32_t base = lo & ~15u; base < hi; base += 1024u) {
					const uint32_t c = base + 16u * lane;
					u32x4 v = load16(rs, c < hi ? c : nbytes, nbytes);
					const int a = (int)(lo - c);   // bytes to drop at the front
					const int e = (int)(hi - c);   // bytes valid from the front
					uint32_t d[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
					for (int k = 0; k < 4; k++) {
						int lo_b = a - 4 * k; lo_b = lo_b < 0 ? 0 : (lo_b > 4 ? 4 : lo_b);
						int hi_b = e - 4 * k; hi_b = hi_b < 0 ? 0 : (hi_b > 4 ? 4 : hi_b);
						acc += sum16(d[k] & keep_lo(hi_b) & ~keep_lo(lo_b));
					}
				}
				acc = wave_sum(acc);
				if (lane == 0)
					s_tail_sum[i] = acc;
			}
		}
	}
	__syncthreads();

	// ---------------- phase 2: finalise and store ----------------
	if (active) {
		uint32_t tcpc = 0;
		if (need_tcp) {
			const uint32_t seglen = (ip_len - ihl * 4u) & 0xFFFFu;    // (doff<<2) + payloadlen, u16
			uint32_t s = wsum + sum16(saddr) + sum16(daddr) + bswap16(seglen) + 0x0600u;
			if (has_tail) {
				uint32_t ts = s_tail_sum[t];
				ts = (ts & 0xFFFFu) + (ts >> 16);
				ts = (ts & 0xFFFFu) + (ts >> 16);
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
