// mosrx_kernels.hip — gfx950 kernels for mOS's receive-path per-frame transform.
//
// One launch classifies a batch: Ethernet/IPv4/TCP header extraction
// (eth_in.c:27-87, ip_in.c:30-101, tcp.c:258-270, :408-445), ip_fast_csum
// (include/ip_in.h:10-38), TCPCalcChecksum over the full segment
// (tcp_util.c:157-190) and the Toeplitz RSS hash + queue map (util.c:27-131).
// Integer byte work, HBM-bound: no MFMA.
//
// Header work is lane-per-frame ("hdr" below): each lane loads a window of its
// frame from byte 2 (5 x buffer_load_dwordx4 in the SMALL tile, 4 in the stream
// tile, the full 6 = frame bytes [2, 94) for a wave holding IP options or a
// fused BPF set), realigned with v_alignbyte so the IP header sits
// dword-aligned in registers, then parses every field, runs the ip_fast_csum
// carry chain, the Toeplitz hash (24 nibble-table lookups in LDS) and the TCP
// one's-complement sum of the segment bytes in the window: all of them when the
// datagram ends inside it (64-byte frames do), else those before the frame's
// "split", the first 16-byte-aligned buffer offset at or below the window end.
//
// Bytes past the split (the "tail") are streamed by whole waves with
// coalesced 16-byte-aligned loads, 1 KiB per wave instruction, summed as
// 16-bit words on the absolute even address grid with v_dot2_u32_u16 and
// reduced with DPP row steps + 4 readlanes.  The segment-grid sum is the
// absolute-grid sum, byte-swapped when the frame starts at an odd address
// (256 * x == bswap16(x) mod 0xFFFF).
//
// Tile shapes ("kinds", mosrx_internal.h; the tuning shapes live in scripts/):
//   small (MOSRX_SMALL_FRAMES per workgroup of 4 waves): every lane owns one or
//     more frames and finishes them in registers (batches whose frames all end
//     inside the window: the 64-byte configs); a longer frame, only when the
//     shape is forced onto it, is summed by its wave.
//   stream (TILE 64, any batch with longer frames): one header wave parses
//     while three streamer waves read the tile's tail span in buffer order as
//     plain contiguous 1 KiB wave loads and attribute the bytes to tails with
//     one prefix scan per block.

// All frame loads go through a buffer resource whose range is the batch
// buffer: a bad offset can never fault, out-of-range dwords read as zero.

#ifndef __HIPCC_RTC__   // hipRTC compiles this file too, for the fused classify + BPF kernel (bpf_jit.c)
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <errno.h>
#endif

#include "mosrx_device.h"

typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));

#define WIN_RAW 24     // raw dwords a lane window holds at most (96 B)
#define WIN_DW  23     // realigned dwords: frame bytes [2, 94)
// realigned dwords and 16-byte loads of a window ending at frame byte `wend`
#define WIN_NDW(wend)   (((wend) - 2) / 4)
#define WIN_NLOAD(wend) ((WIN_NDW(wend) + 1 + 3) / 4)

static_assert(2 + 4 * WIN_DW == MOSRX_WINDOW_END_FULL, "window end");
static_assert(WIN_NLOAD(MOSRX_WINDOW_END_SMALL) == 5 && WIN_NLOAD(MOSRX_WINDOW_END_STREAM) == 4, "window loads");
static_assert(sizeof(mosrx_result) == 16, "record size");
static_assert(sizeof(mosrx_qdesc) == 64, "queue descriptor size");
// small: 4 waves, one frame per lane; stream: 1 header wave + MOSRX_STREAMERS streamer waves
#define SMALL_THREADS (MOSRX_SMALL_FRAMES < 256u ? MOSRX_SMALL_FRAMES : 256u)
#define WG_THREADS(kind) ((kind) == MOSRX_KIND_SMALL ? SMALL_THREADS : 64 * (1 + MOSRX_STREAMERS))


// 16 bytes at byte offset c (OOB offsets read zero).  No data-dependent branch:
// the compiler can then count outstanding loads (s_waitcnt vmcnt(N)) across groups.
// AUX = cache policy (0 default, 2 = non-temporal).  Kernel variant VAR picks it
// per access class: bit 0 the header windows, bit 1 the tail stream.
template <int AUX>
__device__ __forceinline__ u32x4 load16(__amdgpu_buffer_rsrc_t r, uint32_t c, uint32_t nbytes)
{
	(void)nbytes;
	return __builtin_amdgcn_raw_buffer_load_b128(r, c, 0, AUX);
}
#define WIN_AUX(v)  (((v) & 1) ? 2 : 0)
#define TAIL_AUX(v) (((v) & 2) ? 2 : 0)
// Variant bit 4: TX checksum fill (mosrx_tx_csum_dev) instead of classification.
#define VAR_TX 16
#define IS_TX(v) (((v) & VAR_TX) != 0)
// Variant bit 5: BPF program set fused into the header wave (hipRTC builds only, bpf_jit.c).
#define VAR_BPF 32
// Variant bit 6: also write pkt_info's TCP fields (mosrx_tcpinfo side array, kp.tinfo).
#define VAR_TI 64
#define IS_TI(v) (((v) & VAR_TI) != 0)
// Variant bit 7: 8-byte records (mosrx_result8) into kp.out instead of 16-byte ones.
#define VAR_C8 128
#define IS_C8(v) (((v) & VAR_C8) != 0)
static_assert(sizeof(mosrx_result8) == 8, "compact record size");
// Variant bit 8: the batch's uniform-layout hint (kp.uni) is used by the SMALL
// tile: window loads at the hinted address leave with the descriptor loads.
#define VAR_UNI 256
#define IS_UNI(v) (((v) & VAR_UNI) != 0)

__device__ __forceinline__ uint32_t bswap16(uint32_t x) { return ((x & 0xFFu) << 8) | ((x >> 8) & 0xFFu); }
__device__ __forceinline__ uint32_t be16hi(uint32_t w) { return ((w >> 8) & 0xFF00u) | (w >> 24); } // bytes 2,3
// acc + lo16(d) + hi16(d) in one v_dot2_u32_u16
__device__ __forceinline__ uint32_t add16x2(uint32_t acc, uint32_t d)
{
	return __builtin_amdgcn_udot2(__builtin_bit_cast(u16x2, d), (u16x2){1, 1}, acc, false);
}
// mask keeping the low 32 - sh bits, sh clamped to [0, 32]: v_med3 + one 64-bit
// shift (sh == 32 gives 0), no compares, no lane-mask hazards
__device__ __forceinline__ uint32_t keep_bits(int sh)
{
	return (uint32_t)(0xFFFFFFFFull >> min(max(sh, 0), 32));
}
// mask keeping bytes [0, nb) of a little-endian dword, nb clamped to [0, 4]
__device__ __forceinline__ uint32_t keep_lo(int nb) { return keep_bits(32 - 8 * nb); }
__device__ __forceinline__ uint32_t fold16(uint32_t s)
{
	s = (s & 0xFFFFu) + (s >> 16);
	return (s & 0xFFFFu) + (s >> 16);
}

#define ZERO_OFF 0xFFFFFFF0u   // buffer offset past any batch (loads there are never consumed)

// Wave-uniform value: readfirstlane tells the compiler it lives in an SGPR.
__device__ __forceinline__ uint32_t uni(uint32_t x) { return __builtin_amdgcn_readfirstlane(x); }

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
	const int e = hi > c ? (int)min(hi - c, 16u) : 0;   // valid bytes from the chunk start
	if (e < 16) {                             // the last chunk (or past the end: e == 0)
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

// ---------------------------------------------------------------------------
// Per-frame header state (lane per frame)
// ---------------------------------------------------------------------------
struct hdr_t {
	uint32_t o, fend, split_abs;
	uint32_t wsum;                 // segment-grid sum of the segment bytes in the window (before the split)
	uint32_t saddr, daddr, ip_len, ihl, doff, th0, th3;
	uint32_t th1, th2;             // TI: TCP header dwords 1, 2 (seq, ack_seq; network order)
	uint32_t rss, queue, ipc, reason;
	uint32_t tcw, ipc_tx;          // TX: segment-grid TCP check word, IP checksum with check = 0
	int verdict;
	bool fields, need_tcp, has_tail, is_tcp, tx_ip;
	uint32_t bmatch;               // BPF: the fused set's match mask (VAR_BPF)
};

struct hdr_win_t {
	uint32_t raw[WIN_RAW];
};

template <int AUX, int NLOAD = WIN_RAW / 4>
__device__ __forceinline__ void hdr_load(__amdgpu_buffer_rsrc_t rs, uint32_t nbytes, uint32_t o, bool active,
                                         hdr_win_t &win)
{
	const uint32_t wbase = active ? ((o + 2u) & ~3u) : nbytes;   // inactive lanes read out of range -> 0
#pragma unroll
	for (int m = NLOAD; m < WIN_RAW / 4; m++)
		win.raw[4 * m + 0] = win.raw[4 * m + 1] = win.raw[4 * m + 2] = win.raw[4 * m + 3] = 0;
#pragma unroll
	for (int m = 0; m < NLOAD; m++) {
		u32x4 v = load16<AUX>(rs, wbase + 16u * m, nbytes);
		win.raw[4 * m + 0] = v.x; win.raw[4 * m + 1] = v.y; win.raw[4 * m + 2] = v.z; win.raw[4 * m + 3] = v.w;
	}
}

#ifdef MOSRX_RTC_BPF
#include "mosrx_bpf_hook.h"   // generated by bpf_jit.c: mosrx_bpf_hook(w, o, cap, live, rs), MOSRX_BPF_WEND
#endif
// The window a fused set reads from registers (bpf_jit.c hook_wend): the BPF
// tiles load at least up to it.
#ifndef MOSRX_BPF_WEND
#define MOSRX_BPF_WEND MOSRX_WINDOW_END_FULL
#endif
#define BPF_NLOAD(wend) (WIN_NLOAD(wend) > WIN_NLOAD(MOSRX_BPF_WEND) ? WIN_NLOAD(wend) : WIN_NLOAD(MOSRX_BPF_WEND))

// ip_fast_csum (ip_in.h:10-38) over the realigned header (w[3] = IP dword 0):
// 32-bit adc chain, the final carry added once (its own carry lost), fold, not.
// w5 stands in for IP dword 2 (it carries the check field).
__device__ __forceinline__ uint32_t ip_chain(const uint32_t *w, uint32_t ihl, uint32_t w5)
{
	uint32_t s = w[3];
	if (ihl <= 4u)
		return s & 0xFFFFu;
	unsigned int c;   // v_add_co / v_addc_co chain, carry in VCC
	s = __builtin_addc(s, w[4], 0u, &c);
	s = __builtin_addc(s, w5, c, &c);
	s = __builtin_addc(s, w[6], c, &c);
#pragma unroll
	for (int k = 4; k < 15; k++) {
		unsigned int c2;
		const uint32_t t = __builtin_addc(s, w[3 + k], c, &c2);
		if ((uint32_t)k < ihl) { s = t; c = c2; }
	}
	s += c;
	const uint32_t a = (s >> 16) + (s & 0xFFFFu);
	const uint32_t rr = (a & 0xFFFFu) + (a >> 16);
	return (~rr) & 0xFFFFu;
}

// The ihl-dependent header pieces: TCP header dwords 0 and 3 at iph + ihl*4
// (and the check word for TX), ip_fast_csum (and its TX variant with the check
// zeroed) and the segment sum over frame bytes [14+4*ihl, wend) on the
// realigned grid (dword j = frame bytes [4j+2, 4j+6), the segment grid).  F5:
// every active lane of the wave has ihl == 5 (no IP options, nearly all
// traffic), so every position is a constant and the selects fold away; the
// window holds NDW dwords.  Otherwise the full 23 are there, and a segment that
// starts past wend (IP options beyond the split) has the bytes [wend, 14+4*ihl)
// -- which the tail streamers sum -- taken out again: their one's-complement
// negation 0xFFFF - fold(x) is added (the final fold only sees the sum mod
// 0xFFFF, and the pseudo header keeps it positive).
template <int VAR, bool F5, int NDW>
__device__ __forceinline__ void hdr_ihl(const uint32_t (&w)[WIN_DW], uint32_t ihl_l, int wend, uint32_t &th0,
                                        uint32_t &th3, uint32_t &tcw, uint32_t &ipc, uint32_t &ipc_tx,
                                        uint32_t &wsum, uint32_t &th1, uint32_t &th2)
{
	const uint32_t ihl = F5 ? 5u : ihl_l;
	th0 = 0; th3 = 0; tcw = 0; th1 = 0; th2 = 0;
#pragma unroll
	for (int k = 0; k < 16; k++) {
		if (ihl == (uint32_t)k) {
			th0 = w[3 + k];
			th3 = w[6 + k];
			if (IS_TX(VAR))
				tcw = w[7 + k] & 0xFFFFu;                  // tcph->check (frame bytes 30+4ihl, +1)
			if (IS_TI(VAR)) {
				th1 = w[4 + k];                             // tcph->seq
				th2 = w[5 + k];                             // tcph->ack_seq
			}
		}
	}
	ipc = ip_chain(w, ihl, w[5]);
	// TX: iph->check = 0 first (mos_api.c:1180-1181): the check is frame bytes 24,25 = w[5] bytes 2,3
	ipc_tx = IS_TX(VAR) ? ip_chain(w, ihl, w[5] & 0xFFFFu) : 0u;
	const int u = 8 * wend;
	if constexpr (F5) {
		wsum = 0;
#pragma unroll
		for (int j = 8; j < NDW; j++)
			wsum = add16x2(wsum, w[j] & keep_bits(32 * j + 48 - u));   // keep_lo(wend - (4j + 2))
	} else {
		uint32_t pos = 0, neg = 0;
#pragma unroll
		for (int j = 8; j < WIN_DW; j++) {
			const uint32_t keep = keep_bits(32 * j + 48 - u);
			const bool inseg = (uint32_t)j >= 3u + ihl;
			pos = add16x2(pos, w[j] & (inseg ? keep : 0u));
			neg = add16x2(neg, w[j] & (inseg ? 0u : ~keep));
		}
		wsum = pos + (0xFFFFu - fold16(neg));
	}
}

// verdict + 1 of every reason code, 2 bits per code (eth_in.c:27-87, ip_in.c:30-101, tcp.c:408-445)
#define VT(r, v) ((uint32_t)((v) + 1) << (2 * (r)))
#define VERDICT_TAB                                                                                                    \
	(VT(MOSRX_R_TCP_OK, 1) | VT(MOSRX_R_ARP, 1) | VT(MOSRX_R_NON_IPV4, -1) | VT(MOSRX_R_IP_SHORT, -1) |                \
	 VT(MOSRX_R_IP_BADVER, 0) | VT(MOSRX_R_NOVERIFY_PASS, 1) | VT(MOSRX_R_IP_BADCSUM, -1) | VT(MOSRX_R_NOT_TCP, 0) |   \
	 VT(MOSRX_R_TCP_SHORT, -1) | VT(MOSRX_R_TCP_BADCSUM, -1) | VT(MOSRX_R_TRUNCATED, -1) | VT(MOSRX_R_TCP_LEN_OK, 1) | \
	 VT(MOSRX_R_ICMP_LOCAL, 1))
static_assert(MOSRX_R_COUNT <= 16, "verdict table holds 16 codes");

// Parse + checks + IP checksum + RSS + in-window TCP sum.  Mirrors
// ProcessPacket (eth_in.c:27) -> ProcessInIPv4Packet (ip_in.c:30) ->
// ProcessInTCPPacket prefix (tcp.c:408-445); see oracle/mosrx_oracle.c.
// WEND: the window end of the tile (MOSRX_WINDOW_END_*); `win` holds
// WIN_NLOAD(WEND) chunks, the rest are read here for a wave with IP options.
// RSS (probe builds only, the library uses 0): 0 the 24 nibble tables in LDS,
// 1 no Toeplitz at all (wrong hashes: the bound of any faster form), 2 twelve
// byte tables (12 KiB) in LDS after the library's words, 3 the same twelve
// read from global memory (kp.tables + MOSRX_TAB8_OFF) without staging.
#define MOSRX_TAB8_OFF 1024
template <int VAR, int WEND, int RSS = 0>
__device__ __forceinline__ hdr_t hdr_parse(hdr_win_t win, uint32_t o, uint32_t cap, bool active, uint32_t kflags,
                                           const uint32_t *s_tab, const uint32_t *g_tab, __amdgpu_buffer_rsrc_t rs,
                                           uint32_t nbytes)
{
	constexpr int NDW = WIN_NDW(WEND), NLOAD = WIN_NLOAD(WEND);
	// a fused BPF set reads the realigned window up to MOSRX_BPF_WEND (the tile loaded it)
	constexpr int NDW_R = (VAR & VAR_BPF) && WIN_NDW(MOSRX_BPF_WEND) > NDW ? WIN_NDW(MOSRX_BPF_WEND) : NDW;
	hdr_t h;
	uint32_t w[WIN_DW];
	const uint32_t rsh = (o + 2u) & 3u;
#pragma unroll
	for (int j = 0; j < NDW_R; j++)
		w[j] = __builtin_amdgcn_alignbyte(win.raw[j + 1], win.raw[j], rsh);
	h.bmatch = 0;
#ifdef MOSRX_RTC_BPF
	// the set first, on the registers the parse is about to read: no second
	// realignment, and the raw window is dead from here on
	if constexpr ((VAR & VAR_BPF) != 0)
		h.bmatch = mosrx_bpf_hook<WEND == MOSRX_WINDOW_END_SMALL ? SMALL_THREADS : 64u>(w, o, cap, active, rs);
#endif

	// frame byte f sits in byte (f-2)&3 of w[(f-2)>>2]
	const uint32_t h_proto = be16hi(w[2]);            // frame bytes 12,13  (eth_in.c:34)
	const uint32_t vi = w[3] & 0xFFu;                 // frame byte 14: version/ihl
	const uint32_t ver = vi >> 4, ihl = vi & 0xFu;
	const uint32_t ip_len = be16hi(w[3]);             // frame bytes 16,17  (ip_in.c:39)
	const uint32_t proto = (w[5] >> 8) & 0xFFu;       // frame byte 23
	const uint32_t saddr = w[6], daddr = w[7];        // raw network-order words
	const bool is_tcp = (proto == 6u);
	const uint32_t fend = 14u + ip_len;                // frame byte after the IP datagram
	const uint32_t split_abs = (o + (uint32_t)WEND) & ~15u;
	const uint32_t split = split_abs - o;              // frame byte WEND-15 .. WEND
	// TCP segment sum over frame bytes [14+4*ihl, wend): the whole segment when
	// the datagram ends inside the window, else up to the split (the tail
	// streamers take over there).
	const bool in_win = fend <= (uint32_t)WEND;
	const int wend = (int)(in_win ? fend : split);
	uint32_t th0, th3, tcw, ipc, ipc_tx, wsum, th1, th2;
	if (__ballot(active && ihl != 5u) == 0) {          // no IP options in the wave: constant positions
		hdr_ihl<VAR, true, NDW>(w, ihl, wend, th0, th3, tcw, ipc, ipc_tx, wsum, th1, th2);
	} else {
		if constexpr (NLOAD < WIN_RAW / 4) {           // the rest of the full window (rare)
			const uint32_t wbase = active ? ((o + 2u) & ~3u) : nbytes;
#pragma unroll
			for (int m = NLOAD; m < WIN_RAW / 4; m++) {
				const u32x4 v = load16<0>(rs, wbase + 16u * m, nbytes);
				win.raw[4 * m + 0] = v.x; win.raw[4 * m + 1] = v.y; win.raw[4 * m + 2] = v.z; win.raw[4 * m + 3] = v.w;
			}
		}
#pragma unroll
		for (int j = NDW; j < WIN_DW; j++)
			w[j] = __builtin_amdgcn_alignbyte(win.raw[j + 1], win.raw[j], rsh);
		hdr_ihl<VAR, false, WIN_DW>(w, ihl, wend, th0, th3, tcw, ipc, ipc_tx, wsum, th1, th2);
	}
	const uint32_t doff = is_tcp ? ((th3 >> 4) & 0xFu) : 0u;

	// Toeplitz over saddr|daddr|sport|dport in wire order (util.c:61-99, host-order args)
	uint32_t rss = 0;
	if constexpr (RSS == 1) {
		rss = saddr ^ daddr ^ (is_tcp ? th0 : 0u);
	} else if constexpr (RSS >= 2) {
		const uint32_t tup[3] = {saddr, daddr, is_tcp ? th0 : 0u};
		const uint32_t *t8 = RSS == 2 ? s_tab + MOSRX_TAB_WORDS : g_tab + MOSRX_TAB8_OFF;
#pragma unroll
		for (int d = 0; d < 3; d++)
#pragma unroll
			for (int b = 0; b < 4; b++)
				rss ^= t8[(4 * d + b) * 256 + ((tup[d] >> (8 * b)) & 0xFFu)];
	} else {
		const uint32_t tup[3] = {saddr, daddr, is_tcp ? th0 : 0u};
		const char *tb = reinterpret_cast<const char *>(s_tab);
#pragma unroll
		for (int d = 0; d < 3; d++) {
			// every byte's nibbles as LDS byte offsets (nibble * 4) in two ops
			uint32_t H = (tup[d] >> 2) & 0x3C3C3C3Cu, L = (tup[d] << 2) & 0x3C3C3C3Cu;
			asm("" : "+v"(H), "+v"(L));   // keep the packed form (else it is re-split into shift + and per nibble)
#pragma unroll
			for (int b = 0; b < 4; b++) {
				const int k = 4 * d + b;
				rss ^= *reinterpret_cast<const uint32_t *>(tb + (2 * k) * 64 + ((H >> (8 * b)) & 0xFFu)) ^
				       *reinterpret_cast<const uint32_t *>(tb + (2 * k + 1) * 64 + ((L >> (8 * b)) & 0xFFu));
			}
		}
	}
	const uint32_t queue = (s_tab[MOSRX_TAB_RSS_WORDS + ((rss & 0x1FFu) >> 2)] >> (8 * (rss & 3u))) & 0xFFu;

	// ICMP to one of the netdevs' addresses (ip_in.c:83-85, icmp.c:193-200):
	// ProcessICMPPacket returns TRUE.  Rare, so the address list is read with
	// scalar loads only by a wave that holds an ICMP frame.
	bool icmp_local = false;
	if (__ballot(active && proto == 1u)) {
		const uint32_t nl = min(g_tab[MOSRX_TAB_LOCAL], (uint32_t)MOSRX_MAX_LOCAL);
		for (uint32_t i = 0; i < nl; i++)
			icmp_local |= daddr == g_tab[MOSRX_TAB_LOCAL + 1 + i];
		icmp_local = icmp_local && proto == 1u;
	}

	// verdict chain (eth_in.c:27 -> ip_in.c:30 -> tcp.c:408), evaluated without
	// branches: the reason is a select chain applied from the last check back to
	// the first (so the first failing check wins, as in the reference's early
	// returns), the verdict a 2-bit field of a per-launch table indexed by it.
	const bool verify = kflags & MOSRX_KF_VERIFY;
	const uint32_t l_ip = 14u + ihl * 4u;
	const bool c_nonip = h_proto != 0x0800u;
	const bool c_trunc = cap < 34u || l_ip > cap || fend > cap || (is_tcp && l_ip + 20u > cap);
	const bool c_tshort = ip_len < (ihl + doff) * 4u;
	const bool fields = cap >= 14u && !c_nonip && !c_trunc && ip_len >= 20u && ver == 4u;
	uint32_t reason = (kflags & MOSRX_KF_SKIP_TCP) ? MOSRX_R_TCP_LEN_OK : MOSRX_R_TRUNCATED;   // TRUNCATED: pending TCP sum
	reason = c_tshort ? MOSRX_R_TCP_SHORT : reason;                     // tcp.c:429-430
	reason = !is_tcp ? (icmp_local ? MOSRX_R_ICMP_LOCAL : MOSRX_R_NOT_TCP) : reason;   // ip_in.c:79-93
	reason = ipc != 0u ? MOSRX_R_IP_BADCSUM : reason;                   // ip_in.c:74-77
	reason = !verify ? MOSRX_R_NOVERIFY_PASS : reason;                  // ip_in.c:67-72
	reason = ver != 4u ? MOSRX_R_IP_BADVER : reason;                    // ip_in.c:47-51
	reason = ip_len < 20u ? MOSRX_R_IP_SHORT : reason;                  // ip_in.c:42-45
	reason = c_trunc ? MOSRX_R_TRUNCATED : reason;
	reason = c_nonip ? (h_proto == 0x0806u ? MOSRX_R_ARP : MOSRX_R_NON_IPV4) : reason;   // eth_in.c:62-77
	reason = cap < 14u ? MOSRX_R_TRUNCATED : reason;
	bool need_tcp = fields && verify && ipc == 0u && is_tcp && !c_tshort && !(kflags & MOSRX_KF_SKIP_TCP);
	// verdict + 1 per reason, 2 bits each (NON_IPV4 -> 1 when forwarding non-IP frames)
	const uint32_t vtab = VERDICT_TAB | ((kflags & MOSRX_KF_FWD_NONIP) ? (2u << (2 * MOSRX_R_NON_IPV4)) : 0u);
	const int verdict = (int)((vtab >> (2u * reason)) & 3u) - 1;
	// TX (mtcp_setlastpkt's MOS_UPDATE_*_CHKSUM, mos_api.c:1177-1193): every
	// untruncated IPv4 frame with a full header gets the IP check; TCP frames
	// whose length covers the header also get the TCP check.
	bool tx_ip = false;
	if (IS_TX(VAR)) {
		tx_ip = h_proto == 0x0800u && cap >= 34u && ihl >= 5u && 14u + ihl * 4u <= cap && fend <= cap &&
		        !(is_tcp && 14u + ihl * 4u + 20u > cap);
		need_tcp = tx_ip && is_tcp && ip_len >= (ihl + doff) * 4u && (kflags & MOSRX_KF_TX_TCP);
	}
	if (!active) {
		need_tcp = false;
		tx_ip = false;
	}

	h.o = o; h.fend = fend; h.split_abs = split_abs; h.wsum = wsum;
	h.saddr = saddr; h.daddr = daddr; h.ip_len = ip_len; h.ihl = ihl; h.doff = doff; h.th0 = th0; h.th3 = th3;
	h.th1 = th1; h.th2 = th2;
	h.rss = rss; h.queue = queue; h.ipc = ipc; h.reason = reason; h.verdict = verdict;
	h.tcw = tcw; h.ipc_tx = ipc_tx; h.tx_ip = tx_ip;
	h.fields = fields; h.need_tcp = need_tcp; h.has_tail = need_tcp && !in_win; h.is_tcp = is_tcp;
	return h;
}

// Fold in the tail sum, decide the TCP verdict, build the 16-byte record.
__device__ __forceinline__ u32x4 hdr_finish(hdr_t h, uint32_t tail_sum, uint32_t kflags)
{
	uint32_t tcpc = 0;
	if (h.need_tcp) {
		const uint32_t seglen = (h.ip_len - h.ihl * 4u) & 0xFFFFu;   // (doff<<2) + payloadlen, u16
		uint32_t s = h.wsum + (h.saddr & 0xFFFFu) + (h.saddr >> 16) + (h.daddr & 0xFFFFu) + (h.daddr >> 16) +
		             bswap16(seglen) + 0x0600u;                       // tcp_util.c:178-181
		if (h.has_tail) {
			const uint32_t ts = fold16(tail_sum);
			s += (h.o & 1u) ? bswap16(ts) : ts;
		}
		s = (s >> 16) + (s & 0xFFFFu);
		s += s >> 16;
		tcpc = (~s) & 0xFFFFu;
		h.verdict = tcpc ? -1 : 1;
		h.reason = tcpc ? MOSRX_R_TCP_BADCSUM : MOSRX_R_TCP_OK;
	}
	uint32_t r_rss = 0, r_ipc = 0, r_plen = 0, r_poff = 0, r_q = 0, r_flags = 0, r_ihld = 0;
	if (h.fields) {
		r_rss = h.rss;
		r_q = h.queue;
		r_ihld = (h.ihl << 4) | h.doff;
		if (kflags & MOSRX_KF_VERIFY)
			r_ipc = h.ipc;
		if (h.is_tcp) {
			r_flags = (h.th3 >> 8) & 0xFFu;
			r_plen = (h.ip_len - (h.ihl * 4u + h.doff * 4u)) & 0xFFFFu;   // tcp.c:262
			r_poff = 14u + h.ihl * 4u + h.doff * 4u;
		}
	}
	u32x4 rec;
	rec.x = r_rss;
	rec.y = r_ipc | (tcpc << 16);
	rec.z = r_plen | (r_poff << 16) | (((uint32_t)h.verdict & 0xFFu) << 24);
	rec.w = h.reason | (r_q << 8) | (r_flags << 16) | (r_ihld << 24);
	return rec;
}

// Flow-table hash of FindStream's reversed tuple (tcp.c:185-190): SuperFastHash
// (fhash.c:25-69) over the 12-byte key {daddr, saddr, dport, sport} of
// tcp_stream (tcp_stream.h:239-242) as three little-endian dwords; HashFlow
// (fhash.c:72-92) masks it to NUM_BINS.  Defined where payload_off != 0.
__device__ __forceinline__ uint32_t flow_hash(const hdr_t &h)
{
	const uint32_t key[3] = {h.daddr, h.saddr, __builtin_amdgcn_alignbit(h.th0, h.th0, 16)};
	uint32_t hash = 12u;
#pragma unroll
	for (int k = 0; k < 3; k++) {
		hash += key[k] & 0xFFFFu;
		const uint32_t tmp = ((key[k] >> 16) << 11) ^ hash;
		hash = (hash << 16) ^ tmp;
		hash += hash >> 11;
	}
	hash ^= hash << 3;
	hash += hash >> 5;
	hash ^= hash << 4;
	hash += hash >> 17;
	hash ^= hash << 25;
	hash += hash >> 6;
	return (h.fields && h.is_tcp) ? hash : 0u;
}

// pkt_info's TCP fields (FillPacketContextTCPInfo, tcp.c:258-270): seq,
// ack_seq, window in host order, plus ip_len (FillInPacketIPContext,
// ip_in.c:21-27); zero where the record has no TCP header fields.  One
// 12-byte store per lane.
__device__ __forceinline__ void store_tcpinfo(mosrx_tcpinfo *ti, uint32_t p, const hdr_t &h)
{
	const bool def = h.fields && h.is_tcp;
	u32x3 v;
	v.x = def ? __builtin_bswap32(h.th1) : 0u;
	v.y = def ? __builtin_bswap32(h.th2) : 0u;
	v.z = def ? (((h.th3 >> 24) | ((h.th3 >> 8) & 0xFF00u)) | (h.ip_len << 16)) : 0u;   // window = tcph bytes 14,15
	out_store(reinterpret_cast<uint32_t *>(ti), p, v);
}

// TX: write the fresh checksums into the frame (little-endian u16 stores, as
// `iph->check = ip_fast_csum(..)` and `tcph->check = TCPCalcChecksum(..)` do).
// The TCP value is the full-segment sum with the old check word taken out in
// one's-complement arithmetic: TCPCalcChecksum depends only on the sum mod
// 0xFFFF (the sum is > 0: the pseudo header holds 0x0600).
// With kp.out set the frames stay untouched: each frame's checks go out as an
// 8-byte record (mosrx_tx_check: the two check words, which of them apply,
// ihl) and the host writes them into its own copy of the frames -- what
// crosses PCIe back is 8 bytes per frame instead of the frame.
template <int SAUX = 0, bool DENSE = false>
__device__ __forceinline__ void tx_store(const mosrx_kparams &kp, __amdgpu_buffer_rsrc_t rs, const hdr_t &h,
                                         uint32_t tail_sum, uint32_t p, bool active)
{
	// an even frame start puts both check words on 2-byte boundaries: one short
	// store each (1.5-3 % faster than byte pairs; tails read with the default
	// cache policy so the stores hit L2 lines measured 20 % slower)
	const bool even = (h.o & 1u) == 0u;
	const bool ip = h.tx_ip && (kp.flags & MOSRX_KF_TX_IP);
	uint32_t c = 0;
	if (h.need_tcp) {
		const uint32_t seglen = (h.ip_len - h.ihl * 4u) & 0xFFFFu;
		uint32_t s = h.wsum + (h.saddr & 0xFFFFu) + (h.saddr >> 16) + (h.daddr & 0xFFFFu) + (h.daddr >> 16) +
		             bswap16(seglen) + 0x0600u;
		if (h.has_tail) {
			const uint32_t ts = fold16(tail_sum);
			s += (h.o & 1u) ? bswap16(ts) : ts;
		}
		s = (s >> 16) + (s & 0xFFFFu);
		s += s >> 16;                                   // low 16 bits in [1, 0xFFFF], == S mod 0xFFFF
		// - the old check word, as far as it lies inside the summed segment: a
		// short tot_len (doff < 5 is accepted, tcp.c:429) can leave tcph->check
		// past the ip_len - ihl*4 bytes TCPCalcChecksum covers, wholly or by its
		// second byte (the odd tail keeps the first, tcp_util.c:175-176)
		const uint32_t tcw_in = seglen >= 18u ? h.tcw : seglen == 17u ? (h.tcw & 0xFFu) : 0u;
		uint32_t v = (s & 0xFFFFu) + (0xFFFFu - tcw_in);
		v = (v & 0xFFFFu) + (v >> 16);
		c = (~v) & 0xFFFFu;
	}
	if (kp.out) {
		if (active) {
			u32x2 r;
			r.x = (h.ipc_tx & 0xFFFFu) | (c << 16);
			r.y = (ip ? 1u : 0u) | (h.need_tcp ? 2u : 0u) | (h.ihl << 8);
			out_store(reinterpret_cast<u32x2 *>(kp.out), p, r);
		}
		return;
	}
	if constexpr (DENSE) {   // probe: the same two words, into a dense array instead of the frames
		if (active)
			reinterpret_cast<uint32_t *>(kp.fhash)[p] = (ip ? (h.ipc_tx & 0xFFFFu) : 0u) | (h.need_tcp ? c << 16 : 0u);
		return;
	}
	if (ip) {
		if (even) {
			__builtin_amdgcn_raw_buffer_store_b16((uint16_t)h.ipc_tx, rs, h.o + 24u, 0, SAUX);
		} else {
			__builtin_amdgcn_raw_buffer_store_b8((uint8_t)h.ipc_tx, rs, h.o + 24u, 0, SAUX);
			__builtin_amdgcn_raw_buffer_store_b8((uint8_t)(h.ipc_tx >> 8), rs, h.o + 25u, 0, SAUX);
		}
	}
	if (h.need_tcp) {
		const uint32_t at = h.o + 30u + 4u * h.ihl;
		if (even) {
			__builtin_amdgcn_raw_buffer_store_b16((uint16_t)c, rs, at, 0, SAUX);
		} else {
			__builtin_amdgcn_raw_buffer_store_b8((uint8_t)c, rs, at, 0, SAUX);
			__builtin_amdgcn_raw_buffer_store_b8((uint8_t)(c >> 8), rs, at + 1u, 0, SAUX);
		}
	}
}


// Per-reason counters (the NETSTAT view, eth_in.c:42-45, 80-84): the lanes of
// a wave that store a record add one count per distinct reason to LDS (a ballot
// per reason, usually one), and the workgroup adds its counts to its own shard
// of the global counters (MOSRX_CNT_SHARDS lines of 16 words): adds from every
// workgroup to ONE word serialise at the memory side (~0.01 us each, which cost
// a 1024-workgroup launch ~11 us), spread over 256 lines they do not.
//
// Records and side arrays are written once and read by the host after the
// launch: non-temporal stores (rings 3-4 % faster than default-policy stores:
// 1500 B 122 -> 119 us, IMIX 141 -> 135 us, 64 B 127 -> 123 us).
template <int VAR>
__device__ __forceinline__ void store_record(const mosrx_kparams &kp, uint32_t p, u32x4 rec, uint32_t *s_cnt)
{
	if constexpr (IS_C8(VAR)) {
		// mosrx_result8: rss | reason, queue (rec.w bytes 0-1), verdict (rec.z byte 3), tcp_flags (rec.w byte 2)
		u32x2 c;
		c.x = rec.x;
		c.y = (rec.w & 0xFFFFu) | ((rec.z >> 24) << 16) | (((rec.w >> 16) & 0xFFu) << 24);
		out_store(reinterpret_cast<u32x2 *>(kp.out), p, c);
	} else {
		out_store(reinterpret_cast<u32x4 *>(kp.out), p, rec);
	}
	if (kp.counters) {
		const uint32_t reason = rec.w & 0xFFu;
		uint64_t m = __ballot(1);
		while (m) {
			const uint32_t first = (uint32_t)__builtin_ctzll(m);
			const uint32_t r = uni(__builtin_amdgcn_readlane(reason, first));
			const uint64_t same = __ballot(reason == r);
			if ((threadIdx.x & 63u) == first)
				atomicAdd(&s_cnt[r], (uint32_t)__builtin_popcountll(same));
			m &= ~same;
		}
	}
}

__device__ __forceinline__ void flush_counters(const mosrx_kparams &kp, const uint32_t *s_cnt, uint32_t t)
{
	if (kp.counters) {
		__syncthreads();
		if (t < MOSRX_R_COUNT && s_cnt[t])
			atomicAdd(&kp.counters[(blockIdx.x % MOSRX_CNT_SHARDS) * MOSRX_CNT_STRIDE + t], s_cnt[t]);
	}
}

// ---------------------------------------------------------------------------
// small tile: MOSRX_SMALL_FRAMES frames, lane per frame (or per FPL frames)
// ---------------------------------------------------------------------------
// Every frame whose datagram ends inside the header window (all frames of a
// batch with max_len <= MOSRX_WINDOW_END_SMALL) finishes in its lane: no cross-wave work, no
// barrier (each wave fills the LDS tables itself; a wave's LDS accesses are
// ordered).  Longer frames (only when the shape is forced onto them) are
// summed by their wave tail by tail, 4 KiB per pass.
template <int VAR, uint32_t TILE = MOSRX_KIND_FRAMES(MOSRX_KIND_SMALL), int DBG = 0,
          int WEND = MOSRX_WINDOW_END_SMALL>
__device__ __forceinline__ void classify_tile_small(const mosrx_kparams &kp, uint32_t tile)
{
	constexpr int AUX = TAIL_AUX(VAR);
	// the fused BPF hook reads the window up to MOSRX_BPF_WEND
	constexpr int NLOAD = (VAR & VAR_BPF) ? BPF_NLOAD(WEND) : WIN_NLOAD(WEND);
	constexpr int RSS = (DBG & 16384) ? 1 : 0;   // probe builds: no Toeplitz (hdr_parse RSS form 1)
	// DBG 2 skips the window loads, DBG 4 the record stores, DBG 256 fills the LDS
	// tables once per workgroup behind a barrier (probe builds only).  Tried and slower:
	// windows staged through LDS from contiguous wave loads (64 B config 192 vs
	// 125 us per 8M frames).
	__shared__ __attribute__((aligned(16))) uint32_t s_tab[MOSRX_TAB_WORDS];
	__shared__ uint32_t s_cnt[MOSRX_R_COUNT + 1];

	// FPL frames per lane: lane t owns frames tile*TILE + 256*i + t, and every
	// one of its descriptor and window loads is issued before the first parse
	// (FPL x the bytes in flight per wave).
	// (probe builds also launch tiles of 64 / 128 frames, one per lane)
	constexpr uint32_t FPL = TILE > 256u ? TILE / 256u : 1u;
	static_assert(TILE <= 256u || TILE % 256u == 0, "whole workgroups of frames");
	const uint32_t t = threadIdx.x, lane = t & 63u;
	const __amdgpu_buffer_rsrc_t rs = frame_rsrc(kp.frames, kp.frames_bytes);
	const uint32_t nbytes = kp.frames_bytes;
	uint32_t pv[FPL], ov[FPL], capv[FPL];
	bool actv[FPL];
	hdr_win_t winv[FPL];
	const u32x4 *tg = reinterpret_cast<const u32x4 *>(kp.tables);
	u32x4 ta, tb;   // the lane's share of the LDS tables
	// VAR_UNI: frame p is expected at (uni >> 16) + p * (uni & 0xFFFF) (the
	// batch's layout hint): its window and the tables are requested first, the
	// descriptors behind them, so all of the tile's loads are in flight before
	// its first wait -- one HBM round trip instead of two.  off[p] still
	// decides: a lane whose offset differs reloads its window (below).
	// uni == 0 (a queue batch without a hint): the hinted loads are off and
	// every lane reloads, i.e. waits for its descriptor as without VAR_UNI.
	const bool hinted = IS_UNI(VAR) && kp.uni != 0u;
	if constexpr (IS_UNI(VAR) && (DBG & 2) == 0) {
#pragma unroll
		for (uint32_t i = 0; i < FPL; i++) {
			const uint32_t p = tile * TILE + 256u * i + t;
			hdr_load<WIN_AUX(VAR), NLOAD>(rs, nbytes, (kp.uni >> 16) + p * (kp.uni & 0xFFFFu), p < kp.n && hinted,
			                              winv[i]);
		}
		ta = tg[lane];
		tb = tg[lane + 64];
	}
#pragma unroll
	for (uint32_t i = 0; i < FPL; i++) {
		pv[i] = tile * TILE + 256u * i + t;
		actv[i] = pv[i] < kp.n;
		// unconditional loads from a clamped index: the descriptor pointers then
		// come in the kernel's first scalar loads instead of a second, dependent
		// round trip behind a branch (the ramp of every tile)
		const uint32_t q = min(pv[i], kp.n - 1u);
		const uint32_t o = kp.off[q];
		uint32_t l = kp.len[q];
		asm volatile("" : "+v"(l));   // keep the len[] load unconditional
		ov[i] = actv[i] ? o : 0u;
		capv[i] = actv[i] ? eff_caplen(o, l, nbytes) : 0u;
	}
	if constexpr (IS_UNI(VAR) && (DBG & 2) == 0) {
#pragma unroll
		for (uint32_t i = 0; i < FPL; i++) {
			const bool miss = actv[i] && (!hinted || ov[i] != (kp.uni >> 16) + pv[i] * (kp.uni & 0xFFFFu));
			if (__ballot(miss)) {                 // the hint was wrong for some lane (or absent): reload
				hdr_win_t w2;
				hdr_load<WIN_AUX(VAR), NLOAD>(rs, nbytes, ov[i], miss, w2);
#pragma unroll
				for (int j = 0; j < WIN_RAW; j++)
					winv[i].raw[j] = miss ? w2.raw[j] : winv[i].raw[j];
			}
		}
	} else {
#pragma unroll
		for (uint32_t i = 0; i < FPL; i++) {
			if constexpr (DBG & 2) {
#pragma unroll
				for (int j = 0; j < WIN_RAW; j++)
					winv[i].raw[j] = ov[i] + j;
			} else {
				hdr_load<WIN_AUX(VAR), NLOAD>(rs, nbytes, ov[i], actv[i], winv[i]);
			}
		}
		ta = tg[lane];
		tb = tg[lane + 64];
	}
	if constexpr ((DBG & 256) != 0 && TILE >= 256u) {
		// probe builds: the workgroup fills the tables once (8 bytes per lane) and
		// waits at a barrier, instead of each wave filling all of them itself
		(void)ta; (void)tb;
		reinterpret_cast<u32x2 *>(s_tab)[t] = reinterpret_cast<const u32x2 *>(kp.tables)[t];
		__syncthreads();
	} else {
		reinterpret_cast<u32x4 *>(s_tab)[lane] = ta;
		reinterpret_cast<u32x4 *>(s_tab)[lane + 64] = tb;
	}
	if (kp.counters) {                        // uniform: the whole workgroup takes this barrier or none
		if (t <= MOSRX_R_COUNT)
			s_cnt[t] = 0;
		__syncthreads();
	}
#pragma unroll
	for (uint32_t fi = 0; fi < FPL; fi++) {
	const uint32_t p = pv[fi], o = ov[fi], cap = capv[fi];
	const bool active = actv[fi];
	const hdr_win_t &win = winv[fi];
	const hdr_t h = hdr_parse<VAR, WEND, RSS>(win, o, cap, active, kp.flags, s_tab, kp.tables, rs, nbytes);
	uint32_t tail = 0;
	for (uint64_t m = __ballot(h.has_tail); m; m &= m - 1) {
		const uint32_t f = (uint32_t)__builtin_ctzll(m);
		const uint32_t lo = uni(__builtin_amdgcn_readlane(h.split_abs, f));
		const uint32_t hi = uni(__builtin_amdgcn_readlane(o + h.fend, f));
		uint32_t acc = 0;
#pragma unroll 1
		for (uint32_t base = lo; base < hi; base += 4096u) {
			u32x4 v[4];
#pragma unroll
			for (int i = 0; i < 4; i++) {
				const uint32_t c = base + 1024u * i + 16u * lane;
				v[i] = load16<AUX>(rs, c < hi ? c : ZERO_OFF, 0);
			}
#pragma unroll
			for (int i = 0; i < 4; i++)
				acc = chunk_sum(v[i], base + 1024u * i + 16u * lane, hi, acc);
		}
		const uint32_t x = wave_sum(acc);
		if (lane == f)
			tail = x;
	}
	if constexpr (IS_TX(VAR)) {
		tx_store(kp, rs, h, tail, p, active);
	} else if constexpr ((DBG & 4) != 0) {   // probe: records kept live, (almost) never stored
		const u32x4 r = hdr_finish(h, tail, kp.flags);
		if (active && (r.x ^ r.y ^ r.z ^ r.w) == 0x9E3779B9u)
			store_record<VAR>(kp, p, r, s_cnt);
	} else {
		if (active)
			store_record<VAR>(kp, p, hdr_finish(h, tail, kp.flags), s_cnt);
		if (active && kp.fhash)
			out_store(kp.fhash, p, flow_hash(h));
		if constexpr (IS_TI(VAR)) {
			if (active)
				store_tcpinfo(kp.tinfo, p, h);
		}
	}
#ifdef MOSRX_RTC_BPF
	if constexpr ((VAR & VAR_BPF) != 0) {
		if (active)
			out_store(kp.bmatch, p, h.bmatch);
	}
#endif
	}
	flush_counters(kp, s_cnt, t);
}

// Absolute-grid word sum of the bytes [a, b) (any alignment), whole wave.
__device__ __forceinline__ uint32_t range_sum(__amdgpu_buffer_rsrc_t rs, uint32_t nbytes, uint32_t a, uint32_t b,
                                              uint32_t lane)
{
	uint32_t acc = 0;
#pragma unroll 1
	for (uint32_t base = a & ~15u; base < b; base += 1024u) {
		const uint32_t c = base + 16u * lane;
		u32x4 v = load16<0>(rs, c < b ? c : nbytes, nbytes);
		const int h = (int)(a - c);   // bytes to drop at the front
		v.x &= ~keep_lo(h);
		v.y &= ~keep_lo(h - 4);
		v.z &= ~keep_lo(h - 8);
		v.w &= ~keep_lo(h - 12);
		acc = chunk_sum(v, c, b, acc);
	}
	return wave_sum(acc);
}

// Header wave epilogue of the tail-streaming shapes: `tail` is the speculative
// tail sum over [split, off + caplen).  Bytes between the datagram end and the
// capture end (Ethernet padding of a long capture) were summed too: subtract
// them (exact integer sums, so the difference is the true tail sum).  Rare: a
// wave-wide pass per such frame.  Then the record (or the TX rewrite).
template <int VAR, int DBG = 0>
__device__ __forceinline__ void hdr_emit(const mosrx_kparams &kp, __amdgpu_buffer_rsrc_t rs, uint32_t nbytes,
                                         const hdr_t &h, uint32_t lo_l, uint32_t hi_l, uint32_t tail, uint32_t p,
                                         bool active, uint32_t lane, uint32_t *s_cnt)
{
	const uint32_t true_hi = h.o + h.fend;
	uint64_t fm = __ballot(h.has_tail && true_hi < hi_l);
#pragma unroll 1
	while (fm) {
		const uint32_t f = (uint32_t)__builtin_ctzll(fm);
		fm &= fm - 1;
		const uint32_t a = max(__builtin_amdgcn_readlane(lo_l, f), __builtin_amdgcn_readlane(true_hi, f));
		const uint32_t s = range_sum(rs, nbytes, a, __builtin_amdgcn_readlane(hi_l, f), lane);
		if (lane == f)
			tail -= s;
	}
	if constexpr (IS_TX(VAR)) {
		tx_store<(DBG & 8388608) ? 2 : (DBG & 33554432) ? 17 : 0, (DBG & 16777216) != 0>(kp, rs, h, tail, p, active);
	} else if (active) {
		store_record<VAR>(kp, p, hdr_finish(h, tail, kp.flags), s_cnt);
		if (kp.fhash)
			out_store(kp.fhash, p, flow_hash(h));
		if constexpr (IS_TI(VAR))
			store_tcpinfo(kp.tinfo, p, h);
	}
}

// The header wave's LDS state: the RSS nibble tables + queue map, and zeroed
// reason counts (a wave's LDS accesses are ordered: no barrier needed for its
// own use).
template <int RSS = 0>
__device__ __forceinline__ void tab_fill(const mosrx_kparams &kp, uint32_t *s_tab, uint32_t *s_cnt, uint32_t lane)
{
	const u32x4 *tg = reinterpret_cast<const u32x4 *>(kp.tables);
	const u32x4 a = tg[lane], b = tg[lane + 64];
	reinterpret_cast<u32x4 *>(s_tab)[lane] = a;
	reinterpret_cast<u32x4 *>(s_tab)[lane + 64] = b;
	if constexpr (RSS == 2) {   // probe: the byte tables after the library's words
		u32x4 v[12];
#pragma unroll
		for (int i = 0; i < 12; i++)
			v[i] = tg[MOSRX_TAB8_OFF / 4 + 64 * i + lane];
#pragma unroll
		for (int i = 0; i < 12; i++)
			reinterpret_cast<u32x4 *>(s_tab + MOSRX_TAB_WORDS)[64 * i + lane] = v[i];
	}
	if (lane <= MOSRX_R_COUNT)
		s_cnt[lane] = 0;
}

// What the stream tile's header wave keeps of a parsed frame across its
// barrier: the record with everything but the TCP checksum verdict filled in,
// the TCP sum before the tail, the overshoot of the capture's last chunk and
// the datagram end (for the padding fix).  Everything that does not need the
// tail sum is done before the barrier, where the header wave waits for the
// streamers anyway: after it only the fold, the store and the counts remain,
// and the workgroup's slots free sooner (0.3-0.7 % on every row, interleaved
// medians of scripts/probe_timeline; DBG 8192 keeps the whole record after B).
struct hdr_pend_t {
	u32x4 rec;
	uint32_t spre, ovs, true_hi, bits;   // bits: 1 need_tcp, 2 has_tail, 4 odd start
};

__device__ __forceinline__ hdr_pend_t hdr_pend(const hdr_t &h, uint32_t kflags, uint32_t ovs)
{
	hdr_pend_t q;
	hdr_t hn = h;
	hn.need_tcp = false;   // the TCP verdict bytes are filled in by pend_finish
	q.rec = hdr_finish(hn, 0u, kflags);
	q.spre = 0;
	if (h.need_tcp) {
		const uint32_t seglen = (h.ip_len - h.ihl * 4u) & 0xFFFFu;   // tcp_util.c:178-181, as hdr_finish
		q.spre = h.wsum + (h.saddr & 0xFFFFu) + (h.saddr >> 16) + (h.daddr & 0xFFFFu) + (h.daddr >> 16) +
		         bswap16(seglen) + 0x0600u;
	}
	q.ovs = ovs;
	q.true_hi = h.o + h.fend;
	q.bits = (h.need_tcp ? 1u : 0u) | (h.has_tail ? 2u : 0u) | ((h.o & 1u) ? 4u : 0u);
	return q;
}

// hdr_finish's TCP part on a pending record
__device__ __forceinline__ u32x4 pend_finish(const hdr_pend_t &q, uint32_t tail)
{
	u32x4 rec = q.rec;
	if (q.bits & 1u) {
		uint32_t s = q.spre;
		if (q.bits & 2u) {
			const uint32_t ts = fold16(tail);
			s += (q.bits & 4u) ? bswap16(ts) : ts;
		}
		s = (s >> 16) + (s & 0xFFFFu);
		s += s >> 16;
		const uint32_t tcpc = (~s) & 0xFFFFu;
		rec.y |= tcpc << 16;
		rec.z = (rec.z & 0x00FFFFFFu) | (((uint32_t)(tcpc ? -1 : 1) & 0xFFu) << 24);
		rec.w = (rec.w & ~0xFFu) | (tcpc ? MOSRX_R_TCP_BADCSUM : MOSRX_R_TCP_OK);
	}
	return rec;
}

// After the barrier: `tail` = the streamers' sum minus the overshoot.  Bytes
// between the datagram end and the capture end (Ethernet padding of a long
// capture) were summed too and come out here (rare: a wave-wide pass per such
// frame), then the record.
template <int VAR>
__device__ __forceinline__ void pend_emit(const mosrx_kparams &kp, __amdgpu_buffer_rsrc_t rs, uint32_t nbytes,
                                          const hdr_pend_t &q, uint32_t lo_l, uint32_t hi_l, uint32_t tail,
                                          uint32_t p, bool active, uint32_t lane, uint32_t *s_cnt)
{
	uint64_t fm = __ballot((q.bits & 2u) && q.true_hi < hi_l);
#pragma unroll 1
	while (fm) {
		const uint32_t f = (uint32_t)__builtin_ctzll(fm);
		fm &= fm - 1;
		const uint32_t a = max(__builtin_amdgcn_readlane(lo_l, f), __builtin_amdgcn_readlane(q.true_hi, f));
		const uint32_t sm = range_sum(rs, nbytes, a, __builtin_amdgcn_readlane(hi_l, f), lane);
		if (lane == f)
			tail -= sm;
	}
	if (active)
		store_record<VAR>(kp, p, pend_finish(q, tail), s_cnt);
}

// ---------------------------------------------------------------------------
// stream tile: 64 frames, one header wave + S streamers over the tile's tail span
// ---------------------------------------------------------------------------
// Frames of a received batch sit in buffer order (an rx ring, a pcap file, the
// loopback source): frame j+1 starts at or after the capture end of frame j.
// Then the speculative tails [split_j, off_j + caplen_j) of a tile are
// disjoint, sorted and start on 16-byte boundaries, and every 16-byte chunk
// holds bytes of at most one tail (the next tail starts >= 79 bytes past this
// capture's end).  The tile's bytes from the first split to the last capture
// end (the "span") are read as plain contiguous 1 KiB wave loads: streamer s
// of S takes the s-th run of the span's 1 KiB blocks with STREAM_U loads in
// flight per lane, every lane busy (chunks outside all tails are header
// windows and short frames, read again from L2, and never counted).  A tail
// [lo, hi) covers the chunks lo .. ec = (hi - 1) & ~15 with only ec partial,
// so its sum over a run is E(ec) + partial(ec) - E(lo), E being the run's
// exclusive prefix of whole-chunk sums: per block one wave scan gives E for
// its 64 chunks; the frame lanes (lane = frame) whose lo or ec falls in the
// block fetch E there with ds_bpermute, and an ending frame sums its last
// chunk's bytes below hi from an LDS copy of the block.  A tail entering the
// run counts from 0, one leaving it ends at the run total.  No ownership
// walk, no per-tail reduction; the header wave adds the S rows.  Tiles not in
// buffer order stream tail by tail (stream_frames).
#ifndef STREAM_U
#define STREAM_U 4
#endif

// Inclusive prefix sum over the 64 lanes: row scans (4 DPP row shifts), then
// row_bcast:15 and row_bcast:31 carry the row totals up.
__device__ __forceinline__ uint32_t wave_scan(uint32_t v)
{
	int x = (int)v;
	x += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xF, 0xF, false);   // row_shr:1
	x += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xF, 0xF, false);   // row_shr:2
	x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xF, 0xF, false);   // row_shr:4
	x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xF, 0xF, false);   // row_shr:8
	x += __builtin_amdgcn_update_dpp(0, x, 0x142, 0xA, 0xF, false);   // row_bcast:15 -> rows 1, 3
	x += __builtin_amdgcn_update_dpp(0, x, 0x143, 0xC, 0xF, false);   // row_bcast:31 -> rows 2, 3
	return (uint32_t)x;
}

// Streamer sidx of S over its run of the span [A, Z); the frame lanes' sums go
// to row[lane].  A tail is summed in whole 16-byte chunks, from its split to the
// end of the chunk holding its last captured byte: the header wave subtracts
// the few bytes past the capture end (chunk_overshoot), so a block costs one
// scan and two ds_bpermute reads whatever its frames.  DBG 4 (probe builds):
// loads only.
template <int S, int AUX, int DBG = 0, int U = STREAM_U>
__device__ __forceinline__ void stream_scan(__amdgpu_buffer_rsrc_t rs, uint32_t lo_l, uint32_t hi_l, uint32_t A,
                                            uint32_t Z, uint32_t sidx, uint32_t lane, uint32_t *row)
{
	const uint32_t nblk = (Z - A + 1023u) >> 10;
	const uint32_t b0 = uni((nblk * sidx) / S), b1 = uni((nblk * (sidx + 1u)) / S);
	const bool cand = hi_l > lo_l;
	const uint32_t ec_l = (hi_l - 1u) & ~15u;
	const uint32_t R1 = A + (b1 << 10);
	// per frame lane, once per tile: the block and the lane (as a ds_bpermute
	// byte address) of its tail's first and last chunk in the span (lo_l >= A
	// for every candidate of a tile in buffer order)
	const uint32_t blo = cand ? (lo_l - A) >> 10 : 0xFFFFFFFFu, bec = cand ? (ec_l - A) >> 10 : 0xFFFFFFFFu;
	const int alo = (int)(((lo_l - A) >> 2) & 0xFCu), aec = (int)(((ec_l - A) >> 2) & 0xFCu);
	uint32_t acc = 0, carry = 0;

	u32x4 v[U];
#pragma unroll
	for (int i = 0; i < U; i++) {
		const uint32_t b = b0 + (uint32_t)i;
		v[i] = load16<AUX>(rs, b < b1 ? A + (b << 10) + 16u * lane : ZERO_OFF, 0);
	}
#pragma unroll 1
	for (uint32_t k = b0; k < b1; k += U) {
#pragma unroll
		for (int i = 0; i < U; i++) {
			const uint32_t b = k + (uint32_t)i;
			if constexpr (DBG & 4) {
				acc ^= v[i].x ^ v[i].y ^ v[i].z ^ v[i].w;
			} else if (b < b1) {
				uint32_t s = add16x2(0u, v[i].x);
				s = add16x2(s, v[i].y);
				s = add16x2(s, v[i].z);
				s = add16x2(s, v[i].w);
				const uint32_t X = carry + wave_scan(s);   // inclusive prefix of the run
				carry = (uint32_t)__builtin_amdgcn_readlane((int)X, 63);
				const bool es = blo == b, ee = bec == b;
				if (__ballot(es || ee)) {
					// tail = X(end chunk) - E(start chunk), E = X - s the exclusive prefix
					const uint32_t Es = (uint32_t)__builtin_amdgcn_ds_bpermute(alo, (int)(X - s));
					const uint32_t Xe = (uint32_t)__builtin_amdgcn_ds_bpermute(aec, (int)X);
					acc = es ? acc - Es : acc;
					acc = ee ? acc + Xe : acc;
				}
			}
			const uint32_t bn = b + U;
			v[i] = load16<AUX>(rs, bn < b1 ? A + (bn << 10) + 16u * lane : ZERO_OFF, 0);
		}
	}
	if constexpr (DBG & 4) {
		if (acc == 0x9E3779B9u)
			row[lane] = acc;
		return;
	}
	if (cand && lo_l < R1 && ec_l >= R1)
		acc += carry;                        // tail continuing past the run
	row[lane] = acc;
}

// Absolute-grid word sum of the bytes of the 16-byte chunk at c (the chunk
// holding byte hi - 1) at or past hi: what stream_scan summed beyond a capture.
__device__ __forceinline__ uint32_t chunk_overshoot(u32x4 v, uint32_t c, uint32_t hi)
{
	const int h = (int)(hi - c);   // bytes of the capture in the chunk, 1..16
	v.x &= ~keep_lo(h);
	v.y &= ~keep_lo(h - 4);
	v.z &= ~keep_lo(h - 8);
	v.w &= ~keep_lo(h - 12);
	uint32_t acc = add16x2(0u, v.x);
	acc = add16x2(acc, v.y);
	acc = add16x2(acc, v.z);
	return add16x2(acc, v.w);
}

// Tiles not in buffer order: streamer sidx sums the candidates of rank
// sidx, sidx + S, ... one tail at a time, 4 KiB per pass.  Lean on registers
// on purpose (the tile's VGPR count sets its occupancy, and the span path
// needs 54): such tiles are rare (descriptors reordered after capture).
template <int S, int AUX>
__device__ __forceinline__ void stream_frames(__amdgpu_buffer_rsrc_t rs, uint32_t lo_l, uint32_t hi_l,
                                              uint32_t sidx, uint32_t lane, uint32_t *row)
{
	uint64_t m = __ballot(hi_l > lo_l);
	for (uint32_t r = 0; m; r++, m &= m - 1) {
		if (r % S != sidx)
			continue;
		const uint32_t f = (uint32_t)__builtin_ctzll(m);
		const uint32_t lo = uni(__builtin_amdgcn_readlane(lo_l, f)), hi = uni(__builtin_amdgcn_readlane(hi_l, f));
		uint32_t acc = 0;
#pragma unroll 1
		for (uint32_t base = lo; base < hi; base += 4096u) {
			u32x4 v[4];
#pragma unroll
			for (int i = 0; i < 4; i++) {
				const uint32_t c = base + 1024u * i + 16u * lane;
				v[i] = load16<AUX>(rs, c < hi ? c : ZERO_OFF, 0);
			}
#pragma unroll
			for (int i = 0; i < 4; i++)
				acc = chunk_sum(v[i], base + 1024u * i + 16u * lane, hi, acc);
		}
		const uint32_t x = wave_sum(acc);
		if (lane == 0)
			row[f] = x;
	}
}

// DBG (probe builds only, the library uses 0): 1 no parse/records, 2 no header
// window loads, 4 streamer loads only, 16 no unsorted-tile path, 32 header wave
// at raised issue priority, 128 per-tile timeline stamps into kp.bmatch
// (scripts/probe_timeline.hip: 16 words per tile, 100 MHz real-time clock),
// 131072 the fused set's masks computed but (almost) never stored, 262144 a
// constant mask stored without a set, 524288 the masks stored through the
// cache instead of non-temporally (scripts/probe_fused_fixed.hip), 1048576 the
// 78-byte (5-chunk) window (scripts/probe_guided.hip), 2097152 streamer 0
// reads the descriptors of tile + 2048 (the tile that takes this slot's place
// in a 4096-tile launch, same XCD) into L2, 4194304 also the first line of
// each of that tile's frames (scripts/probe_prefetch.hip), 8388608 the TX
// check words stored non-temporally, 16777216 stored as one u32 per frame into
// a dense array (kp.fhash) instead of the frames, 33554432 stored write-through
// at system scope (sc0 | sc1) (scripts/probe_tx_store.hip).
#define TILE_STAMP(i)                                                                             \
	do {                                                                                          \
		if constexpr ((DBG & 128) != 0) {                                                         \
			__builtin_amdgcn_s_waitcnt(0);                                                        \
			if (lane == 0)                                                                        \
				kp.bmatch[tile * 16u + (i)] = (uint32_t)__builtin_amdgcn_s_memrealtime();         \
		}                                                                                         \
	} while (0)
// One stream tile over frames [first, first + cnt), cnt <= T <= 64 (`tile`
// only numbers the timeline stamps); the library's tiles are classify_tile_stream.
template <int S, int VAR, int DBG = 0, int U = STREAM_U, uint32_t T = 64>
__device__ __forceinline__ void classify_span_stream(const mosrx_kparams &kp, uint32_t tile, uint32_t first,
                                                     uint32_t cnt)
{
	constexpr int AUX = TAIL_AUX(VAR);
	// DBG 2048: the full 96-byte window (the round-1 form, 4 % slower)
	constexpr int WEND = (DBG & 2048) ? MOSRX_WINDOW_END_FULL : (DBG & 1048576) ? MOSRX_WINDOW_END_SMALL
	                                                                             : MOSRX_WINDOW_END_STREAM;
	constexpr int NLOAD = (VAR & VAR_BPF) ? BPF_NLOAD(WEND) : WIN_NLOAD(WEND);
	// DBG 16384 / 32768 / 65536: RSS form 1 / 2 / 3 of hdr_parse (probe builds)
	constexpr int RSS = (DBG & 16384) ? 1 : (DBG & 32768) ? 2 : (DBG & 65536) ? 3 : 0;
	__shared__ __attribute__((aligned(16))) uint32_t s_tab[MOSRX_TAB_WORDS + (RSS == 2 ? 12 * 256 : 0)];
	__shared__ uint32_t s_part[S][64];   // streamer s's tail sums
	__shared__ uint32_t s_cnt[MOSRX_R_COUNT + 1];

	const uint32_t t = threadIdx.x, lane = t & 63u, wave = t >> 6;
	const __amdgpu_buffer_rsrc_t rs = frame_rsrc(kp.frames, kp.frames_bytes);
	const uint32_t nbytes = kp.frames_bytes;
	const uint32_t nact = cnt;

	if (wave == 0)
		TILE_STAMP(0);
	// every wave reads the tile's descriptors (lane = frame)
	const uint32_t p = first + lane;
	const bool active = lane < nact;
	// unconditional (clamped to the tile's first frame, cnt >= 1): no branch
	// between the kernel's scalar loads and the descriptor loads
	const uint32_t q = active ? p : first;
	const uint32_t od = kp.off[q];
	uint32_t ld = kp.len[q];
	asm volatile("" : "+v"(ld));   // keep the len[] load unconditional (not sunk into a branch)
	const uint32_t o = active ? od : 0u, cap = active ? eff_caplen(od, ld, nbytes) : 0u;
	// speculative tail bounds from the capture length: [split, off + caplen)
	const uint32_t lo_l = (o + (uint32_t)WEND) & ~15u;
	const uint32_t hi_l = active ? o + cap : 0u;
	// buffer order: the next frame starts at or after this capture's end
	const uint32_t onext = (uint32_t)__shfl_down((int)o, 1);
	const bool sorted = __ballot(lane + 1u < nact && onext < hi_l) == 0;

	if (wave == 0) {
		// ---- header wave (fills s_tab itself: a wave's LDS accesses are ordered) ----
		if constexpr (DBG & 32)
			__builtin_amdgcn_s_setprio(2);
		TILE_STAMP(1);
		if constexpr ((DBG & 128) != 0) {
			if (lane == 0) {
				kp.bmatch[tile * 16u + 10u] = __builtin_amdgcn_s_getreg(4 | (31 << 11));    // HW_ID
				kp.bmatch[tile * 16u + 11u] = __builtin_amdgcn_s_getreg(20 | (31 << 11));   // XCC_ID
			}
		}
		if constexpr ((DBG & 512) != 0)
			__syncthreads();   // B first: windows read after the streamers passed them
		// Small-frame mixes (cached tails) fill the LDS tables first: the window
		// loads then leave a table round trip later, when the streamers (whose
		// span starts at the tile's first byte) have the lines on the way (IMIX
		// 256K 20.38 vs 20.66 us, 2M frames 140.4 vs 141.4, interleaved medians).
		// Long frames (non-temporal tails) issue the windows first (1500 B 64K
		// 17.68 vs 17.90 us).  DBG 4096 flips the order (probe builds).
		constexpr bool TAB_FIRST = (TAIL_AUX(VAR) == 0) != ((DBG & 4096) != 0);
		if constexpr (TAB_FIRST)
			tab_fill<RSS>(kp, s_tab, s_cnt, lane);
		hdr_win_t win;
		if constexpr (DBG & 2) {
#pragma unroll
			for (int i = 0; i < WIN_RAW; i++)
				win.raw[i] = o + i;
		} else {
			hdr_load<WIN_AUX(VAR), NLOAD>(rs, nbytes, o, active, win);
		}
		// the chunk holding the capture's last byte (stream_scan sums it whole)
		const bool cand = hi_l > lo_l;
		const u32x4 ov = load16<WIN_AUX(VAR)>(rs, sorted && cand ? (hi_l - 1u) & ~15u : ZERO_OFF, 0);
		if constexpr (!TAB_FIRST)
			tab_fill<RSS>(kp, s_tab, s_cnt, lane);
		if constexpr (DBG & 1) {
			uint32_t x = 0;
#pragma unroll
			for (int i = 0; i < WIN_RAW; i++)
				x ^= win.raw[i];
			__syncthreads();   // B
			if (active && (x ^ s_part[0][lane]) == 0x9E3779B9u)
				kp.out[p].rss = x;
		} else {
			TILE_STAMP(2);
			const hdr_t h = hdr_parse<VAR, WEND, RSS>(win, o, cap, active, kp.flags, s_tab, kp.tables, rs, nbytes);
			if constexpr (IS_TX(VAR) || (DBG & 8192) != 0) {   // DBG 8192: the whole record after the barrier
				TILE_STAMP(3);
				__syncthreads();   // B: s_part ready
				TILE_STAMP(4);
				uint32_t tail = 0;
				if (h.has_tail) {
#pragma unroll
					for (int s = 0; s < S; s++)
						tail += s_part[s][lane];
					if (sorted)
						tail -= chunk_overshoot(ov, (hi_l - 1u) & ~15u, hi_l);
				}
				hdr_emit<VAR, DBG>(kp, rs, nbytes, h, lo_l, hi_l, tail, p, active, lane, s_cnt);
			} else {
				// the outputs that do not need the tail sum go out before the barrier
				if (active && kp.fhash)
					out_store(kp.fhash, p, flow_hash(h));
				if constexpr (IS_TI(VAR)) {
					if (active)
						store_tcpinfo(kp.tinfo, p, h);
				}
#ifdef MOSRX_RTC_BPF
				if constexpr ((VAR & VAR_BPF) != 0) {
					if (active && ((DBG & 131072) == 0 || h.bmatch == 0x5A5A5A5Au)) {
						if constexpr ((DBG & 524288) != 0)
							kp.bmatch[p] = h.bmatch;   // probe: a cached store
						else
							out_store(kp.bmatch, p, h.bmatch);
					}
				}
#endif
				if constexpr ((DBG & 262144) != 0) {
					if (active)
						out_store(kp.bmatch, p, 0xFFu);
				}
				const hdr_pend_t q =
				    hdr_pend(h, kp.flags, sorted && cand ? chunk_overshoot(ov, (hi_l - 1u) & ~15u, hi_l) : 0u);
				TILE_STAMP(3);
				if constexpr ((DBG & 512) == 0)
					__syncthreads();   // B: s_part ready
				TILE_STAMP(4);
				uint32_t tail = 0;
				if (q.bits & 2u) {
#pragma unroll
					for (int s = 0; s < S; s++)
						tail += s_part[s][lane];
					tail -= q.ovs;
				}
				pend_emit<VAR>(kp, rs, nbytes, q, lo_l, hi_l, tail, p, active, lane, s_cnt);
			}
			TILE_STAMP(5);
			// only this wave counted (its LDS accesses are ordered): it adds the
			// tile's counts to its shard without a second barrier, so the
			// streamers retire at B and the next tile can start on their slots
			if (kp.counters && lane < MOSRX_R_COUNT && s_cnt[lane])
				atomicAdd(&kp.counters[(blockIdx.x % MOSRX_CNT_SHARDS) * MOSRX_CNT_STRIDE + lane], s_cnt[lane]);
		}
	} else {
		// ---- streamer sidx ----
		const uint32_t sidx = wave - 1u;
		uint32_t *row = s_part[sidx];
		if (sidx == 0)
			TILE_STAMP(6);
		uint32_t pf_o = 0, pf_l = 0;
		if constexpr ((DBG & (2097152 | 4194304)) != 0) {
			const uint32_t qn = first + 2048u * T + lane;
			if (sidx == 0 && qn < kp.n) {
				pf_o = kp.off[qn];
				pf_l = kp.len[qn];
			}
		}
		row[lane] = 0;
		const uint64_t cmask = __ballot(hi_l > lo_l);
		if (sorted && cmask) {
			// the span runs from the first candidate's split to the last
			// candidate's capture end (in buffer order both are monotone, and a
			// candidate's capture is clipped to the buffer, so a bogus offset on a
			// frame without a tail can never stretch the span)
			// (from the tile's first byte: the streamers pass over the header
			// windows in buffer order too, measured 2 % faster than starting at
			// the first split; DBG 1024 keeps the split start for comparison)
			uint32_t A = uni(__builtin_amdgcn_readlane(lo_l, (int)__builtin_ctzll(cmask)));
			const uint32_t Z = uni(__builtin_amdgcn_readlane(hi_l, 63 - (int)__builtin_clzll(cmask)));
			if constexpr ((DBG & 1024) == 0)
				A = min(A, uni(__builtin_amdgcn_readfirstlane(o)) & ~15u);
			stream_scan<S, AUX, DBG, U>(rs, lo_l, hi_l, A, Z, sidx, lane, row);
		} else if (!sorted) {
			if constexpr (!(DBG & 16))
				stream_frames<S, AUX>(rs, lo_l, hi_l, sidx, lane, row);
		}
		if constexpr ((DBG & (2097152 | 4194304)) != 0) {
			if constexpr ((DBG & 4194304) != 0) {
				if (sidx == 0 && pf_l)
					pf_l += load16<0>(rs, pf_o & ~15u, nbytes).x;
			}
			asm volatile("" ::"v"(pf_o), "v"(pf_l));
		}
		TILE_STAMP(7 + sidx);
		__syncthreads();   // B
	}
}

template <int S, int VAR, int DBG = 0, int U = STREAM_U, uint32_t T = 64>
__device__ __forceinline__ void classify_tile_stream(const mosrx_kparams &kp, uint32_t tile)
{
	classify_span_stream<S, VAR, DBG, U, T>(kp, tile, tile * T, min(T, kp.n - tile * T));
}

template <int KIND, int VAR>
__device__ __forceinline__ void classify_tile(const mosrx_kparams &kp, uint32_t tile)
{
	if constexpr (KIND == MOSRX_KIND_SMALL)
		classify_tile_small<VAR>(kp, tile);
	else
		classify_tile_stream<MOSRX_STREAMERS, VAR>(kp, tile);
}

// The stream tiles are held to 64 VGPRs: 8 waves per SIMD.
#define MIN_WAVES(kind) ((kind) != MOSRX_KIND_SMALL ? 8 : 1)

// The fields every tile needs before its first frame byte lead the argument
// list as scalars: the build preloads them into SGPRs at dispatch
// (-amdgpu-kernarg-preload-count, Makefile), so a tile's first memory access is
// its descriptor load, not a kernarg round trip.  The rest of kp is read from
// the kernarg segment while the descriptors are on their way.
template <int KIND, int VAR>
__global__ __launch_bounds__(WG_THREADS(KIND)) __attribute__((amdgpu_waves_per_eu(MIN_WAVES(KIND))))
void mosrx_classify_kernel(const uint32_t *off, const uint16_t *len, const uint8_t *frames, const uint32_t *tables,
                           uint32_t frames_bytes, uint32_t n, uint32_t flags, uint32_t uni, mosrx_kparams kp)
{
	kp.off = off;
	kp.len = len;
	kp.frames = frames;
	kp.tables = tables;
	kp.frames_bytes = frames_bytes;
	kp.n = n;
	kp.flags = flags;
	kp.uni = uni;
	classify_tile<KIND, VAR>(kp, blockIdx.x);
}

// Batch queue: one launch over nb resident batches (descriptor table in HBM).
// Workgroup b finds its batch by one scalar division when every batch has the
// same tile count (the usual rx ring of equal batches), else by a binary
// search of tile_base[] (a chain of dependent scalar loads).
// The fused classify + BPF kernels (hipRTC, bpf_jit.c) instantiate the same
// body with VAR_BPF: their descriptors carry the match masks where the
// classify kernels carry pkt_info (mosrx_qdesc's union).
template <int KIND, int VAR>
__device__ __forceinline__ void queue_tile(const mosrx_qdesc *desc, uint32_t tpb, uint32_t nb, const mosrx_qparams &qp)
{
	const uint32_t b = blockIdx.x;
	uint32_t lo = 0, hi = nb;                  // find k: tile_base[k] <= b < tile_base[k+1]
	if (tpb)
		lo = hi = min(b / tpb, nb - 1u);
	while (hi - lo > 1) {
		const uint32_t mid = (lo + hi) >> 1;
		if (__builtin_amdgcn_readfirstlane(desc[mid].tile_base) <= b)
			lo = mid;
		else
			hi = mid;
	}
	const mosrx_qdesc *d = &desc[lo];
	mosrx_kparams kp;
	kp.frames = d->frames;
	kp.off = d->off;
	kp.len = d->len;
	kp.out = d->out;
	kp.tables = qp.tables;
	kp.counters = qp.counters;
	kp.fhash = d->fhash;
	kp.bmatch = (VAR & VAR_BPF) ? d->bmatch : nullptr;
	kp.tinfo = (VAR & VAR_BPF) ? nullptr : d->tinfo;
	kp.frames_bytes = d->frames_bytes;
	kp.n = d->n;
	kp.flags = qp.flags;
	kp.uni = d->uni;
	classify_tile<KIND, VAR>(kp, b - d->tile_base);
}

template <int KIND, int VAR>
__global__ __launch_bounds__(WG_THREADS(KIND)) __attribute__((amdgpu_waves_per_eu(MIN_WAVES(KIND))))
void mosrx_classify_queue_kernel(const mosrx_qdesc *desc, uint32_t tpb, uint32_t nb, mosrx_qparams qp)
{
	// desc / tpb / nb preloaded (see mosrx_classify_kernel): the batch lookup starts at dispatch
	queue_tile<KIND, VAR>(desc, tpb, nb, qp);
}

#ifndef __HIPCC_RTC__
// Streaming-read ceiling of the box: each workgroup reads one contiguous slab
// with coalesced non-temporal 16-byte loads, 8 in flight per lane; a
// data-dependent sink keeps them live.  32 KiB slabs (grid bytes / 32 KiB):
// the fastest shape of scripts/probe_bw.hip (6.9-7.0 TB/s at 512-800 MiB per
// launch vs 6.7-6.9 with 2048 slabs).  Diagnostic for the roofline report.
#define BW_U 8
#define BW_SLAB (32u << 10)
__global__ __launch_bounds__(256) void mosrx_read_bw_kernel(const u32x4 *p, uint64_t n16, uint32_t *sink)
{
	uint32_t acc = 0;
	const uint64_t per = (n16 + gridDim.x - 1) / gridDim.x;
	const uint64_t lo = (uint64_t)blockIdx.x * per, hi = min(n16, lo + per);
	for (uint64_t i = lo + threadIdx.x; i < hi; i += 256u * BW_U) {
		u32x4 v[BW_U];
#pragma unroll
		for (int u = 0; u < BW_U; u++) {
			const uint64_t j = i + 256u * u;
			v[u] = j < hi ? __builtin_nontemporal_load(p + j) : (u32x4){0, 0, 0, 0};
		}
#pragma unroll
		for (int u = 0; u < BW_U; u++)
			acc += v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
	}
	if (acc == 0x9E3779B9u)
		sink[0] = acc;
}

static uint32_t bw_grid(uint64_t bytes)
{
	const uint64_t g = bytes / BW_SLAB;
	return (uint32_t)(g < 2048u ? 2048u : g > 65535u ? 65535u : g);
}

extern "C" int mosrx_launch_read_bw(const void *p, uint64_t bytes, uint32_t *sink, void *stream)
{
	hipLaunchKernelGGL(mosrx_read_bw_kernel, dim3(bw_grid(bytes)), dim3(256), 0, (hipStream_t)stream,
	                   (const u32x4 *)p, bytes / 16, sink);
	return hipGetLastError() == hipSuccess ? 0 : -EIO;
}

// Host -> HBM pull by the CUs (mosrx_memcpy_h2d_pull): every lane reads 16-byte
// chunks of pinned host memory over PCIe, PULL_U in flight, and stores them to
// HBM; the byte head / tail outside the 16-byte grid by lane 0 of block 0.  The
// SDMA engine's alternative for the backend's group copies.
#define PULL_U 8
__global__ __launch_bounds__(256) void mosrx_pull_kernel(uint8_t *dst, const uint8_t *src, uint64_t bytes)
{
	const uint64_t head = (16u - ((uintptr_t)dst & 15u)) & 15u;
	const uint64_t h = head < bytes ? head : bytes;
	const uint64_t n16 = (bytes - h) / 16u;
	u32x4 *d = (u32x4 *)(dst + h);
	const u32x4 *s = (const u32x4 *)(src + h);
	const uint64_t step = (uint64_t)gridDim.x * 256u * PULL_U;
	for (uint64_t i = (uint64_t)blockIdx.x * 256u * PULL_U + threadIdx.x; i < n16; i += step) {
		u32x4 v[PULL_U];
#pragma unroll
		for (int u = 0; u < PULL_U; u++) {
			const uint64_t j = i + 256u * u;
			if (j < n16)
				v[u] = s[j];
		}
#pragma unroll
		for (int u = 0; u < PULL_U; u++) {
			const uint64_t j = i + 256u * u;
			if (j < n16)
				d[j] = v[u];
		}
	}
	if (blockIdx.x == 0 && threadIdx.x == 0) {
		for (uint64_t k = 0; k < h; k++)
			dst[k] = src[k];
		for (uint64_t k = h + n16 * 16u; k < bytes; k++)
			dst[k] = src[k];
	}
}

extern "C" int mosrx_launch_pull(void *dst, const void *src, uint64_t bytes, void *stream)
{
	uint64_t g = bytes / (256u * PULL_U * 16u);
	if (!bytes)
		return 0;
	g = g < 1 ? 1 : g > 4096 ? 4096 : g;
	hipLaunchKernelGGL(mosrx_pull_kernel, dim3((uint32_t)g), dim3(256), 0, (hipStream_t)stream, (uint8_t *)dst,
	                   (const uint8_t *)src, bytes);
	return hipGetLastError() == hipSuccess ? 0 : -EIO;
}

// An empty kernel of a classify launch's grid: its dispatch-stamped duration is
// what the stamp itself reads for a launch that does nothing (mosrx_probe_stamp_floor;
// the short rows' bench figures are stated against it).  Diagnostic only.
__global__ void mosrx_empty_kernel(uint32_t) {}
#endif

#ifndef __HIPCC_RTC__
// Dispatch-stamped timing (mosrx_time_op_dispatch / mosrx_time_queue_dispatch):
// the next classify or queue launch of this thread carries a start / stop
// event pair that the runtime stamps at the dispatch's own begin and end
// (hipExtLaunchKernel) -- the kernel duration rocprofv3's trace reports,
// without the gap between back-to-back dispatches that events recorded around
// the launches include.  The count lets the caller check that an operation
// was exactly one launch.
static thread_local hipEvent_t t_stamp0, t_stamp1;
static thread_local uint32_t t_launches;
extern "C" void mosrx__stamp_next(void *start, void *stop)
{
	t_stamp0 = (hipEvent_t)start;
	t_stamp1 = (hipEvent_t)stop;
}
extern "C" uint32_t mosrx__launch_count(void) { return t_launches; }
// For launches made elsewhere (the hipRTC modules of bpf_jit.c, the interpreter
// kernel): counts the launch and hands over the pending stamp pair, if any.
extern "C" int mosrx__stamp_take(void **start, void **stop)
{
	t_launches++;
	*start = t_stamp0;
	*stop = t_stamp1;
	t_stamp0 = t_stamp1 = nullptr;
	return *start != nullptr;
}

template <typename... P, typename... A>
static void launch_one(void (*k)(P...), uint32_t grid, uint32_t block, hipStream_t s, const A &...a)
{
	t_launches++;
	if (t_stamp0) {
		hipExtLaunchKernelGGL(k, dim3(grid), dim3(block), 0, s, t_stamp0, t_stamp1, 0, a...);
		t_stamp0 = t_stamp1 = nullptr;
	} else {
		hipLaunchKernelGGL(k, dim3(grid), dim3(block), 0, s, a...);
	}
}

extern "C" int mosrx_launch_empty(int kind, uint32_t tiles, void *stream)
{
	if (kind < 0 || kind >= MOSRX_KIND_COUNT || tiles == 0)
		return -EINVAL;
	launch_one(mosrx_empty_kernel, tiles, WG_THREADS(kind), (hipStream_t)stream, tiles);
	return hipGetLastError() == hipSuccess ? 0 : -EIO;
}

template <int KIND, int VAR>
static void launch_queue_v(const mosrx_qparams *qp, uint32_t total_tiles, hipStream_t s)
{
	launch_one(mosrx_classify_queue_kernel<KIND, VAR>, total_tiles, WG_THREADS(KIND), s, qp->desc, qp->tpb, qp->nb,
	           *qp);
}

template <int KIND, int VAR>
static void launch_v(const mosrx_kparams *kp, hipStream_t s)
{
	constexpr uint32_t tile = MOSRX_KIND_FRAMES(KIND);
	launch_one(mosrx_classify_kernel<KIND, VAR>, (kp->n + tile - 1) / tile, WG_THREADS(KIND), s, kp->off, kp->len,
	           kp->frames, kp->tables, kp->frames_bytes, kp->n, kp->flags, kp->uni, *kp);
}

// Compiled variants: 0 = default cache policy, 2 = non-temporal tail stream
// (the nt header-window variants 1 and 3 measured slower everywhere and are
// folded onto 0 and 2).
extern "C" int mosrx_launch_queue(const mosrx_qparams *qp, uint32_t total_tiles, int kind, int variant, void *stream)
{
	if (!qp || qp->nb == 0 || total_tiles == 0)
		return qp ? 0 : -EINVAL;
	if (kind < 0 || kind >= MOSRX_KIND_COUNT)
		return -EINVAL;
	const hipStream_t s = (hipStream_t)stream;
	// [hinted][kind][form]: the SMALL tile's hinted forms (VAR_UNI) when some
	// batch of the queue carries a layout hint (qp->uni); the stream tile has none
#define QROW(k, u)                                                                                                 \
	{launch_queue_v<k, 0 | (u)>, launch_queue_v<k, 2 | (u)>, launch_queue_v<k, 2 | VAR_TI>,                        \
	 launch_queue_v<k, VAR_C8 | (u)>, launch_queue_v<k, 2 | VAR_C8 | (u)>}
	static void (*const tab[2][MOSRX_KIND_COUNT][5])(const mosrx_qparams *, uint32_t, hipStream_t) = {
		{QROW(MOSRX_KIND_SMALL, 0), QROW(MOSRX_KIND_S13, 0)}, {QROW(MOSRX_KIND_SMALL, VAR_UNI), QROW(MOSRX_KIND_S13, 0)}};
#undef QROW
	const int tv = (variant >> 1) & 1;
	const int hinted = qp->uni && total_tiles <= MOSRX_UNI_MAX_TILES;
	tab[hinted][kind][qp->tinfo == 1 ? 2 : qp->tinfo == 2 ? 3 + tv : tv](qp, total_tiles, s);
	return hipGetLastError() == hipSuccess ? 0 : -EIO;
}

extern "C" int mosrx_launch_classify(const mosrx_kparams *kp, int kind, int variant, void *stream)
{
	if (!kp || kp->n == 0)
		return kp ? 0 : -EINVAL;
	if (kind < 0 || kind >= MOSRX_KIND_COUNT)
		return -EINVAL;
	const hipStream_t s = (hipStream_t)stream;
	// [hinted][kind][form], as in mosrx_launch_queue (kp->uni != 0: the SMALL tile's VAR_UNI forms)
#define KROW(k, u)                                                                                         \
	{launch_v<k, 0 | (u)>, launch_v<k, 2 | (u)>, launch_v<k, 2 | VAR_TX>, launch_v<k, 2 | VAR_TI>,          \
	 launch_v<k, VAR_C8 | (u)>, launch_v<k, 2 | VAR_C8 | (u)>}
	static void (*const tab[2][MOSRX_KIND_COUNT][6])(const mosrx_kparams *, hipStream_t) = {
		{KROW(MOSRX_KIND_SMALL, 0), KROW(MOSRX_KIND_S13, 0)}, {KROW(MOSRX_KIND_SMALL, VAR_UNI), KROW(MOSRX_KIND_S13, 0)}};
#undef KROW
	const int tv = (variant >> 1) & 1;
	// MOSRX_KF_COMPACT is the host's request for 8-byte records; the kernel's flags never carry it
	const int v = (kp->flags & (MOSRX_KF_TX_IP | MOSRX_KF_TX_TCP)) ? 2 : kp->tinfo ? 3
	            : (kp->flags & MOSRX_KF_COMPACT) ? 4 + tv : tv;
	mosrx_kparams k = *kp;
	k.flags &= ~(uint32_t)MOSRX_KF_COMPACT;
	const uint32_t tiles = (k.n + MOSRX_KIND_FRAMES(kind) - 1) / MOSRX_KIND_FRAMES(kind);
	tab[k.uni && tiles <= MOSRX_UNI_MAX_TILES ? 1 : 0][kind][v](&k, s);
	return hipGetLastError() == hipSuccess ? 0 : -EIO;
}
#endif   // __HIPCC_RTC__
