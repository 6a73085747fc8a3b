// probe_h2.h — stream tile with H header waves (diagnostic only).
//
// The round-1 review asked for the S-shape with the 64 frames of a tile parsed
// by two header waves (32 frames each) next to the streamers.  Header wave h
// takes the frames of lanes [64h/H, 64(h+1)/H): its window loads and parse
// cover half the frames, the other lanes sit idle.  Streamers as in
// classify_tile_stream.  Each header wave fills the LDS tables itself (the same
// words) and keeps its own reason counts.  Included after mosrx_kernels.hip by
// scripts/probe_timeline.hip; records compared against the library shape there.
#pragma once

template <int H, int S, int VAR, int U = STREAM_U>
__device__ __forceinline__ void classify_tile_stream_h(const mosrx_kparams &kp, uint32_t tile)
{
	constexpr int AUX = TAIL_AUX(VAR);
	constexpr int WEND = MOSRX_WINDOW_END_STREAM;
	constexpr int NLOAD = WIN_NLOAD(WEND);
	constexpr uint32_t T = 64;
	constexpr uint32_t FPW = 64u / H;   // frames per header wave
	__shared__ __attribute__((aligned(16))) uint32_t s_tab[MOSRX_TAB_WORDS];
	__shared__ uint32_t s_part[S][64];
	__shared__ uint32_t s_cnt[H][MOSRX_R_COUNT + 1];

	const uint32_t t = threadIdx.x, lane = t & 63u, wave = t >> 6;
	const __amdgpu_buffer_rsrc_t rs = frame_rsrc(kp.frames, kp.frames_bytes);
	const uint32_t nbytes = kp.frames_bytes;
	const uint32_t nact = min(T, kp.n - tile * T);

	const uint32_t p = tile * T + lane;
	const bool active = lane < nact;
	uint32_t o = 0, cap = 0;
	if (active) {
		o = kp.off[p];
		cap = eff_caplen(o, kp.len[p], nbytes);
	}
	const uint32_t lo_l = (o + (uint32_t)WEND) & ~15u;
	const uint32_t hi_l = active ? o + cap : 0u;
	const uint32_t onext = (uint32_t)__shfl_down((int)o, 1);
	const bool sorted = __ballot(lane + 1u < nact && onext < hi_l) == 0;

	if (wave < (uint32_t)H) {
		const bool mine = active && lane / FPW == wave;
		uint32_t *cnt = s_cnt[wave];
		hdr_win_t win;
		hdr_load<WIN_AUX(VAR), NLOAD>(rs, nbytes, o, mine, win);
		const bool cand = hi_l > lo_l;
		const u32x4 ov = load16<WIN_AUX(VAR)>(rs, mine && sorted && cand ? (hi_l - 1u) & ~15u : ZERO_OFF, 0);
		{
			const u32x4 *tg = reinterpret_cast<const u32x4 *>(kp.tables);
			const u32x4 a = tg[lane], b = tg[lane + 64];
			reinterpret_cast<u32x4 *>(s_tab)[lane] = a;
			reinterpret_cast<u32x4 *>(s_tab)[lane + 64] = b;
			if (lane <= MOSRX_R_COUNT)
				cnt[lane] = 0;
		}
		const hdr_t h = hdr_parse<VAR, WEND>(win, o, mine ? cap : 0u, mine, kp.flags, s_tab, kp.tables, rs, nbytes);
		__syncthreads();   // B: s_part ready
		uint32_t tail = 0;
		if (h.has_tail) {
#pragma unroll
			for (int s = 0; s < S; s++)
				tail += s_part[s][lane];
			if (sorted)
				tail -= chunk_overshoot(ov, (hi_l - 1u) & ~15u, hi_l);
		}
		hdr_emit<VAR>(kp, rs, nbytes, h, lo_l, hi_l, tail, p, mine, lane, cnt);
		if (kp.counters && lane < MOSRX_R_COUNT && cnt[lane])
			atomicAdd(&kp.counters[(blockIdx.x % MOSRX_CNT_SHARDS) * MOSRX_CNT_STRIDE + lane], cnt[lane]);
	} else {
		const uint32_t sidx = wave - (uint32_t)H;
		uint32_t *row = s_part[sidx];
		row[lane] = 0;
		const uint64_t cmask = __ballot(hi_l > lo_l);
		if (sorted && cmask) {
			uint32_t A = uni(__builtin_amdgcn_readlane(lo_l, (int)__builtin_ctzll(cmask)));
			const uint32_t Z = uni(__builtin_amdgcn_readlane(hi_l, 63 - (int)__builtin_clzll(cmask)));
			A = min(A, uni(__builtin_amdgcn_readfirstlane(o)) & ~15u);
			stream_scan<S, AUX, 0, U>(rs, lo_l, hi_l, A, Z, sidx, lane, row);
		} else if (!sorted) {
			stream_frames<S, AUX>(rs, lo_l, hi_l, sidx, lane, row);
		}
		__syncthreads();   // B
	}
}
