// probe_decoupled.h — classify_tile_stream_nt (diagnostic only): the S13 tile
// with its header wave and streamers decoupled over NT tiles.  Measured slower
// than S13 (M1500 512K: 139.4 vs 136.0 us; IMIX 2M: 173.3 vs 155.3 us), so it
// left the library.  Included after mosrx_kernels.hip.
#pragma once

// NT stream tiles (64 frames each) per workgroup with the header wave and the
// streamers DECOUPLED: the streamers walk the NT tiles' spans back to back,
// publishing each tile's rows in LDS with a counter (release at workgroup
// scope), and the header wave parses tile k while they stream tile k+1, waiting
// only on tile k's counter before it emits tile k's records.  One workgroup
// barrier at the start (the counters zeroed), none after: a tile's header
// chain (descriptors -> windows -> parse) no longer holds the streamers, so a
// workgroup keeps its loads in flight over NT tiles.  Everything per tile is
// classify_tile_stream's.
template <int S, int VAR, int NT, int U = STREAM_U>
__device__ __forceinline__ void classify_tile_stream_nt(const mosrx_kparams &kp, uint32_t tile)
{
	constexpr int AUX = TAIL_AUX(VAR);
	__shared__ __attribute__((aligned(16))) uint32_t s_tab[MOSRX_TAB_WORDS];
	__shared__ uint32_t s_part[NT][S][64];   // streamer s's tail sums, per tile
	__shared__ uint32_t s_cnt[MOSRX_R_COUNT + 1];
	__shared__ uint32_t s_done[NT];          // streamers finished with tile k

	const uint32_t t = threadIdx.x, lane = t & 63u, wave = t >> 6;
	const __amdgpu_buffer_rsrc_t rs = frame_rsrc(kp.frames, kp.frames_bytes);
	const uint32_t nbytes = kp.frames_bytes;
	if (t < (uint32_t)NT)
		s_done[t] = 0;
	__syncthreads();

	if (wave == 0) {
		{
			const u32x4 *tg = reinterpret_cast<const u32x4 *>(kp.tables);
			const u32x4 a = tg[lane], b = tg[lane + 64];
			reinterpret_cast<u32x4 *>(s_tab)[lane] = a;
			reinterpret_cast<u32x4 *>(s_tab)[lane + 64] = b;
			if (lane <= MOSRX_R_COUNT)
				s_cnt[lane] = 0;
		}
#pragma unroll 1
		for (uint32_t k = 0; k < (uint32_t)NT; k++) {
			const uint32_t base = (tile * NT + k) * 64u;
			if (base >= kp.n)
				break;
			const uint32_t nact = min(64u, kp.n - base);
			const uint32_t p = base + lane;
			const bool active = lane < nact;
			uint32_t o = 0, cap = 0;
			if (active) {
				o = kp.off[p];
				cap = eff_caplen(o, kp.len[p], nbytes);
			}
			const uint32_t lo_l = (o + (uint32_t)MOSRX_WINDOW_END_FULL) & ~15u;
			const uint32_t hi_l = active ? o + cap : 0u;
			const uint32_t onext = (uint32_t)__shfl_down((int)o, 1);
			const bool sorted = __ballot(lane + 1u < nact && onext < hi_l) == 0;
			hdr_win_t win;
			hdr_load<WIN_AUX(VAR)>(rs, nbytes, o, active, win);
			const bool cand = hi_l > lo_l;
			const u32x4 ov = load16<WIN_AUX(VAR)>(rs, sorted && cand ? (hi_l - 1u) & ~15u : ZERO_OFF, 0);
			const hdr_t h = hdr_parse<VAR, MOSRX_WINDOW_END_FULL>(win, o, cap, active, kp.flags, s_tab, kp.tables, rs, nbytes);
			while (__hip_atomic_load(&s_done[k], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < (uint32_t)S)
				__builtin_amdgcn_s_sleep(1);
			uint32_t tail = 0;
			if (h.has_tail) {
#pragma unroll
				for (int s = 0; s < S; s++)
					tail += s_part[k][s][lane];
				if (sorted)
					tail -= chunk_overshoot(ov, (hi_l - 1u) & ~15u, hi_l);
			}
			hdr_emit<VAR>(kp, rs, nbytes, h, lo_l, hi_l, tail, p, active, lane, s_cnt);
		}
		// only this wave counted: it adds the workgroup's counts to its shard
		if (kp.counters && lane < MOSRX_R_COUNT && s_cnt[lane])
			atomicAdd(&kp.counters[(blockIdx.x % MOSRX_CNT_SHARDS) * MOSRX_CNT_STRIDE + lane], s_cnt[lane]);
	} else {
		const uint32_t sidx = wave - 1u;
#pragma unroll 1
		for (uint32_t k = 0; k < (uint32_t)NT; k++) {
			const uint32_t base = (tile * NT + k) * 64u;
			if (base >= kp.n)
				break;
			const uint32_t nact = min(64u, kp.n - base);
			const bool active = lane < nact;
			uint32_t o = 0, cap = 0;
			if (active) {
				o = kp.off[base + lane];
				cap = eff_caplen(o, kp.len[base + lane], nbytes);
			}
			const uint32_t lo_l = (o + (uint32_t)MOSRX_WINDOW_END_FULL) & ~15u;
			const uint32_t hi_l = active ? o + cap : 0u;
			const uint32_t onext = (uint32_t)__shfl_down((int)o, 1);
			const bool sorted = __ballot(lane + 1u < nact && onext < hi_l) == 0;
			uint32_t *row = s_part[k][sidx];
			row[lane] = 0;
			const uint64_t cmask = __ballot(hi_l > lo_l);
			if (sorted && cmask) {
				const uint32_t A = uni(__builtin_amdgcn_readlane(lo_l, (int)__builtin_ctzll(cmask)));
				const uint32_t Z = uni(__builtin_amdgcn_readlane(hi_l, 63 - (int)__builtin_clzll(cmask)));
				stream_scan<S, AUX, 0, U>(rs, lo_l, hi_l, A, Z, sidx, lane, row);
			} else if (!sorted) {
				stream_frames<S, AUX>(rs, lo_l, hi_l, sidx, lane, row);
			}
			if (lane == 0)
				__hip_atomic_fetch_add(&s_done[k], 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
		}
	}
}
