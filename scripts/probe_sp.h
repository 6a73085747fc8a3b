// probe_sp.h — the pipelined stream tile (SP), diagnostic only: NT tiles per
// workgroup, header windows prefetched into LDS with buffer_load ... lds, the
// streamers' shares of the NT spans as one stream, no barrier after the start.
// Records equal the library's S13 (scripts/probe_timeline.hip checks), but it
// measured slower: IMIX 256K 23.0 (NT 1) / 24.1 (NT 2) vs 20.9 us, M1500 64K
// 19.1 / 20.9 vs 17.9 us (profiles/r02_probe/).  Included after mosrx_kernels.hip.
#pragma once

// ---------------------------------------------------------------------------
// pipelined stream tiles (SP): NT consecutive 64-frame tiles per workgroup
// ---------------------------------------------------------------------------
// In the S13 tile every phase is paid once per tile and in series: descriptor
// latency, then the header windows (one more HBM round trip) and the parse on
// one side, the span stream on the other, one barrier, the records.  With two
// or three rounds of tiles per launch those latencies are not hidden.  Here a
// workgroup owns NT tiles and nothing waits on a workgroup barrier after the
// start: the streamers stream the NT spans back to back (the loads of tile k+1
// are in flight while tile k's last blocks are summed), publishing each tile's
// rows with an LDS counter; the header wave prefetches tile k+1's windows into
// LDS with buffer_load ... lds (no registers held) while it parses tile k,
// waits on tile k's counter only to emit.
#define SP_MAX_NT 2
#define SP_CHUNKS 7            // the 6 window chunks + the chunk holding the capture's last byte
typedef __attribute__((address_space(3))) void lds_void;

struct sp_view {               // one tile's frames, lane = frame
	uint32_t o, cap, lo_l, hi_l;
	bool active, sorted;
};

__device__ __forceinline__ sp_view sp_tile_view(const uint32_t *s_o, const uint32_t *s_cap, uint32_t nact, uint32_t lane)
{
	sp_view v;
	v.active = lane < nact;
	v.o = s_o[lane];
	v.cap = s_cap[lane];
	v.lo_l = (v.o + (uint32_t)MOSRX_WINDOW_END_STREAM) & ~15u;
	v.hi_l = v.active ? v.o + v.cap : 0u;
	const uint32_t onext = s_o[min(lane + 1u, 63u)];
	v.sorted = __ballot(lane + 1u < nact && onext < v.hi_l) == 0;
	return v;
}

// Tile k's 64 header windows (6 chunks per lane) and the chunk holding each
// capture's last byte, straight into LDS buffer `buf` (lane l's chunk m at
// buf[m][l]): buffer_load ... lds, no registers held while they are in flight.
template <int AUX>
__device__ __forceinline__ void sp_issue_windows(__amdgpu_buffer_rsrc_t rs, uint32_t nbytes, const sp_view &v,
                                                 u32x4 (*buf)[64])
{
	const uint32_t wbase = v.active ? ((v.o + 2u) & ~3u) : nbytes;   // out of range -> 0
	const uint32_t ovoff = v.sorted && v.hi_l > v.lo_l ? (v.hi_l - 1u) & ~15u : ZERO_OFF;
#pragma unroll
	for (int m = 0; m < WIN_RAW / 4; m++)
		__builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void *)&buf[m][0], 16, wbase + 16u * m, 0, 0, AUX);
	__builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void *)&buf[WIN_RAW / 4][0], 16, ovoff, 0, 0, AUX);
}

// Streamer sidx's share of a tile's span: blocks [b0, b0 + nb) of 1 KiB from A
// (nb = 0: nothing for this streamer, or the tile is not in buffer order).
struct sp_share {
	uint32_t A, b0, nb, R1;
};
template <int S>
__device__ __forceinline__ sp_share sp_tile_share(const sp_view &v, uint32_t sidx)
{
	sp_share sh = {0u, 0u, 0u, 0u};
	const uint64_t cmask = __ballot(v.hi_l > v.lo_l);
	if (v.sorted && cmask) {
		uint32_t A = uni(__builtin_amdgcn_readlane(v.lo_l, (int)__builtin_ctzll(cmask)));
		const uint32_t Z = uni(__builtin_amdgcn_readlane(v.hi_l, 63 - (int)__builtin_clzll(cmask)));
		A = min(A, uni(__builtin_amdgcn_readfirstlane(v.o)) & ~15u);   // from the tile's first byte
		const uint32_t nblk = (Z - A + 1023u) >> 10;
		const uint32_t b0 = uni((nblk * sidx) / S), b1 = uni((nblk * (sidx + 1u)) / S);
		sh.A = A; sh.b0 = b0; sh.nb = b1 - b0; sh.R1 = A + (b1 << 10);
	}
	return sh;
}

template <int S, int VAR, int NT, int DBG = 0, int U = STREAM_U>
__device__ __forceinline__ void classify_tile_sp(const mosrx_kparams &kp, uint32_t grp)
{
	constexpr int AUX = TAIL_AUX(VAR);
	static_assert(NT >= 1 && NT <= SP_MAX_NT, "tiles per workgroup");
	__shared__ __attribute__((aligned(16))) uint32_t s_tab[MOSRX_TAB_WORDS];
	__shared__ __attribute__((aligned(16))) u32x4 s_win[2][SP_CHUNKS][64];
	__shared__ uint32_t s_o[NT][64], s_cap[NT][64];
	__shared__ uint32_t s_part[NT][S][64];
	__shared__ uint32_t s_cnt[MOSRX_R_COUNT + 1];
	__shared__ uint32_t s_done[NT];

	const uint32_t t = threadIdx.x, lane = t & 63u, wave = t >> 6;
	const __amdgpu_buffer_rsrc_t rs = frame_rsrc(kp.frames, kp.frames_bytes);
	const uint32_t nbytes = kp.frames_bytes;
	const uint32_t tile0 = grp * NT;
	const uint32_t ntile = uni(min((uint32_t)NT, ((kp.n + 63u) >> 6) - tile0));

	// every tile's descriptors into LDS (wave w loads tile w), rows zeroed, counters reset
	if (wave < ntile) {
		const uint32_t p = (tile0 + wave) * 64u + lane;
		uint32_t o = 0, cap = 0;
		if (p < kp.n) {
			o = kp.off[p];
			cap = eff_caplen(o, kp.len[p], nbytes);
		}
		s_o[wave][lane] = o;
		s_cap[wave][lane] = cap;
	}
	if (wave >= 1) {
#pragma unroll
		for (int k = 0; k < NT; k++)
			s_part[k][wave - 1][lane] = 0;
	}
	if (t < (uint32_t)NT)
		s_done[t] = 0;
	__syncthreads();   // the only workgroup barrier

	if (wave == 0) {
		// ---- header wave ----
		{
			const u32x4 *tg = reinterpret_cast<const u32x4 *>(kp.tables);
			const u32x4 a = tg[lane], b = tg[lane + 64];
			reinterpret_cast<u32x4 *>(s_tab)[lane] = a;
			reinterpret_cast<u32x4 *>(s_tab)[lane + 64] = b;
			if (lane <= MOSRX_R_COUNT)
				s_cnt[lane] = 0;
		}
		sp_issue_windows<WIN_AUX(VAR)>(rs, nbytes, sp_tile_view(s_o[0], s_cap[0], min(64u, kp.n - tile0 * 64u), lane),
		                               s_win[0]);
#pragma unroll
		for (int k = 0; k < NT; k++) {
			if ((uint32_t)k >= ntile)
				break;
			// tile k's windows: every vector memory op but the newest one (tile
			// k-1's last record store) has completed
			if (k == 0)
				asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
			else
				asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
			hdr_win_t win;
#pragma unroll
			for (int m = 0; m < WIN_RAW / 4; m++) {
				const u32x4 x = s_win[k & 1][m][lane];
				win.raw[4 * m + 0] = x.x; win.raw[4 * m + 1] = x.y; win.raw[4 * m + 2] = x.z; win.raw[4 * m + 3] = x.w;
			}
			const u32x4 ov = s_win[k & 1][WIN_RAW / 4][lane];
			asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // read before the buffer is refilled
			if (k + 1 < NT && (uint32_t)k + 1u < ntile)
				sp_issue_windows<WIN_AUX(VAR)>(
					rs, nbytes, sp_tile_view(s_o[k + 1], s_cap[k + 1], min(64u, kp.n - (tile0 + k + 1) * 64u), lane),
					s_win[(k + 1) & 1]);
			const uint32_t nact = min(64u, kp.n - (tile0 + k) * 64u);
			const sp_view v = sp_tile_view(s_o[k], s_cap[k], nact, lane);
			const uint32_t p = (tile0 + k) * 64u + lane;
			const hdr_t h = hdr_parse<VAR, MOSRX_WINDOW_END_STREAM>(win, v.o, v.cap, v.active, kp.flags, s_tab, kp.tables,
			                                                       rs, nbytes);
			while (__hip_atomic_load(&s_done[k], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < (uint32_t)S)
				__builtin_amdgcn_s_sleep(1);
			uint32_t tail = 0;
			if (h.has_tail) {
#pragma unroll
				for (int s2 = 0; s2 < S; s2++)
					tail += s_part[k][s2][lane];
				if (v.sorted)
					tail -= chunk_overshoot(ov, (v.hi_l - 1u) & ~15u, v.hi_l);
			}
			hdr_emit<VAR>(kp, rs, nbytes, h, v.lo_l, v.hi_l, tail, p, v.active, lane, s_cnt);
		}
		if (kp.counters && lane < MOSRX_R_COUNT && s_cnt[lane])
			atomicAdd(&kp.counters[(blockIdx.x % MOSRX_CNT_SHARDS) * MOSRX_CNT_STRIDE + lane], s_cnt[lane]);
		return;
	}

	// ---- streamer sidx: its shares of the NT spans as one stream of blocks, U loads in flight ----
	const uint32_t sidx = wave - 1u;
	sp_share sh[NT];
	uint32_t unsorted = 0, total = 0;
#pragma unroll
	for (int k = 0; k < NT; k++) {
		sh[k] = (sp_share){0u, 0u, 0u, 0u};
		if ((uint32_t)k < ntile) {
			const sp_view v = sp_tile_view(s_o[k], s_cap[k], min(64u, kp.n - (tile0 + k) * 64u), lane);
			if (!v.sorted)
				unsorted |= 1u << k;
			sh[k] = sp_tile_share<S>(v, sidx);
		}
		total += sh[k].nb;
	}
	// item j of the stream -> (tile, block address)
	auto item_tile = [&](uint32_t j) -> uint32_t {
		uint32_t k = 0, acc = sh[0].nb;
#pragma unroll
		for (int q = 1; q < NT; q++) {
			k = j >= acc ? (uint32_t)q : k;
			acc += sh[q].nb;
		}
		return k;
	};
	auto item_addr = [&](uint32_t j) -> uint32_t {
		uint32_t a = sh[0].A + ((sh[0].b0 + j) << 10), acc = sh[0].nb;
#pragma unroll
		for (int q = 1; q < NT; q++) {
			a = j >= acc ? sh[q].A + ((sh[q].b0 + j - acc) << 10) : a;
			acc += sh[q].nb;
		}
		return a;
	};
	u32x4 v[U];
#pragma unroll
	for (int i = 0; i < U; i++)
		v[i] = load16<AUX>(rs, (uint32_t)i < total ? item_addr(i) + 16u * lane : ZERO_OFF, 0);
	uint32_t sk = 0xFFFFFFFFu, sR1 = 0, carry = 0, acc = 0, lo_l = 0, ec_l = 0, signalled = 0;
	bool cand = false;
#pragma unroll 1
	for (uint32_t j0 = 0; j0 < total; j0 += U) {
#pragma unroll
		for (int i = 0; i < U; i++) {
			const uint32_t j = j0 + (uint32_t)i;
			if (j < total) {
				const uint32_t k = uni(item_tile(j));
				if (k != sk) {
					// leave tile sk (its row, tails continuing past the run), signal every tile below k
					if (sk != 0xFFFFFFFFu) {
						if (cand && lo_l < sR1 && ec_l >= sR1)
							acc += carry;
						s_part[sk][sidx][lane] = acc;
					}
					for (; signalled < k; signalled++)
						if (!((unsorted >> signalled) & 1u) && lane == 0)
							__hip_atomic_fetch_add(&s_done[signalled], 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
					const sp_view tv = sp_tile_view(s_o[k], s_cap[k], min(64u, kp.n - (tile0 + k) * 64u), lane);
					sk = k;
					sR1 = 0;
#pragma unroll
					for (int q = 0; q < NT; q++)
						if ((uint32_t)q == k)
							sR1 = sh[q].R1;
					lo_l = tv.lo_l; ec_l = (tv.hi_l - 1u) & ~15u; cand = tv.hi_l > tv.lo_l;
					carry = 0; acc = 0;
				}
				const uint32_t c0 = item_addr(j);
				uint32_t s = add16x2(0u, v[i].x);
				s = add16x2(s, v[i].y);
				s = add16x2(s, v[i].z);
				s = add16x2(s, v[i].w);
				const uint32_t X = carry + wave_scan(s);
				carry = (uint32_t)__builtin_amdgcn_readlane((int)X, 63);
				const uint32_t rl = lo_l - c0, re = ec_l - c0;
				const bool es = cand && rl < 1024u, ee = cand && re < 1024u;
				if (__ballot(es || ee)) {
					const uint32_t Es = (uint32_t)__builtin_amdgcn_ds_bpermute((int)((rl >> 2) & 0xFCu), (int)(X - s));
					const uint32_t Xe = (uint32_t)__builtin_amdgcn_ds_bpermute((int)((re >> 2) & 0xFCu), (int)X);
					acc = es ? acc - Es : acc;
					acc = ee ? acc + Xe : acc;
				}
			}
			const uint32_t jn = j + U;
			v[i] = load16<AUX>(rs, jn < total ? item_addr(jn) + 16u * lane : ZERO_OFF, 0);
		}
	}
	if (sk != 0xFFFFFFFFu) {
		if (cand && lo_l < sR1 && ec_l >= sR1)
			acc += carry;
		s_part[sk][sidx][lane] = acc;
	}
	for (; signalled < ntile; signalled++)
		if (!((unsorted >> signalled) & 1u) && lane == 0)
			__hip_atomic_fetch_add(&s_done[signalled], 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
	// tiles whose frames are not in buffer order: tail by tail
	for (uint32_t m = unsorted; m; m &= m - 1) {
		const uint32_t k = (uint32_t)__builtin_ctz(m);
		const sp_view tv = sp_tile_view(s_o[k], s_cap[k], min(64u, kp.n - (tile0 + k) * 64u), lane);
		stream_frames<S, AUX>(rs, tv.lo_l, tv.hi_l, sidx, lane, s_part[k][sidx]);
		if (lane == 0)
			__hip_atomic_fetch_add(&s_done[k], 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
	}
}

