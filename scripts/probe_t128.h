// probe_t128.h — stream tile over F x 64 frames (diagnostic only).
//
// A 256K-frame IMIX batch is 4096 64-frame tiles: two rounds of the 2048
// resident workgroups, and the second round's late starters set a ~6 us drain
// (DESIGN.md §4.4).  Here one workgroup takes F x 64 frames: the header wave
// parses its F frame sets one after the other (window loads of set j + 1 in
// flight during the parse of set j), the streamers scan the whole span once and
// resolve each set's tails with their own ds_bpermute pair per block.  F = 2
// halves the tile count (one round for 256K frames) and doubles the bytes per
// streamer.  Included after mosrx_kernels.hip by scripts/probe_timeline.hip;
// records compared against the library shape there.
#pragma once

// hdr_pend_t / hdr_pend / pend_emit: mosrx_kernels.hip

template <int F, int S, int AUX, int U>
__device__ __forceinline__ void stream_scan_f(__amdgpu_buffer_rsrc_t rs, const uint32_t (&lo_l)[F],
                                              const uint32_t (&hi_l)[F], uint32_t A, uint32_t Z, uint32_t sidx,
                                              uint32_t lane, uint32_t *row)
{
	const uint32_t nblk = (Z - A + 1023u) >> 10;
	const uint32_t b0 = uni((nblk * sidx) / S), b1 = uni((nblk * (sidx + 1u)) / S);
	const uint32_t R1 = A + (b1 << 10);
	uint32_t blo[F], bec[F], acc[F];
	int alo[F], aec[F];
#pragma unroll
	for (int j = 0; j < F; j++) {
		const bool cand = hi_l[j] > lo_l[j];
		const uint32_t ec = (hi_l[j] - 1u) & ~15u;
		blo[j] = cand ? (lo_l[j] - A) >> 10 : 0xFFFFFFFFu;
		bec[j] = cand ? (ec - A) >> 10 : 0xFFFFFFFFu;
		alo[j] = (int)(((lo_l[j] - A) >> 2) & 0xFCu);
		aec[j] = (int)(((ec - A) >> 2) & 0xFCu);
		acc[j] = 0;
	}
	uint32_t carry = 0;
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
			if (b < b1) {
				uint32_t s = add16x2(0u, v[i].x);
				s = add16x2(s, v[i].y);
				s = add16x2(s, v[i].z);
				s = add16x2(s, v[i].w);
				const uint32_t X = carry + wave_scan(s);
				carry = (uint32_t)__builtin_amdgcn_readlane((int)X, 63);
#pragma unroll
				for (int j = 0; j < F; j++) {
					const bool es = blo[j] == b, ee = bec[j] == b;
					if (__ballot(es || ee)) {
						const uint32_t Es = (uint32_t)__builtin_amdgcn_ds_bpermute(alo[j], (int)(X - s));
						const uint32_t Xe = (uint32_t)__builtin_amdgcn_ds_bpermute(aec[j], (int)X);
						acc[j] = es ? acc[j] - Es : acc[j];
						acc[j] = ee ? acc[j] + Xe : acc[j];
					}
				}
			}
			const uint32_t bn = b + U;
			v[i] = load16<AUX>(rs, bn < b1 ? A + (bn << 10) + 16u * lane : ZERO_OFF, 0);
		}
	}
#pragma unroll
	for (int j = 0; j < F; j++) {
		const uint32_t ec = (hi_l[j] - 1u) & ~15u;
		if (hi_l[j] > lo_l[j] && lo_l[j] < R1 && ec >= R1)
			acc[j] += carry;
		row[64 * j + lane] = acc[j];
	}
}

template <int F, int S, int VAR, int U = STREAM_U>
__device__ __forceinline__ void classify_tile_stream_f(const mosrx_kparams &kp, uint32_t tile)
{
	constexpr int AUX = TAIL_AUX(VAR);
	constexpr int WEND = MOSRX_WINDOW_END_STREAM;
	constexpr int NLOAD = WIN_NLOAD(WEND);
	constexpr uint32_t T = 64u * F;
	__shared__ __attribute__((aligned(16))) uint32_t s_tab[MOSRX_TAB_WORDS];
	__shared__ uint32_t s_part[S][T];
	__shared__ uint32_t s_cnt[MOSRX_R_COUNT + 1];

	const uint32_t t = threadIdx.x, lane = t & 63u, wave = t >> 6;
	const __amdgpu_buffer_rsrc_t rs = frame_rsrc(kp.frames, kp.frames_bytes);
	const uint32_t nbytes = kp.frames_bytes;
	const uint32_t nact = min(T, kp.n - tile * T);

	uint32_t o[F], cap[F], lo_l[F], hi_l[F];
	bool active[F];
#pragma unroll
	for (int j = 0; j < F; j++) {
		const uint32_t g = 64u * j + lane;
		active[j] = g < nact;
		o[j] = 0;
		cap[j] = 0;
		if (active[j]) {
			o[j] = kp.off[tile * T + g];
			cap[j] = eff_caplen(o[j], kp.len[tile * T + g], nbytes);
		}
		lo_l[j] = (o[j] + (uint32_t)WEND) & ~15u;
		hi_l[j] = active[j] ? o[j] + cap[j] : 0u;
	}
	// buffer order over all T frames (lane 63 of set j looks at lane 0 of set j + 1)
	bool sorted = true;
#pragma unroll
	for (int j = 0; j < F; j++) {
		uint32_t onext = (uint32_t)__shfl_down((int)o[j], 1);
		if (j + 1 < F && lane == 63u)
			onext = (uint32_t)__builtin_amdgcn_readfirstlane((int)o[j + 1]);
		sorted = sorted && __ballot(64u * j + lane + 1u < nact && onext < hi_l[j]) == 0;
	}

	if (wave == 0) {
		hdr_pend_t q[F];
		{
			const u32x4 *tg = reinterpret_cast<const u32x4 *>(kp.tables);
			const u32x4 a = tg[lane], b = tg[lane + 64];
			reinterpret_cast<u32x4 *>(s_tab)[lane] = a;
			reinterpret_cast<u32x4 *>(s_tab)[lane + 64] = b;
			if (lane <= MOSRX_R_COUNT)
				s_cnt[lane] = 0;
		}
#pragma unroll
		for (int j = 0; j < F; j++) {
			hdr_win_t win;
			hdr_load<WIN_AUX(VAR), NLOAD>(rs, nbytes, o[j], active[j], win);
			const bool cand = hi_l[j] > lo_l[j];
			const u32x4 ov = load16<WIN_AUX(VAR)>(rs, sorted && cand ? (hi_l[j] - 1u) & ~15u : ZERO_OFF, 0);
			const hdr_t h = hdr_parse<VAR, WEND>(win, o[j], cap[j], active[j], kp.flags, s_tab, kp.tables, rs, nbytes);
			const uint32_t p = tile * T + 64u * j + lane;
			// the parts of the output that do not depend on the tail go out now
			if (active[j] && kp.fhash)
				kp.fhash[p] = flow_hash(h);
			if constexpr (IS_TI(VAR)) {
				if (active[j])
					store_tcpinfo(kp.tinfo, p, h);
			}
			q[j] = hdr_pend(h, kp.flags, sorted && cand ? chunk_overshoot(ov, (hi_l[j] - 1u) & ~15u, hi_l[j]) : 0u);
		}
		__syncthreads();   // B: s_part ready
#pragma unroll
		for (int j = 0; j < F; j++) {
			uint32_t tail = 0;
			if (q[j].bits & 2u) {
#pragma unroll
				for (int s = 0; s < S; s++)
					tail += s_part[s][64 * j + lane];
				tail -= q[j].ovs;
			}
			pend_emit(kp, rs, nbytes, q[j], lo_l[j], hi_l[j], tail, tile * T + 64u * j + lane, active[j], lane, s_cnt);
		}
		if (kp.counters && lane < MOSRX_R_COUNT && s_cnt[lane])
			atomicAdd(&kp.counters[(blockIdx.x % MOSRX_CNT_SHARDS) * MOSRX_CNT_STRIDE + lane], s_cnt[lane]);
	} else {
		const uint32_t sidx = wave - 1u;
		uint32_t *row = s_part[sidx];
#pragma unroll
		for (int j = 0; j < F; j++)
			row[64 * j + lane] = 0;
		int jf = -1, jl = -1;
		uint64_t mf = 0, ml = 0;
#pragma unroll
		for (int j = 0; j < F; j++) {
			const uint64_t m = __ballot(hi_l[j] > lo_l[j]);
			if (m && jf < 0) { jf = j; mf = m; }
			if (m) { jl = j; ml = m; }
		}
		if (sorted && jf >= 0) {
			uint32_t A = 0, Z = 0;
#pragma unroll
			for (int j = 0; j < F; j++) {
				if (j == jf)
					A = uni(__builtin_amdgcn_readlane(lo_l[j], (int)__builtin_ctzll(mf)));
				if (j == jl)
					Z = uni(__builtin_amdgcn_readlane(hi_l[j], 63 - (int)__builtin_clzll(ml)));
			}
			A = min(A, uni(__builtin_amdgcn_readfirstlane(o[0])) & ~15u);
			stream_scan_f<F, S, AUX, U>(rs, lo_l, hi_l, A, Z, sidx, lane, row);
		} else if (!sorted) {
#pragma unroll
			for (int j = 0; j < F; j++)
				stream_frames<S, AUX>(rs, lo_l[j], hi_l[j], sidx, lane, row + 64 * j);
		}
		__syncthreads();   // B
	}
}
