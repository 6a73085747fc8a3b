// probe_persist2.hip — the IMIX / 1500 B single launch against its ramp and
// drain (diagnostic only).
//
// The library's stream tile (classify_tile_stream, unchanged) run as
//   grid           one workgroup per tile, block b = tile b (the library),
//   grid xcd       block b -> tile by the bijective XCD remap (blocks that share
//                  an XCD, b % 8, take one contiguous range of tiles: neighbour
//                  tiles share their boundary lines in one L2),
//   grid heavy     block b -> the b-th heaviest tile (span bytes, sorted on the
//                  host: a bound for any static heaviest-first order -- on a
//                  device-resident batch no one knows the spans before the launch),
//   persist xcd    resident workgroups pulling tiles from 8 per-XCD counters
//                  (XCC_ID from s_getreg; XCD x takes tiles x, x + 8, ...), the
//                  next index fetched while the current tile runs,
//   persist xcd heavy  the same over the heaviest-first order.
// Every form's records are checked against the library form's before timing.
#include "../mos-networking-stack_amd/csrc/mosrx_kernels.hip"
#include "../include/mosrx_trace.h"
#include <algorithm>
#include <numeric>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <vector>

#define CHK(x) do { if ((x) != hipSuccess) { printf("HIP error %s line %d\n", #x, __LINE__); return 1; } } while (0)
#define S 3
#define WG (64 * (1 + S))
#define CTR_STRIDE 32   // one 128-byte line per counter

__device__ __forceinline__ uint32_t xcd_remap(uint32_t b, uint32_t nwg)
{
	const uint32_t q = nwg / 8, r = nwg % 8, x = b % 8;
	return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + b / 8;
}

__global__ __launch_bounds__(WG) __attribute__((amdgpu_waves_per_eu(8))) void k_grid(mosrx_kparams kp)
{
	classify_tile_stream<S, 0>(kp, blockIdx.x);
}

__global__ __launch_bounds__(WG) __attribute__((amdgpu_waves_per_eu(8))) void k_grid_xcd(mosrx_kparams kp)
{
	classify_tile_stream<S, 0>(kp, xcd_remap(blockIdx.x, gridDim.x));
}

__global__ __launch_bounds__(WG) __attribute__((amdgpu_waves_per_eu(8)))
void k_grid_order(mosrx_kparams kp, const uint32_t *order)
{
	classify_tile_stream<S, 0>(kp, order[blockIdx.x]);
}

// every workgroup leaves when its XCD's tiles are taken (no stealing): the
// exit condition every wave reaches
__global__ __launch_bounds__(WG) __attribute__((amdgpu_waves_per_eu(8)))
void k_persist_xcd(mosrx_kparams kp, uint32_t *ctr, const uint32_t *order, uint32_t ntiles)
{
	__shared__ uint32_t s_next;
	const uint32_t x = __builtin_amdgcn_s_getreg(20 | (31 << 11)) & 7u;   // HW_REG_XCC_ID
	uint32_t *c = ctr + CTR_STRIDE * x;
	if (threadIdx.x == 0)
		s_next = atomicAdd(c, 1u);
	__syncthreads();
	uint32_t k = s_next;
	for (;;) {
		const uint32_t t = 8u * k + x;
		if (t >= ntiles)
			break;                             // uniform: k is the workgroup's
		__syncthreads();                       // everyone has read s_next
		if (threadIdx.x == 0)
			s_next = atomicAdd(c, 1u);         // the next index, in flight during this tile
		classify_tile_stream<S, 0>(kp, order ? order[t] : t);
		__syncthreads();
		k = s_next;
	}
}

enum { F_GRID, F_XCD, F_HEAVY, F_PX, F_PXH, F_N };
static const char *names[F_N] = {"grid (library)", "grid xcd remap", "grid heaviest-first", "persist xcd",
                                 "persist xcd heaviest"};

static void launch(int f, const mosrx_kparams &kp, uint32_t *ctr, const uint32_t *order, uint32_t ntiles, int grid,
                   hipStream_t st)
{
	switch (f) {
	case F_GRID: hipLaunchKernelGGL(k_grid, dim3(ntiles), dim3(WG), 0, st, kp); break;
	case F_XCD: hipLaunchKernelGGL(k_grid_xcd, dim3(ntiles), dim3(WG), 0, st, kp); break;
	case F_HEAVY: hipLaunchKernelGGL(k_grid_order, dim3(ntiles), dim3(WG), 0, st, kp, order); break;
	case F_PX: hipLaunchKernelGGL(k_persist_xcd, dim3(grid), dim3(WG), 0, st, kp, ctr, (const uint32_t *)nullptr,
	                              ntiles); break;
	default: hipLaunchKernelGGL(k_persist_xcd, dim3(grid), dim3(WG), 0, st, kp, ctr, order, ntiles); break;
	}
}

int main(int argc, char **argv)
{
	const int kind = argc > 1 ? atoi(argv[1]) : MOSRX_TRACE_IMIX;
	const uint32_t n = argc > 2 ? (uint32_t)atoi(argv[2]) : 262144;
	const int nb = 12;
	mosrx_trace t;
	if (mosrx_trace_gen(kind, n, 1000000, 0, &t)) {
		printf("trace_gen failed\n");
		return 1;
	}
	const uint32_t ntiles = (n + 63) / 64;
	std::vector<uint32_t> span(ntiles), ord(ntiles);
	for (uint32_t k = 0; k < ntiles; k++) {
		const uint32_t a = k * 64, b = std::min(n, a + 64) - 1;
		span[k] = t.off[b] + t.len[b] - t.off[a];
	}
	std::iota(ord.begin(), ord.end(), 0u);
	std::stable_sort(ord.begin(), ord.end(), [&](uint32_t x, uint32_t y) { return span[x] > span[y]; });
	mosrx_params p;
	mosrx_params_default(&p);
	uint32_t tab[MOSRX_TAB_ALLOC_WORDS];
	memset(tab, 0, sizeof(tab));
	mosrx_rss_tables(p.rss_key, p.rss_key_len, tab);
	uint32_t *tables, *order, *ctrs;
	CHK(hipMalloc((void **)&tables, sizeof(tab)));
	CHK(hipMemcpy(tables, tab, sizeof(tab), hipMemcpyHostToDevice));
	CHK(hipMalloc((void **)&order, ntiles * 4));
	CHK(hipMemcpy(order, ord.data(), ntiles * 4, hipMemcpyHostToDevice));
	const int maxl = 256;                      // launches per timing run, each its own 8 counters
	CHK(hipMalloc((void **)&ctrs, (size_t)maxl * 8 * CTR_STRIDE * 4));
	mosrx_kparams kps[nb];
	for (int i = 0; i < nb; i++) {
		uint8_t *f; uint32_t *o; uint16_t *l; mosrx_result *r;
		CHK(hipMalloc((void **)&f, t.frames_bytes + 64));
		CHK(hipMemcpy(f, t.frames, t.frames_bytes + 64, hipMemcpyHostToDevice));
		CHK(hipMalloc((void **)&o, n * 4));
		CHK(hipMemcpy(o, t.off, n * 4, hipMemcpyHostToDevice));
		CHK(hipMalloc((void **)&l, n * 2));
		CHK(hipMemcpy(l, t.len, n * 2, hipMemcpyHostToDevice));
		CHK(hipMalloc((void **)&r, n * 16));
		kps[i] = (mosrx_kparams){f, o, l, r, tables, NULL, NULL, NULL, NULL, (uint32_t)t.frames_bytes, n,
		                         MOSRX_KF_VERIFY};
	}
	int ncu = 0, occ = 0;
	CHK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
	CHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k_persist_xcd, WG, 0));
	const int grid = std::min<int>(ncu * occ, (int)ntiles);
	const double bytes = (double)t.caplen_sum + 22.0 * n;
	printf("trace kind %d n %u tiles %u: %.2f MB algorithmic; %d CUs, %d resident blocks/CU, persistent grid %d\n",
	       kind, n, ntiles, bytes / 1e6, ncu, occ, grid);
	std::vector<mosrx_result> want(n), got(n);
	hipStream_t st = 0;
	CHK(hipMemset(ctrs, 0, (size_t)maxl * 8 * CTR_STRIDE * 4));
	launch(F_GRID, kps[0], ctrs, order, ntiles, grid, st);
	CHK(hipDeviceSynchronize());
	CHK(hipMemcpy(want.data(), kps[0].out, n * 16, hipMemcpyDeviceToHost));
	hipEvent_t a, b;
	CHK(hipEventCreate(&a));
	CHK(hipEventCreate(&b));
	std::vector<hipEvent_t> e0(maxl), e1(maxl);
	for (int i = 0; i < maxl; i++) {
		CHK(hipEventCreate(&e0[i]));
		CHK(hipEventCreate(&e1[i]));
	}
	for (int rep = 0; rep < 3; rep++) {
		for (int f = 0; f < F_N; f++) {
			CHK(hipMemset(kps[1].out, 0xEE, n * 16));
			CHK(hipMemset(ctrs, 0, (size_t)maxl * 8 * CTR_STRIDE * 4));
			CHK(hipDeviceSynchronize());
			launch(f, kps[1], ctrs, order, ntiles, grid, st);
			CHK(hipDeviceSynchronize());
			CHK(hipMemcpy(got.data(), kps[1].out, n * 16, hipMemcpyDeviceToHost));
			if (memcmp(got.data(), want.data(), (size_t)n * 16)) {
				printf("%s: RECORDS DIFFER\n", names[f]);
				return 2;
			}
			const int iters = maxl;
			CHK(hipMemset(ctrs, 0, (size_t)maxl * 8 * CTR_STRIDE * 4));
			CHK(hipDeviceSynchronize());
			CHK(hipEventRecord(a, st));
			for (int i = 0; i < iters; i++)
				launch(f, kps[i % nb], ctrs + (size_t)i * 8 * CTR_STRIDE, order, ntiles, grid, st);
			CHK(hipEventRecord(b, st));
			CHK(hipEventSynchronize(b));
			float ms;
			CHK(hipEventElapsedTime(&ms, a, b));
			// dispatch-stamped: each launch's own duration (the library's launch_us)
			CHK(hipMemset(ctrs, 0, (size_t)maxl * 8 * CTR_STRIDE * 4));
			CHK(hipDeviceSynchronize());
			for (int i = 0; i < iters; i++) {
				uint32_t *c = ctrs + (size_t)i * 8 * CTR_STRIDE;
				const mosrx_kparams &kp = kps[i % nb];
				switch (f) {
				case F_GRID: hipExtLaunchKernelGGL(k_grid, dim3(ntiles), dim3(WG), 0, st, e0[i], e1[i], 0, kp); break;
				case F_XCD: hipExtLaunchKernelGGL(k_grid_xcd, dim3(ntiles), dim3(WG), 0, st, e0[i], e1[i], 0, kp); break;
				case F_HEAVY: hipExtLaunchKernelGGL(k_grid_order, dim3(ntiles), dim3(WG), 0, st, e0[i], e1[i], 0, kp,
				                                    (const uint32_t *)order); break;
				case F_PX: hipExtLaunchKernelGGL(k_persist_xcd, dim3(grid), dim3(WG), 0, st, e0[i], e1[i], 0, kp, c,
				                                 (const uint32_t *)nullptr, ntiles); break;
				default: hipExtLaunchKernelGGL(k_persist_xcd, dim3(grid), dim3(WG), 0, st, e0[i], e1[i], 0, kp, c,
				                               (const uint32_t *)order, ntiles); break;
				}
			}
			CHK(hipDeviceSynchronize());
			std::vector<float> d(iters);
			for (int i = 0; i < iters; i++)
				CHK(hipEventElapsedTime(&d[i], e0[i], e1[i]));
			std::sort(d.begin(), d.end());
			const double med = d[iters / 2] * 1e-3;
			printf("rep %d %-22s stamped median %7.2f us (%.3f of 8 TB/s) | back-to-back %7.2f us\n", rep, names[f],
			       med * 1e6, bytes / med / 8e12, ms * 1e3 / iters);
		}
	}
	return 0;
}
