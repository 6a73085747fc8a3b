// probe_persist.hip — persistent-grid forms of the stream tile (diagnostic only).
//
// a single-batch launch pays ~5 us of ramp and drain (DESIGN
// §4.4).  Here the library's stream tile (classify_tile_stream, unchanged) runs
//   grid    one workgroup per tile (the library),
//   persist a grid of resident workgroups pulling tiles from an atomic
//           counter (one counter per launch, zeroed once up front),
//   sorted  the same, tiles taken in descending order of their span bytes
//           (an order array made on the host from the descriptors),
// with 3 / 5 / 7 streamer waves per tile.  Every form is checked against the
// library kernel's records before it is timed.
#include "../mos-networking-stack_amd/csrc/mosrx_kernels.hip"
#include "../include/mosrx_trace.h"
#include <algorithm>
#include <numeric>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <vector>

#define CHK(x) do { if ((x) != hipSuccess) { printf("HIP error %s line %d\n", #x, __LINE__); return 1; } } while (0)

template <int S>
__global__ __launch_bounds__(64 * (1 + S)) __attribute__((amdgpu_waves_per_eu(8)))
void k_grid(mosrx_kparams kp)
{
	classify_tile_stream<S, 2>(kp, blockIdx.x);
}

template <int S>
__global__ __launch_bounds__(64 * (1 + S)) __attribute__((amdgpu_waves_per_eu(8)))
void k_persist(mosrx_kparams kp, uint32_t *ctr, const uint32_t *order, uint32_t ntiles)
{
	__shared__ uint32_t s_tile;
	for (;;) {
		__syncthreads();                      // the previous tile's LDS is no longer read
		if (threadIdx.x == 0)
			s_tile = atomicAdd(ctr, 1u);
		__syncthreads();
		const uint32_t k = s_tile;
		if (k >= ntiles)
			break;                            // every wave of the workgroup leaves together
		classify_tile_stream<S, 2>(kp, order ? order[k] : k);
	}
}

struct Form {
	const char *name;
	int s, persist, sorted;
};

template <int S>
static void launch(const Form &f, const mosrx_kparams &kp, uint32_t *ctr, const uint32_t *order, uint32_t ntiles,
                   int grid, hipStream_t st)
{
	if (!f.persist)
		hipLaunchKernelGGL((k_grid<S>), dim3(ntiles), dim3(64 * (1 + S)), 0, st, kp);
	else
		hipLaunchKernelGGL((k_persist<S>), dim3(grid), dim3(64 * (1 + S)), 0, st, kp, ctr, f.sorted ? order : nullptr,
		                   ntiles);
}

static void launch_any(const Form &f, const mosrx_kparams &kp, uint32_t *ctr, const uint32_t *order, uint32_t ntiles,
                       const int *grids, hipStream_t st)
{
	if (f.s == 3) launch<3>(f, kp, ctr, order, ntiles, grids[0], st);
	else if (f.s == 5) launch<5>(f, kp, ctr, order, ntiles, grids[1], st);
	else launch<7>(f, kp, ctr, order, ntiles, grids[2], st);
}

int main(int argc, char **argv)
{
	const int kind = argc > 1 ? atoi(argv[1]) : MOSRX_TRACE_M1500;
	const uint32_t n = argc > 2 ? (uint32_t)atoi(argv[2]) : 65536;
	const int nb = 12;                        // resident batch copies cycled (> 1.2 GB for the big traces)
	mosrx_trace t;
	if (mosrx_trace_gen(kind, n, 1000000, 0, &t)) {
		printf("trace_gen failed\n");
		return 1;
	}
	const uint32_t ntiles = (n + 63) / 64;
	// tile spans and the descending-span order
	std::vector<uint32_t> span(ntiles), ord(ntiles);
	for (uint32_t k = 0; k < ntiles; k++) {
		const uint32_t a = k * 64, b = std::min(n, a + 64) - 1;
		span[k] = t.off[b] + t.len[b] - t.off[a];
	}
	std::iota(ord.begin(), ord.end(), 0u);
	std::stable_sort(ord.begin(), ord.end(), [&](uint32_t x, uint32_t y) { return span[x] > span[y]; });

	// tables: the library's default key / queue map
	mosrx_params p;
	mosrx_params_default(&p);
	uint32_t tab[MOSRX_TAB_ALLOC_WORDS];
	memset(tab, 0, sizeof(tab));
	mosrx_rss_tables(p.rss_key, p.rss_key_len, tab);
	for (uint32_t x = 0; x < 512; x++)
		((uint8_t *)(tab + MOSRX_TAB_RSS_WORDS))[x] = 0;   // num_queues 1
	uint32_t *tables, *order, *ctrs;
	CHK(hipMalloc((void **)&tables, sizeof(tab)));
	CHK(hipMemcpy(tables, tab, sizeof(tab), hipMemcpyHostToDevice));
	CHK(hipMalloc((void **)&order, ntiles * 4));
	CHK(hipMemcpy(order, ord.data(), ntiles * 4, hipMemcpyHostToDevice));
	const int maxl = 4096;
	CHK(hipMalloc((void **)&ctrs, maxl * 4));

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
	int ncu = 0, occ[3] = {0, 0, 0}, grids[3];
	CHK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
	CHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ[0], k_persist<3>, 256, 0));
	CHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ[1], k_persist<5>, 384, 0));
	CHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ[2], k_persist<7>, 512, 0));
	for (int i = 0; i < 3; i++)
		grids[i] = std::min<int>(ncu * occ[i], (int)ntiles);
	const double bytes = (double)t.caplen_sum + 22.0 * n;
	printf("trace kind %d n %u tiles %u: %.2f MB algorithmic; %d CUs, resident blocks/CU S3 %d S5 %d S7 %d\n", kind, n,
	       ntiles, bytes / 1e6, ncu, occ[0], occ[1], occ[2]);

	const Form forms[] = {{"grid S3 (library)", 3, 0, 0}, {"persist S3", 3, 1, 0}, {"persist S3 sorted", 3, 1, 1},
	                      {"grid S5", 5, 0, 0},           {"persist S5", 5, 1, 0}, {"grid S7", 7, 0, 0},
	                      {"persist S7", 7, 1, 0},        {"persist S7 sorted", 7, 1, 1}};
	// reference records: the library form on batch 0
	std::vector<mosrx_result> want(n), got(n);
	hipStream_t st = 0;
	CHK(hipMemset(ctrs, 0, maxl * 4));
	launch_any(forms[0], kps[0], ctrs, order, ntiles, grids, st);
	CHK(hipDeviceSynchronize());
	CHK(hipMemcpy(want.data(), kps[0].out, n * 16, hipMemcpyDeviceToHost));
	hipEvent_t a, b;
	CHK(hipEventCreate(&a));
	CHK(hipEventCreate(&b));
	for (int rep = 0; rep < 3; rep++) {
		for (const Form &f : forms) {
			// parity first
			CHK(hipMemset(kps[1].out, 0xEE, n * 16));
			CHK(hipMemset(ctrs, 0, maxl * 4));
			launch_any(f, kps[1], ctrs, order, ntiles, grids, st);
			CHK(hipDeviceSynchronize());
			CHK(hipMemcpy(got.data(), kps[1].out, n * 16, hipMemcpyDeviceToHost));
			if (memcmp(got.data(), want.data(), (size_t)n * 16)) {
				printf("%s: RECORDS DIFFER\n", f.name);
				return 2;
			}
			// back-to-back and single launches (counter k for launch k)
			const int iters = 200;
			CHK(hipMemset(ctrs, 0, maxl * 4));
			CHK(hipDeviceSynchronize());
			CHK(hipEventRecord(a, st));
			for (int i = 0; i < iters; i++)
				launch_any(f, kps[i % nb], ctrs + i, order, ntiles, grids, st);
			CHK(hipEventRecord(b, st));
			CHK(hipEventSynchronize(b));
			float ms, one = 0;
			CHK(hipEventElapsedTime(&ms, a, b));
			CHK(hipMemset(ctrs, 0, maxl * 4));
			CHK(hipDeviceSynchronize());
			for (int i = 0; i < iters; i++) {
				float tt;
				CHK(hipEventRecord(a, st));
				launch_any(f, kps[i % nb], ctrs + i, order, ntiles, grids, st);
				CHK(hipEventRecord(b, st));
				CHK(hipEventSynchronize(b));
				CHK(hipEventElapsedTime(&tt, a, b));
				one += tt;
			}
			printf("rep %d %-22s back-to-back %7.2f us (%5.0f GB/s, %.3f of 8 TB/s) | single %7.2f us\n", rep, f.name,
			       ms * 1e3 / iters, bytes / (ms * 1e-3 / iters) / 1e9, bytes / (ms * 1e-3 / iters) / 8e12,
			       one * 1e3 / iters);
		}
	}
	return 0;
}
