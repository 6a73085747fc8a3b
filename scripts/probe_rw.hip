// probe_rw.hip — streaming read+write rate of one MI355X at the classify rows'
// read:write mixes.  Diagnostic only (roofline calibration for DESIGN.md §5);
// not part of the product.
//
// Each workgroup streams one contiguous 96 KiB read slab (non-temporal 16-byte
// loads, 8 per lane in flight) and, for every R loads, writes one 16-byte
// record per lane to its own slab of the output with a non-temporal store — the shape of
// the SMALL tile (lane per frame: a 64-byte frame + 6 descriptor bytes in, a
// 16-byte record out, about 4:1) and of the stream tile (records ≈ 4 % of an
// IMIX tile's bytes, 24:1).  R = 0 writes nothing (the read probe).
//   usage: probe_rw [MiB read per launch, default 648] [buffers, default 2]
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

#define CHK(x) do { if ((x) != hipSuccess) { printf("HIP error %s line %d\n", #x, __LINE__); return 1; } } while (0)

// 96 KiB slabs: three rounds of 8 loads per lane; R >= 8 writes one record
// every R/8 rounds, R < 8 writes 8/R per round (each the XOR of R loads).
#define SLAB16 (3u * 8u * 256u)
template <int R>
__global__ __launch_bounds__(256) void rw_slab(const u32x4 *p, uint64_t n16, u32x4 *out, uint32_t *sink)
{
	constexpr int U = 8, RPI = R >= 8 ? 1 : (R > 0 ? 8 / R : 0), EVERY = R >= 8 ? R / 8 : 1;
	uint32_t acc = 0;
	const uint64_t lo = (uint64_t)blockIdx.x * SLAB16, hi = min(n16, lo + SLAB16);
	uint64_t w = R > 0 ? lo / R : 0;
	int it = 0;
	for (uint64_t i = lo + threadIdx.x; i < hi; i += 256u * U, it++) {
		u32x4 v[U];
#pragma unroll
		for (int u = 0; u < U; u++) {
			const uint64_t j = i + 256u * u;
			v[u] = j < hi ? __builtin_nontemporal_load(p + j) : (u32x4){0, 0, 0, 0};
		}
		if constexpr (R > 0) {
			if (it % EVERY == EVERY - 1) {
#pragma unroll
				for (int q = 0; q < RPI; q++) {
					u32x4 r = {0, 0, 0, 0};
#pragma unroll
					for (int u = q * (U / RPI); u < (q + 1) * (U / RPI); u++)
						r ^= v[u];
					__builtin_nontemporal_store(r, out + w + threadIdx.x);
					w += 256u;
				}
			}
		} else {
#pragma unroll
			for (int u = 0; u < U; u++)
				acc += v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
		}
	}
	if (acc == 0x9E3779B9u)
		sink[0] = acc;
}

typedef void (*kfn)(const u32x4 *, uint64_t, u32x4 *, uint32_t *);

static int run(const char *name, kfn k, int r, int grid, void **bufs, u32x4 **outs, int nbuf, uint64_t bytes,
               uint32_t *sink)
{
	hipEvent_t a, b;
	CHK(hipEventCreate(&a));
	CHK(hipEventCreate(&b));
	for (int i = 0; i < nbuf; i++)
		hipLaunchKernelGGL(k, dim3(grid), dim3(256), 0, 0, (const u32x4 *)bufs[i], bytes / 16, outs[i], sink);
	const int iters = 40;
	CHK(hipEventRecord(a, 0));
	for (int i = 0; i < iters; i++)
		hipLaunchKernelGGL(k, dim3(grid), dim3(256), 0, 0, (const u32x4 *)bufs[i % nbuf], bytes / 16, outs[i % nbuf],
		                   sink);
	CHK(hipEventRecord(b, 0));
	CHK(hipEventSynchronize(b));
	float ms;
	CHK(hipEventElapsedTime(&ms, a, b));
	const double wr = r > 0 ? (double)bytes / r : 0.0;
	const double us = ms * 1e3 / iters;
	printf("%-14s grid %5d: read %7.1f GB/s + write %6.1f GB/s = %7.1f GB/s  (%.1f us/launch, write %.1f %%)\n",
	       name, grid, bytes / (us * 1e3), wr / (us * 1e3), (bytes + wr) / (us * 1e3), us, 100.0 * wr / (bytes + wr));
	return 0;
}

int main(int argc, char **argv)
{
	const uint64_t bytes = (argc > 1 ? (uint64_t)atoi(argv[1]) : 648ull) << 20;
	const int nbuf = argc > 2 ? atoi(argv[2]) : 2;
	void *bufs[8];
	u32x4 *outs[8];
	uint32_t *sink;
	if (nbuf < 1 || nbuf > 8)
		return 1;
	for (int i = 0; i < nbuf; i++) {
		CHK(hipMalloc(&bufs[i], bytes));
		CHK(hipMemset(bufs[i], i + 1, bytes));
		CHK(hipMalloc((void **)&outs[i], bytes / 2 + (1u << 20)));
	}
	CHK(hipMalloc(&sink, 4));
	const int grid = (int)(bytes / (16u * SLAB16));
	for (int rep = 0; rep < 3; rep++) {
		run("read only", rw_slab<0>, 0, grid, bufs, outs, nbuf, bytes, sink);
		run("read:write 24", rw_slab<24>, 24, grid, bufs, outs, nbuf, bytes, sink);
		run("read:write 8", rw_slab<8>, 8, grid, bufs, outs, nbuf, bytes, sink);
		run("read:write 4", rw_slab<4>, 4, grid, bufs, outs, nbuf, bytes, sink);
		run("read:write 2", rw_slab<2>, 2, grid, bufs, outs, nbuf, bytes, sink);
	}
	return 0;
}
