// probe_bw.hip — streaming-read ceiling of one MI355X for several access shapes.
// Diagnostic only (roofline calibration for DESIGN.md); not part of the product.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

#define CHK(x) do { if ((x) != hipSuccess) { printf("HIP error %s line %d\n", #x, __LINE__); return 1; } } while (0)

// A: grid-stride, U loads in flight per lane
template <int U>
__global__ __launch_bounds__(256) void rd_stride(const u32x4 *p, uint64_t n16, uint32_t *sink)
{
	uint32_t acc = 0;
	const uint64_t stride = (uint64_t)gridDim.x * 256u;
	uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x;
	for (; i + (U - 1) * stride < n16; i += U * stride) {
		u32x4 v[U];
#pragma unroll
		for (int u = 0; u < U; u++)
			v[u] = p[i + u * stride];
#pragma unroll
		for (int u = 0; u < U; u++)
			acc += v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
	}
	for (; i < n16; i += stride)
		acc += p[i].x;
	if (acc == 0x9E3779B9u)
		sink[0] = acc;
}

// B: each workgroup streams one contiguous slab (chunk = n16 / gridDim), U in flight
template <int U, bool NT>
__global__ __launch_bounds__(256) void rd_slab(const u32x4 *p, uint64_t n16, uint32_t *sink)
{
	uint32_t acc = 0;
	const uint64_t per = (n16 + gridDim.x - 1) / gridDim.x;
	const uint64_t lo = (uint64_t)blockIdx.x * per, hi = min(n16, lo + per);
	for (uint64_t i = lo + threadIdx.x; i < hi; i += 256u * U) {
		u32x4 v[U];
#pragma unroll
		for (int u = 0; u < U; u++) {
			const uint64_t j = i + 256u * u;
			if (NT)
				v[u] = j < hi ? __builtin_nontemporal_load(p + j) : (u32x4){0, 0, 0, 0};
			else
				v[u] = j < hi ? p[j] : (u32x4){0, 0, 0, 0};
		}
#pragma unroll
		for (int u = 0; u < U; u++)
			acc += v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
	}
	if (acc == 0x9E3779B9u)
		sink[0] = acc;
}

// C: each WAVE streams its own contiguous slab, 1 KiB per load, U in flight
// (the classify streamers' access shape), buffer loads, AUX cache policy
template <int U, int AUX>
__global__ __launch_bounds__(256) void rd_wave(const u32x4 *p, uint64_t n16, uint32_t *sink)
{
	uint32_t acc = 0;
	const uint32_t lane = threadIdx.x & 63u;
	const uint64_t nw = (uint64_t)gridDim.x * 4u, w = (uint64_t)blockIdx.x * 4u + (threadIdx.x >> 6);
	const uint64_t per = ((n16 + nw - 1) / nw + 63u) & ~(uint64_t)63u;
	const uint64_t lo = w * per, hi = min(n16, lo + per);
	const uint32_t nbytes = lo < hi ? (uint32_t)((hi - lo) * 16u) : 0u;
	// records = the slab: offsets past it (the 0xFFFFFFF0 filler) read 0 without a memory access
	const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void *)(p + (lo < n16 ? lo : 0)), (short)0, (int)nbytes, 0x00020000);
	for (uint32_t b = 0; b < nbytes; b += 1024u * U) {
		u32x4 v[U];
#pragma unroll
		for (int u = 0; u < U; u++)
			v[u] = __builtin_amdgcn_raw_buffer_load_b128(rs, b + 1024u * u + 16u * lane < nbytes ? b + 1024u * u + 16u * lane : 0xFFFFFFF0u, 0, AUX);
#pragma unroll
		for (int u = 0; u < U; u++)
			acc += v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
	}
	if (acc == 0x9E3779B9u)
		sink[0] = acc;
}

typedef void (*kfn)(const u32x4 *, uint64_t, uint32_t *);

static int run(const char *name, kfn k, int grid, void **bufs, int nbuf, uint64_t bytes, uint32_t *sink)
{
	hipEvent_t a, b;
	CHK(hipEventCreate(&a));
	CHK(hipEventCreate(&b));
	for (int i = 0; i < nbuf; i++)
		hipLaunchKernelGGL(k, dim3(grid), dim3(256), 0, 0, (const u32x4 *)bufs[i], bytes / 16, sink);
	const int iters = 60;
	CHK(hipEventRecord(a, 0));
	for (int i = 0; i < iters; i++)
		hipLaunchKernelGGL(k, dim3(grid), dim3(256), 0, 0, (const u32x4 *)bufs[i % nbuf], bytes / 16, sink);
	CHK(hipEventRecord(b, 0));
	CHK(hipEventSynchronize(b));
	float ms;
	CHK(hipEventElapsedTime(&ms, a, b));
	printf("%-28s grid %5d: %7.1f GB/s  (%.1f us/pass)\n", name, grid, (double)bytes * iters / (ms * 1e-3) / 1e9,
	       ms * 1e3 / iters);
	return 0;
}

int main(int argc, char **argv)
{
	const uint64_t bytes = (argc > 1 ? (uint64_t)atoi(argv[1]) : 512ull) << 20;
	const int nbuf = argc > 2 ? atoi(argv[2]) : 3;
	void *bufs[16];
	uint32_t *sink;
	for (int i = 0; i < nbuf; i++) {
		CHK(hipMalloc(&bufs[i], bytes));
		CHK(hipMemset(bufs[i], i + 1, bytes));
	}
	CHK(hipMalloc(&sink, 4));
	for (int rep = 0; rep < 2; rep++) {
		run("slab U=4 nt (library probe)", rd_slab<4, true>, 2048, bufs, nbuf, bytes, sink);
		for (int g : {4096, 5461, 8192, 16384, 32768}) {
			run("slab U=4 nt", rd_slab<4, true>, g, bufs, nbuf, bytes, sink);
			run("slab U=8 nt", rd_slab<8, true>, g, bufs, nbuf, bytes, sink);
		}
		run("slab U=2 nt", rd_slab<2, true>, 8192, bufs, nbuf, bytes, sink);
		run("wave U=4 nt", rd_wave<4, 2>, 8192, bufs, nbuf, bytes, sink);
		run("wave U=4 nt", rd_wave<4, 2>, 16384, bufs, nbuf, bytes, sink);
	}
	return 0;
}
