// probe_shape.hip — where the 1500 B classify kernel's time goes (diagnostic only).
// Read-only kernels over the same 100.66 MB layout as BASELINE config #3
// (65536 frames of 1514 B at 16 B + 2 strides), timed back-to-back and one launch
// at a time, so the access structure of the LARGE shape can be compared with a
// plain slab stream without any header work.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
#define CHK(x) do { if ((x) != hipSuccess) { printf("HIP error %s line %d\n", #x, __LINE__); return 1; } } while (0)

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void *p, uint32_t n)
{
	return __builtin_amdgcn_make_buffer_rsrc((void *)p, (short)0, (int)n, 0x00020000);
}
__device__ __forceinline__ u32x4 ld(__amdgpu_buffer_rsrc_t r, uint32_t c) { return __builtin_amdgcn_raw_buffer_load_b128(r, c, 0, 2); }

// slab: each workgroup of WG threads streams bytes [blk*per, (blk+1)*per), U 16 B loads in flight per lane
template <int WG, int U>
__global__ __launch_bounds__(WG) void k_slab(const uint8_t *p, uint32_t nbytes, const uint32_t *off, uint32_t *sink)
{
	const __amdgpu_buffer_rsrc_t r = rsrc(p, nbytes);
	const uint32_t per = ((nbytes / gridDim.x) + 15u) & ~15u;
	const uint32_t lo = blockIdx.x * per, hi = min(nbytes, lo + per);
	uint32_t acc = 0;
	for (uint32_t c = lo + 16u * threadIdx.x; c < hi; c += 16u * WG * U) {
		u32x4 v[U];
#pragma unroll
		for (int u = 0; u < U; u++) {
			const uint32_t a = c + 16u * WG * u;
			v[u] = ld(r, a < hi ? a : nbytes);
		}
#pragma unroll
		for (int u = 0; u < U; u++)
			acc += v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
	}
	if (acc == 0x9E3779B9u)
		sink[0] = acc;
}

// tails: LARGE's structure without compute.  64 frames per workgroup; wave 0
// idles (stands for the header wave), waves 1..4 each take 4 consecutive frames per
// group, 2 x 1 KiB loads per frame from its split, two groups in flight.  DESC:
// frame offsets come from the descriptor array (one dependent load first).
template <bool DESC>
__global__ __launch_bounds__(320) void k_tails(const uint8_t *p, uint32_t nbytes, const uint32_t *off, uint32_t *sink)
{
	const __amdgpu_buffer_rsrc_t r = rsrc(p, nbytes);
	const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63u;
	__syncthreads();
	if (wave == 0)
		return;
	const uint32_t q = wave - 1;
	uint32_t o_l = DESC ? off[blockIdx.x * 64u + lane] : (blockIdx.x * 64u + lane) * 1520u + 2u;
	uint32_t acc = 0;
	u32x4 v[2][4][2];
#pragma unroll
	for (int g = 0; g < 4; g++) {
		const int bsel = g & 1;
#pragma unroll
		for (int u = 0; u < 4; u++) {
			const uint32_t f = 16u * g + 4u * q + u;
			const uint32_t o = __builtin_amdgcn_readlane(o_l, f);
			const uint32_t lo = (o + 94u) & ~15u, hi = o + 1514u;
#pragma unroll
			for (int k = 0; k < 2; k++) {
				const uint32_t c = lo + 1024u * k + 16u * lane;
				if (g >= 2) {
					const u32x4 w = v[bsel][u][k];
					acc += w.x ^ w.y ^ w.z ^ w.w;
				}
				v[bsel][u][k] = ld(r, c < hi ? c : nbytes);
			}
		}
	}
#pragma unroll
	for (int b = 0; b < 2; b++)
#pragma unroll
		for (int u = 0; u < 4; u++)
#pragma unroll
			for (int k = 0; k < 2; k++)
				acc += v[b][u][k].x ^ v[b][u][k].w;
	if (acc == 0x9E3779B9u)
		sink[0] = acc;
}

typedef void (*kfn)(const uint8_t *, uint32_t, const uint32_t *, uint32_t *);

static int run(const char *name, kfn k, int grid, int wg, void **bufs, uint32_t **offs, int nbuf, uint32_t bytes,
               uint32_t *sink)
{
	hipEvent_t a, b;
	CHK(hipEventCreate(&a));
	CHK(hipEventCreate(&b));
	for (int i = 0; i < nbuf; i++)
		hipLaunchKernelGGL(k, dim3(grid), dim3(wg), 0, 0, (const uint8_t *)bufs[i], bytes, offs[i], sink);
	const int iters = 60;
	CHK(hipEventRecord(a, 0));
	for (int i = 0; i < iters; i++)
		hipLaunchKernelGGL(k, dim3(grid), dim3(wg), 0, 0, (const uint8_t *)bufs[i % nbuf], bytes, offs[i % nbuf], sink);
	CHK(hipEventRecord(b, 0));
	CHK(hipEventSynchronize(b));
	float ms, one = 0;
	CHK(hipEventElapsedTime(&ms, a, b));
	for (int i = 0; i < iters; i++) {
		float t;
		CHK(hipEventRecord(a, 0));
		hipLaunchKernelGGL(k, dim3(grid), dim3(wg), 0, 0, (const uint8_t *)bufs[i % nbuf], bytes, offs[i % nbuf], sink);
		CHK(hipEventRecord(b, 0));
		CHK(hipEventSynchronize(b));
		CHK(hipEventElapsedTime(&t, a, b));
		one += t;
	}
	printf("%-34s grid %5d x %3d: back-to-back %6.2f us (%6.0f GB/s) | single %6.2f us (%6.0f GB/s)\n", name, grid,
	       wg, ms * 1e3 / iters, (double)bytes * iters / (ms * 1e-3) / 1e9, one * 1e3 / iters,
	       (double)bytes * iters / (one * 1e-3) / 1e9);
	return 0;
}

int main()
{
	const uint32_t n = 65536, stride = 1520;
	const uint32_t bytes = n * stride;   // 99.6 MB of frames (+ descriptors are extra)
	const int nbuf = 6;
	void *bufs[nbuf];
	uint32_t *offs[nbuf], *sink;
	uint32_t *h = (uint32_t *)malloc(n * 4);
	for (uint32_t i = 0; i < n; i++)
		h[i] = i * stride + 2;
	for (int i = 0; i < nbuf; i++) {
		CHK(hipMalloc(&bufs[i], bytes));
		CHK(hipMemset(bufs[i], i + 1, bytes));
		CHK(hipMalloc((void **)&offs[i], n * 4));
		CHK(hipMemcpy(offs[i], h, n * 4, hipMemcpyHostToDevice));
	}
	CHK(hipMalloc(&sink, 4));
	run("slab 256 U=4", k_slab<256, 4>, 2048, 256, bufs, offs, nbuf, bytes, sink);
	run("slab 256 U=4", k_slab<256, 4>, 1024, 256, bufs, offs, nbuf, bytes, sink);
	run("slab 256 U=8", k_slab<256, 8>, 1024, 256, bufs, offs, nbuf, bytes, sink);
	run("slab 256 U=8", k_slab<256, 8>, 2048, 256, bufs, offs, nbuf, bytes, sink);
	run("slab 512 U=4", k_slab<512, 4>, 1024, 512, bufs, offs, nbuf, bytes, sink);
	run("slab 256 U=2", k_slab<256, 2>, 4096, 256, bufs, offs, nbuf, bytes, sink);
	run("tails (LARGE structure)", k_tails<false>, 1024, 320, bufs, offs, nbuf, bytes, sink);
	run("tails + descriptor load", k_tails<true>, 1024, 320, bufs, offs, nbuf, bytes, sink);
	return 0;
}
