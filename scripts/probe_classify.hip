// probe_classify.hip — time shares of the LARGE and stream classify tiles (diagnostic only).
// Builds the library's kernel source with the DBG knob of classify_tile_large
// (1: no header parse/records, 2: no header window loads, 4: no streamer sums)
// and times each build on the BASELINE config #3 trace, back-to-back and one
// launch at a time.  Results are meaningless for DBG != 0; only time counts.
#include "../mos-networking-stack_amd/csrc/mosrx_kernels.hip"
#include "probe_large.h"
#include "probe_decoupled.h"
#include "../include/mosrx_trace.h"
#include <stdio.h>
#include <stdlib.h>

#define CHK(x) do { if ((x) != hipSuccess) { printf("HIP error %s line %d\n", #x, __LINE__); return 1; } } while (0)

template <int DBG, int MINB = 1>
__global__ __launch_bounds__(320) __attribute__((amdgpu_waves_per_eu(MINB > 1 ? 8 : 1))) void k_dbg(mosrx_kparams kp)
{
	classify_tile_large<1, 4, 2, DBG>(kp, blockIdx.x);
}

template <int S, int DBG, int W = 6, int U = 8, uint32_t T = 64>
__global__ __launch_bounds__(64 * (1 + S)) __attribute__((amdgpu_waves_per_eu(W))) void k_sdbg(mosrx_kparams kp)
{
	classify_tile_stream<S, 2, DBG, U, T>(kp, blockIdx.x);
}

template <uint32_t T, int DBG = 0>
__global__ __launch_bounds__(T) __attribute__((amdgpu_waves_per_eu(8))) void k_small(mosrx_kparams kp)
{
	classify_tile_small<2, T, DBG>(kp, blockIdx.x);
}

typedef void (*lfn)(const mosrx_kparams *, hipStream_t);
template <uint32_t T, int DBG = 0>
static void launch_small(const mosrx_kparams *kp, hipStream_t s)
{
	hipLaunchKernelGGL((k_small<T, DBG>), dim3((kp->n + T - 1) / T), dim3(T), 0, s, *kp);
}
template <int DBG, int MINB = 1>
static void launch_dbg(const mosrx_kparams *kp, hipStream_t s)
{
	hipLaunchKernelGGL((k_dbg<DBG, MINB>), dim3((kp->n + 63) / 64), dim3(320), 0, s, *kp);
}
template <int S, int DBG, int W = 6, int U = 8, uint32_t T = 64>
static void launch_sdbg(const mosrx_kparams *kp, hipStream_t s)
{
	hipLaunchKernelGGL((k_sdbg<S, DBG, W, U, T>), dim3((kp->n + T - 1) / T), dim3(64 * (1 + S)), 0, s, *kp);
}
static void launch_product(const mosrx_kparams *kp, hipStream_t s)
{
	launch_dbg<0, 1>(kp, s);   // LARGE (no longer in the library)
}
static void launch_stream(const mosrx_kparams *kp, hipStream_t s)
{
	mosrx_launch_classify(kp, MOSRX_KIND_S13, 2, s);
}
template <int NT>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(8))) void k_snt(mosrx_kparams kp)
{
	classify_tile_stream_nt<3, 2, NT>(kp, blockIdx.x);
}
template <int NT>
static void launch_snt(const mosrx_kparams *kp, hipStream_t s)
{
	hipLaunchKernelGGL((k_snt<NT>), dim3((kp->n + 64 * NT - 1) / (64 * NT)), dim3(256), 0, s, *kp);
}

static int run(const char *name, lfn f, mosrx_kparams *kps, int nb, double bytes)
{
	hipEvent_t a, b;
	CHK(hipEventCreate(&a));
	CHK(hipEventCreate(&b));
	for (int i = 0; i < nb; i++)
		f(&kps[i], 0);
	const int iters = 60;
	float best_bb = 1e9, best_one = 1e9;
	for (int rep = 0; rep < 3; rep++) {
		float ms, one = 0;
		CHK(hipEventRecord(a, 0));
		for (int i = 0; i < iters; i++)
			f(&kps[i % nb], 0);
		CHK(hipEventRecord(b, 0));
		CHK(hipEventSynchronize(b));
		CHK(hipEventElapsedTime(&ms, a, b));
		for (int i = 0; i < iters; i++) {
			float t;
			CHK(hipEventRecord(a, 0));
			f(&kps[i % nb], 0);
			CHK(hipEventRecord(b, 0));
			CHK(hipEventSynchronize(b));
			CHK(hipEventElapsedTime(&t, a, b));
			one += t;
		}
		if (ms / iters < best_bb) best_bb = ms / iters;
		if (one / iters < best_one) best_one = one / iters;
	}
	printf("%-40s back-to-back %6.2f us (%5.0f GB/s) | single %6.2f us (%5.0f GB/s)\n", name, best_bb * 1e3,
	       bytes / (best_bb * 1e-3) / 1e9, best_one * 1e3, bytes / (best_one * 1e-3) / 1e9);
	return 0;
}

int main(int argc, char **argv)
{
	int kind = argc > 1 ? atoi(argv[1]) : MOSRX_TRACE_M1500;
	uint32_t n = argc > 2 ? (uint32_t)atoi(argv[2]) : 65536;
	mosrx_trace t;
	if (mosrx_trace_gen(kind, n, 1000000, 0, &t)) {
		printf("trace_gen failed\n");
		return 1;
	}
	if (argc > 3 && argv[3][0] == 'r') {   // descriptors in reverse buffer order: unsorted tiles
		for (uint32_t i = 0; i < n / 2; i++) {
			uint32_t to = t.off[i]; t.off[i] = t.off[n - 1 - i]; t.off[n - 1 - i] = to;
			uint16_t tl = t.len[i]; t.len[i] = t.len[n - 1 - i]; t.len[n - 1 - i] = tl;
		}
		printf("descriptors reversed\n");
	}
	const int nb = argc > 4 ? atoi(argv[4]) : 6;
	mosrx_kparams kps[64];
	uint32_t *tables;
	CHK(hipMalloc((void **)&tables, MOSRX_TAB_ALLOC_WORDS * 4));
	CHK(hipMemset(tables, 0, MOSRX_TAB_ALLOC_WORDS * 4));
	for (int i = 0; i < nb; i++) {
		uint8_t *f; uint32_t *o; uint16_t *l; mosrx_result *r;
		CHK(hipMalloc((void **)&f, t.frames_bytes + 64));
		CHK(hipMemcpy(f, t.frames, t.frames_bytes + 64, hipMemcpyHostToDevice));
		CHK(hipMalloc((void **)&o, n * 4));
		CHK(hipMemcpy(o, t.off, n * 4, hipMemcpyHostToDevice));
		CHK(hipMalloc((void **)&l, n * 2));
		CHK(hipMemcpy(l, t.len, n * 2, hipMemcpyHostToDevice));
		CHK(hipMalloc((void **)&r, n * 16));
		kps[i] = (mosrx_kparams){f, o, l, r, tables, NULL, NULL, NULL, NULL, (uint32_t)t.frames_bytes, n, MOSRX_KF_VERIFY};
	}
	const double bytes = (double)t.caplen_sum + 22.0 * n;
	printf("trace kind %d n %u: %.2f MB algorithmic\n", kind, n, bytes / 1e6);
	if (kind == MOSRX_TRACE_S64 || kind == MOSRX_TRACE_FW64) {
		run("product SMALL 256 (gathered windows)", launch_small<256>, kps, nb, bytes);
		run("SMALL 256 no window loads", launch_small<256, 2>, kps, nb, bytes);
		run("SMALL 128", launch_small<128>, kps, nb, bytes);
		return 0;
	}
	run("product S13", launch_stream, kps, nb, bytes);
	run("S13 x2 decoupled", launch_snt<2>, kps, nb, bytes);
	run("S13 x3 decoupled", launch_snt<3>, kps, nb, bytes);
	run("S13 x4 decoupled", launch_snt<4>, kps, nb, bytes);
	if (argc > 5)
		return 0;
	run("LARGE", launch_product, kps, nb, bytes);
	// S13 as the library builds it (8 waves/SIMD, 4 blocks in flight) with pieces removed
	run("S13 full", launch_sdbg<3, 0, 8, 4>, kps, nb, bytes);
	run("S13 streamers: loads only", launch_sdbg<3, 4, 8, 4>, kps, nb, bytes);
	run("S13 header: no parse", launch_sdbg<3, 1, 8, 4>, kps, nb, bytes);
	run("S13 header: no window loads", launch_sdbg<3, 2, 8, 4>, kps, nb, bytes);
	run("S13 no parse + streamer loads only", launch_sdbg<3, 5, 8, 4>, kps, nb, bytes);
	// streamer waves per 64-frame tile (S11 .. S14), library occupancy and depth
	run("S11 W8 U4", launch_sdbg<1, 0, 8, 4>, kps, nb, bytes);
	run("S12 W8 U4", launch_sdbg<2, 0, 8, 4>, kps, nb, bytes);
	run("S14 W8 U4", launch_sdbg<4, 0, 8, 4>, kps, nb, bytes);
	run("S12 W8 U6", launch_sdbg<2, 0, 8, 6>, kps, nb, bytes);
	return 0;
}
