// probe_prefetch.hip — the IMIX single launch's second round (diagnostic only).
// A 256K-frame IMIX launch has 4096 stream tiles of which 2048 are resident at
// once (8 waves per SIMD); tile b + 2048 runs on tile b's XCD after the first
// round retires, and its first act is a dependent descriptor round trip to
// HBM.  Here the library's stream tile (classify_tile_stream<3, 0>, the IMIX
// variant) is built three ways: as the library has it, with streamer 0
// reading tile b + 2048's descriptors into L2 while it streams its own tile
// (DBG 2097152), and with it also touching the first line of each of that
// tile's frames before it retires (DBG 4194304).  Records are checked equal to
// the plain form, then single launches over 24 resident batches (2.3 GB, past
// the Infinity Cache) are timed dispatch-stamped, interleaved, 3 rounds.
//
//   hipcc -O3 --offload-arch=gfx950 -mllvm -amdgpu-kernarg-preload-count=7 -o scripts/probe_prefetch \
//     scripts/probe_prefetch.hip -Lmos-networking-stack_amd -lmosrx -Wl,-rpath,'$ORIGIN/../mos-networking-stack_amd'
#include "../mos-networking-stack_amd/csrc/mosrx_kernels.hip"
#include "../include/mosrx_trace.h"
#include <algorithm>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <vector>

#define CHK(x) do { if ((x) != hipSuccess) { printf("HIP error %s line %d\n", #x, __LINE__); return 1; } } while (0)
#define S 3
#define WG (64 * (1 + S))

template <int DBG>
__global__ __launch_bounds__(WG) __attribute__((amdgpu_waves_per_eu(8))) void k_tile(mosrx_kparams kp)
{
	classify_tile_stream<S, 0, DBG>(kp, blockIdx.x);
}

static int stamped(int f, const std::vector<mosrx_kparams> &kps, uint32_t tiles, int iters, double *med)
{
	std::vector<hipEvent_t> e0(iters), e1(iters);
	for (int i = 0; i < iters; i++) {
		CHK(hipEventCreate(&e0[i]));
		CHK(hipEventCreate(&e1[i]));
	}
	for (int i = 0; i < iters; i++) {
		const mosrx_kparams &kp = kps[i % kps.size()];
		switch (f) {
		case 0: hipExtLaunchKernelGGL(k_tile<0>, dim3(tiles), dim3(WG), 0, 0, e0[i], e1[i], 0, kp); break;
		case 1: hipExtLaunchKernelGGL(k_tile<2097152>, dim3(tiles), dim3(WG), 0, 0, e0[i], e1[i], 0, kp); break;
		case 2: hipExtLaunchKernelGGL(k_tile<4194304>, dim3(tiles), dim3(WG), 0, 0, e0[i], e1[i], 0, kp); break;
		}
	}
	CHK(hipDeviceSynchronize());
	std::vector<float> d(iters);
	for (int i = 0; i < iters; i++) {
		CHK(hipEventElapsedTime(&d[i], e0[i], e1[i]));
		CHK(hipEventDestroy(e0[i]));
		CHK(hipEventDestroy(e1[i]));
	}
	std::sort(d.begin(), d.end());
	*med = d[iters / 2] * 1e3;
	return 0;
}

int main(int argc, char **argv)
{
	const uint32_t n = argc > 1 ? (uint32_t)atoi(argv[1]) : 262144;
	const int nb = 24;
	mosrx_trace t;
	if (mosrx_trace_gen(MOSRX_TRACE_IMIX, n, 1000000, 0, &t)) {
		printf("trace_gen failed\n");
		return 1;
	}
	mosrx_params p;
	mosrx_params_default(&p);
	static uint32_t tab[MOSRX_TAB_ALLOC_WORDS];
	mosrx_rss_tables(p.rss_key, p.rss_key_len, tab);
	uint32_t *tables;
	CHK(hipMalloc((void **)&tables, sizeof(tab)));
	CHK(hipMemcpy(tables, tab, sizeof(tab), hipMemcpyHostToDevice));
	const uint32_t tiles = (n + 63) / 64;
	std::vector<mosrx_kparams> kps(nb);
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
	std::vector<mosrx_result> a(n), b(n);
	hipLaunchKernelGGL(k_tile<0>, dim3(tiles), dim3(WG), 0, 0, kps[0]);
	CHK(hipDeviceSynchronize());
	CHK(hipMemcpy(a.data(), kps[0].out, n * 16, hipMemcpyDeviceToHost));
	for (int f = 1; f < 3; f++) {
		CHK(hipMemset(kps[0].out, 0xEE, n * 16));
		if (f == 1)
			hipLaunchKernelGGL(k_tile<2097152>, dim3(tiles), dim3(WG), 0, 0, kps[0]);
		else
			hipLaunchKernelGGL(k_tile<4194304>, dim3(tiles), dim3(WG), 0, 0, kps[0]);
		CHK(hipDeviceSynchronize());
		CHK(hipMemcpy(b.data(), kps[0].out, n * 16, hipMemcpyDeviceToHost));
		if (memcmp(a.data(), b.data(), (size_t)n * 16)) {
			printf("form %d records differ from plain\n", f);
			return 2;
		}
	}
	const double bytes = (double)t.caplen_sum + 22.0 * n;
	printf("IMIX %u frames, %u tiles, %.2f MB algorithmic; records of all forms equal\n", n, tiles, bytes / 1e6);
	static const char *names[3] = {"library", "prefetch next descriptors", "prefetch descriptors + lines"};
	for (int rep = 0; rep < 3; rep++)
		for (int f = 0; f < 3; f++) {
			double med;
			if (stamped(f, kps, tiles, 256, &med))
				return 1;
			printf("rep %d %-30s stamped median %7.2f us (%.3f of 8 TB/s)\n", rep, names[f], med,
			       bytes / (med * 1e-6) / 8e12);
		}
	return 0;
}
