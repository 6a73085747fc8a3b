// probe_guided.hip — the IMIX single launch with finer tiles at its end
// (diagnostic only): the first b1 blocks take 64 frames each (the library's
// stream tile), the rest 32, so the launch's last round -- whose spread of
// tile lifetimes is the drain -- is made of half-size tiles.  Records are
// checked against the library form before timing; dispatch-stamped medians.
//
//   hipcc -O3 --offload-arch=gfx950 -mllvm -amdgpu-kernarg-preload-count=7 \
//     -o scripts/probe_guided scripts/probe_guided.hip -Lmos-networking-stack_amd -lmosrx \
//     -Wl,-rpath,'$ORIGIN/../mos-networking-stack_amd'
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

__global__ __launch_bounds__(WG) __attribute__((amdgpu_waves_per_eu(8))) void k_plain(mosrx_kparams kp)
{
	classify_tile_stream<S, 0>(kp, blockIdx.x);
}

// the library's tile with the 78-byte window (5 chunks: a 64-byte frame needs no streamer)
__global__ __launch_bounds__(WG) __attribute__((amdgpu_waves_per_eu(8))) void k_w78(mosrx_kparams kp)
{
	classify_tile_stream<S, 0, 1048576>(kp, blockIdx.x);
}

__global__ __launch_bounds__(WG) __attribute__((amdgpu_waves_per_eu(8))) void k_guided(mosrx_kparams kp, uint32_t b1)
{
	const uint32_t b = blockIdx.x;
	const uint32_t first = b < b1 ? 64u * b : 64u * b1 + 32u * (b - b1);
	const uint32_t cnt = min(b < b1 ? 64u : 32u, kp.n - first);
	classify_span_stream<S, 0>(kp, b, first, cnt);
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
	uint32_t tab[MOSRX_TAB_ALLOC_WORDS];
	memset(tab, 0, sizeof(tab));
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
	hipLaunchKernelGGL(k_plain, dim3(tiles), dim3(WG), 0, 0, kps[0]);
	CHK(hipDeviceSynchronize());
	CHK(hipMemcpy(a.data(), kps[0].out, n * 16, hipMemcpyDeviceToHost));
	CHK(hipMemset(kps[0].out, 0xEE, n * 16));
	hipLaunchKernelGGL(k_w78, dim3(tiles), dim3(WG), 0, 0, kps[0]);
	CHK(hipDeviceSynchronize());
	CHK(hipMemcpy(b.data(), kps[0].out, n * 16, hipMemcpyDeviceToHost));
	if (memcmp(a.data(), b.data(), (size_t)n * 16)) {
		printf("78-byte window: RECORDS DIFFER\n");
		return 2;
	}
	const double bytes = (double)t.caplen_sum + 22.0 * n;
	// b1 = tiles * q / 8 blocks of 64 frames, the rest in 32-frame tiles
	const int qs[] = {8, 7, 6, 4, 0};
	for (int q : qs) {
		const uint32_t b1 = tiles * q / 8, nblk = b1 + (n - 64u * b1 + 31u) / 32u;
		CHK(hipMemset(kps[0].out, 0xEE, n * 16));
		hipLaunchKernelGGL(k_guided, dim3(nblk), dim3(WG), 0, 0, kps[0], b1);
		CHK(hipDeviceSynchronize());
		CHK(hipMemcpy(b.data(), kps[0].out, n * 16, hipMemcpyDeviceToHost));
		if (memcmp(a.data(), b.data(), (size_t)n * 16)) {
			printf("guided q=%d: RECORDS DIFFER\n", q);
			return 2;
		}
	}
	printf("IMIX %u frames, %.2f MB algorithmic per batch\n", n, bytes / 1e6);
	const int iters = 128;
	std::vector<hipEvent_t> e0(iters), e1(iters);
	for (int i = 0; i < iters; i++) {
		CHK(hipEventCreate(&e0[i]));
		CHK(hipEventCreate(&e1[i]));
	}
	for (int rep = 0; rep < 3; rep++)
		for (int qi = -2; qi < 5; qi++) {
			if (qi == -2) {
				for (int i = 0; i < iters; i++)
					hipExtLaunchKernelGGL(k_w78, dim3(tiles), dim3(WG), 0, 0, e0[i], e1[i], 0, kps[i % nb]);
				CHK(hipDeviceSynchronize());
				std::vector<float> d(iters);
				for (int i = 0; i < iters; i++)
					CHK(hipEventElapsedTime(&d[i], e0[i], e1[i]));
				std::sort(d.begin(), d.end());
				const double med = d[iters / 2] * 1e-3;
				printf("rep %d 78-byte window                 %7.2f us (%.3f of 8 TB/s)\n", rep, med * 1e6,
				       bytes / med / 8e12);
				continue;
			}
			const int q = qi < 0 ? 8 : qs[qi];
			const uint32_t b1 = tiles * q / 8, nblk = b1 + (n - 64u * b1 + 31u) / 32u;
			for (int i = 0; i < iters; i++) {
				if (qi < 0)
					hipExtLaunchKernelGGL(k_plain, dim3(tiles), dim3(WG), 0, 0, e0[i], e1[i], 0, kps[i % nb]);
				else
					hipExtLaunchKernelGGL(k_guided, dim3(nblk), dim3(WG), 0, 0, e0[i], e1[i], 0, kps[i % nb], b1);
			}
			CHK(hipDeviceSynchronize());
			std::vector<float> d(iters);
			for (int i = 0; i < iters; i++)
				CHK(hipEventElapsedTime(&d[i], e0[i], e1[i]));
			std::sort(d.begin(), d.end());
			const double med = d[iters / 2] * 1e-3;
			if (qi < 0)
				printf("rep %d library (64-frame tiles)      %7.2f us (%.3f of 8 TB/s)\n", rep, med * 1e6,
				       bytes / med / 8e12);
			else
				printf("rep %d 64-frame tiles for %d/8, then 32 %7.2f us (%.3f of 8 TB/s)\n", rep, q, med * 1e6,
				       bytes / med / 8e12);
		}
	return 0;
}
