// probe_small_hdr.hip — the SMALL tile's window in header-only mode (config
// #2's skip of TCPCalcChecksum; diagnostic only).  The library's SMALL tile
// loads 5 chunks (frame bytes [2, 78)) so that a 64-byte frame's TCP sum
// finishes in its lane; with the TCP sum skipped the headers end at byte 54
// and 4 chunks ([2, 62)) would do.  Both forms over one 8M-frame 64 B batch
// with 8-byte records, records compared, dispatch-stamped medians.
//
//   hipcc -O3 --offload-arch=gfx950 -mllvm -amdgpu-kernarg-preload-count=7 \
//     -o scripts/probe_small_hdr scripts/probe_small_hdr.hip -Lmos-networking-stack_amd -lmosrx \
//     -Wl,-rpath,'$ORIGIN/../mos-networking-stack_amd'
#include "../mos-networking-stack_amd/csrc/mosrx_kernels.hip"
#include "../include/mosrx_trace.h"
#include <algorithm>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <vector>

#define CHK(x) do { if ((x) != hipSuccess) { printf("HIP error %s line %d\n", #x, __LINE__); return 1; } } while (0)

template <int WEND>
__global__ __launch_bounds__(256) void k_small(mosrx_kparams kp)
{
	classify_tile_small<VAR_C8, MOSRX_KIND_FRAMES(MOSRX_KIND_SMALL), 0, WEND>(kp, blockIdx.x);
}

int main(int argc, char **argv)
{
	const uint32_t n = argc > 1 ? (uint32_t)atoi(argv[1]) : (1u << 23);
	const int nb = 3;
	mosrx_trace t;
	if (mosrx_trace_gen(MOSRX_TRACE_S64, n, 1000000, 0, &t)) {
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
	const uint32_t tiles = (n + 255) / 256;
	std::vector<mosrx_kparams> kps(nb);
	for (int i = 0; i < nb; i++) {
		uint8_t *f; uint32_t *o; uint16_t *l; mosrx_result *r;
		CHK(hipMalloc((void **)&f, t.frames_bytes + 64));
		CHK(hipMemcpy(f, t.frames, t.frames_bytes + 64, hipMemcpyHostToDevice));
		CHK(hipMalloc((void **)&o, (size_t)n * 4));
		CHK(hipMemcpy(o, t.off, (size_t)n * 4, hipMemcpyHostToDevice));
		CHK(hipMalloc((void **)&l, (size_t)n * 2));
		CHK(hipMemcpy(l, t.len, (size_t)n * 2, hipMemcpyHostToDevice));
		CHK(hipMalloc((void **)&r, (size_t)n * 8));
		kps[i] = (mosrx_kparams){f, o, l, r, tables, NULL, NULL, NULL, NULL, (uint32_t)t.frames_bytes, n,
		                         MOSRX_KF_VERIFY | MOSRX_KF_SKIP_TCP};
	}
	std::vector<uint64_t> a(n), b(n);
	hipLaunchKernelGGL(k_small<MOSRX_WINDOW_END_SMALL>, dim3(tiles), dim3(256), 0, 0, kps[0]);
	CHK(hipDeviceSynchronize());
	CHK(hipMemcpy(a.data(), kps[0].out, (size_t)n * 8, hipMemcpyDeviceToHost));
	CHK(hipMemset(kps[0].out, 0xEE, (size_t)n * 8));
	hipLaunchKernelGGL(k_small<MOSRX_WINDOW_END_STREAM>, dim3(tiles), dim3(256), 0, 0, kps[0]);
	CHK(hipDeviceSynchronize());
	CHK(hipMemcpy(b.data(), kps[0].out, (size_t)n * 8, hipMemcpyDeviceToHost));
	if (memcmp(a.data(), b.data(), (size_t)n * 8)) {
		printf("62-byte window: RECORDS DIFFER\n");
		return 2;
	}
	const double bytes = (double)t.caplen_sum + 14.0 * n;
	printf("S64 %u frames per launch (header-only, 8-byte records): %.1f MB algorithmic\n", n, bytes / 1e6);
	const int iters = 24;
	std::vector<hipEvent_t> e0(iters), e1(iters);
	for (int i = 0; i < iters; i++) {
		CHK(hipEventCreate(&e0[i]));
		CHK(hipEventCreate(&e1[i]));
	}
	for (int rep = 0; rep < 3; rep++)
		for (int w = 0; w < 2; w++) {
			for (int i = 0; i < iters; i++) {
				if (w == 0)
					hipExtLaunchKernelGGL(k_small<MOSRX_WINDOW_END_SMALL>, dim3(tiles), dim3(256), 0, 0, e0[i], e1[i],
					                      0, kps[i % nb]);
				else
					hipExtLaunchKernelGGL(k_small<MOSRX_WINDOW_END_STREAM>, dim3(tiles), dim3(256), 0, 0, e0[i],
					                      e1[i], 0, kps[i % nb]);
			}
			CHK(hipDeviceSynchronize());
			std::vector<float> d(iters);
			for (int i = 0; i < iters; i++)
				CHK(hipEventElapsedTime(&d[i], e0[i], e1[i]));
			std::sort(d.begin(), d.end());
			const double med = d[iters / 2] * 1e-3;
			printf("rep %d %s window  %8.2f us  %.1f Gpkt/s (%.3f of 8 TB/s)\n", rep, w ? "62-byte" : "78-byte",
			       med * 1e6, n / med / 1e9, bytes / med / 8e12);
		}
	return 0;
}
