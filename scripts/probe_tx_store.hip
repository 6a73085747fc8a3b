// probe_tx_store.hip — where the in-place TX rewrite's extra time goes (diagnostic only).
// The 1500 B TX rewrite in place (bench row M1500_tx) takes ~2 us more per 64K
// batch than the same kernel writing 8-byte check records (M1500_txc), while
// its writes are only 3.5 MB more (PMC, profiles/r04/prof_tx).  The library's
// 1500 B TX tile (classify_tile_stream<3, 18>) is built here with the two
// 2-byte check-word stores per frame as the library issues them and with them
// non-temporal (DBG 8388608), with the same two words written as one u32 per
// frame into a dense array instead (DBG 16777216: the frames' scattered
// partial lines out of the picture), with them written through at system
// scope (DBG 33554432: no dirty lines left for the end-of-kernel writeback),
// and timed against the records form, over 24
// resident 64K-frame batches, dispatch-stamped, interleaved, 3 rounds.  Frames
// are restored between rounds (every form rewrites the same words).
//
//   hipcc -O3 --offload-arch=gfx950 -mllvm -amdgpu-kernarg-preload-count=7 -o scripts/probe_tx_store \
//     scripts/probe_tx_store.hip -Lmos-networking-stack_amd -lmosrx -Wl,-rpath,'$ORIGIN/../mos-networking-stack_amd'
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
__global__ __launch_bounds__(WG) __attribute__((amdgpu_waves_per_eu(8))) void k_tx(mosrx_kparams kp)
{
	classify_tile_stream<S, 2 | VAR_TX, DBG>(kp, blockIdx.x);
}

static int stamped(int f, const std::vector<mosrx_kparams> &kps, uint32_t tiles, int iters, double *med)
{
	std::vector<hipEvent_t> e0(iters), e1(iters);
	for (int i = 0; i < iters; i++) {
		CHK(hipEventCreate(&e0[i]));
		CHK(hipEventCreate(&e1[i]));
	}
	for (int i = 0; i < iters; i++) {
		mosrx_kparams kp = kps[i % kps.size()];
		if (f != 2)
			kp.out = NULL;   // in place (form 3: the words into the dense array at kp.fhash)
		if (f == 3)
			kp.fhash = (uint32_t *)kps[i % kps.size()].out;
		switch (f) {
		case 0: case 2: hipExtLaunchKernelGGL(k_tx<0>, dim3(tiles), dim3(WG), 0, 0, e0[i], e1[i], 0, kp); break;
		case 1: hipExtLaunchKernelGGL(k_tx<8388608>, dim3(tiles), dim3(WG), 0, 0, e0[i], e1[i], 0, kp); break;
		case 3: hipExtLaunchKernelGGL(k_tx<16777216>, dim3(tiles), dim3(WG), 0, 0, e0[i], e1[i], 0, kp); break;
		case 4: hipExtLaunchKernelGGL(k_tx<33554432>, dim3(tiles), dim3(WG), 0, 0, e0[i], e1[i], 0, kp); break;
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
	const uint32_t n = argc > 1 ? (uint32_t)atoi(argv[1]) : 65536;
	const int nb = 24;
	mosrx_trace t;
	if (mosrx_trace_gen(MOSRX_TRACE_M1500, n, 1000000, 0, &t)) {
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
	const uint32_t fl = MOSRX_KF_TX_IP | MOSRX_KF_TX_TCP;
	std::vector<mosrx_kparams> kps(nb);
	std::vector<uint8_t *> fr(nb);
	for (int i = 0; i < nb; i++) {
		uint8_t *f; uint32_t *o; uint16_t *l; mosrx_result *r;
		CHK(hipMalloc((void **)&f, t.frames_bytes + 64));
		CHK(hipMemcpy(f, t.frames, t.frames_bytes + 64, hipMemcpyHostToDevice));
		CHK(hipMalloc((void **)&o, n * 4));
		CHK(hipMemcpy(o, t.off, n * 4, hipMemcpyHostToDevice));
		CHK(hipMalloc((void **)&l, n * 2));
		CHK(hipMemcpy(l, t.len, n * 2, hipMemcpyHostToDevice));
		CHK(hipMalloc((void **)&r, n * 16));
		fr[i] = f;
		kps[i] = (mosrx_kparams){f, o, l, r, tables, NULL, NULL, NULL, NULL, (uint32_t)t.frames_bytes, n, fl};
	}
	// the two in-place forms rewrite the same bytes
	std::vector<uint8_t> a(t.frames_bytes), b(t.frames_bytes);
	mosrx_kparams kp = kps[0];
	kp.out = NULL;
	hipLaunchKernelGGL(k_tx<0>, dim3(tiles), dim3(WG), 0, 0, kp);
	CHK(hipDeviceSynchronize());
	CHK(hipMemcpy(a.data(), fr[0], t.frames_bytes, hipMemcpyDeviceToHost));
	CHK(hipMemcpy(fr[0], t.frames, t.frames_bytes, hipMemcpyHostToDevice));
	hipLaunchKernelGGL(k_tx<8388608>, dim3(tiles), dim3(WG), 0, 0, kp);
	CHK(hipDeviceSynchronize());
	CHK(hipMemcpy(b.data(), fr[0], t.frames_bytes, hipMemcpyDeviceToHost));
	if (memcmp(a.data(), b.data(), t.frames_bytes)) {
		printf("non-temporal stores give other frames\n");
		return 2;
	}
	CHK(hipMemcpy(fr[0], t.frames, t.frames_bytes, hipMemcpyHostToDevice));
	hipLaunchKernelGGL(k_tx<33554432>, dim3(tiles), dim3(WG), 0, 0, kp);
	CHK(hipDeviceSynchronize());
	CHK(hipMemcpy(b.data(), fr[0], t.frames_bytes, hipMemcpyDeviceToHost));
	if (memcmp(a.data(), b.data(), t.frames_bytes)) {
		printf("write-through stores give other frames\n");
		return 2;
	}
	const double bytes = (double)t.caplen_sum + 10.0 * n;
	printf("M1500 %u frames, %u tiles, %.2f MB algorithmic (in place); the three in-place forms give the same frames\n", n,
	       tiles, bytes / 1e6);
	static const char *names[5] = {"in place (library)", "in place, non-temporal stores", "8-byte records",
	                               "4-byte words, dense array", "in place, write-through stores"};
	for (int rep = 0; rep < 3; rep++)
		for (int f = 0; f < 5; f++) {
			for (int i = 0; i < nb; i++)
				CHK(hipMemcpy(fr[i], t.frames, t.frames_bytes, hipMemcpyHostToDevice));
			double med;
			if (stamped(f, kps, tiles, 240, &med))
				return 1;
			printf("rep %d %-30s stamped median %7.2f us\n", rep, names[f], med);
		}
	return 0;
}
