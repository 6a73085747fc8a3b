// probe_hint_tiles.hip — config #2's isolated single launch (32K x 64 B) with the
// layout hint (VAR_UNI), at three workgroup sizes (diagnostic only; for
// rocprofv3 --kernel-trace).  New mechanism tested: with the hint the tile's
// chain is one HBM round trip, so what is left is the parse per wave and how
// many CUs share the launch -- 256-frame workgroups (the library: 128 of them,
// 4 waves each, half the CUs) against 128- and 64-frame ones (256 / 512
// workgroups over every CU).  Each launch is isolated (host sync after it), the
// three forms alternate over 256 resident copies (512 MB, past the Infinity
// Cache), and their records are checked equal first.
#include "../mos-networking-stack_amd/csrc/mosrx_kernels.hip"
#include "../include/mosrx_trace.h"
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <vector>

#define CHK(x) do { if ((x) != hipSuccess) { printf("HIP error %s line %d\n", #x, __LINE__); return 1; } } while (0)

template <uint32_t T>
__global__ __launch_bounds__(T) void k_hint(mosrx_kparams kp)
{
	classify_tile_small<VAR_UNI, T>(kp, blockIdx.x);
}

template <uint32_t T>
static void launch(const mosrx_kparams &kp)
{
	hipLaunchKernelGGL((k_hint<T>), dim3((kp.n + T - 1) / T), dim3(T), 0, 0, kp);
}

int main(int argc, char **argv)
{
	const int iters = argc > 1 ? atoi(argv[1]) : 3000;
	const uint32_t n = 32768u;
	const int nb = 256;
	mosrx_trace t;
	if (mosrx_trace_gen(MOSRX_TRACE_S64, n, 1, 0, &t)) {
		printf("trace_gen failed\n");
		return 1;
	}
	const uint32_t stride = t.off[1] - t.off[0];
	for (uint32_t i = 0; i < n; i++)
		if (t.off[i] != t.off[0] + i * stride) {
			printf("trace not uniform\n");
			return 1;
		}
	mosrx_params p;
	mosrx_params_default(&p);
	std::vector<uint32_t> tab(MOSRX_TAB_ALLOC_WORDS, 0);
	std::vector<uint8_t> lut(512);
	mosrx_rss_tables(p.rss_key, p.rss_key_len, tab.data());
	for (uint32_t h = 0; h < 512; h++)   // num_queues 1: every queue 0
		lut[h] = 0;
	memcpy(tab.data() + MOSRX_TAB_RSS_WORDS, lut.data(), 512);
	uint32_t *tables;
	CHK(hipMalloc((void **)&tables, tab.size() * 4));
	CHK(hipMemcpy(tables, tab.data(), tab.size() * 4, hipMemcpyHostToDevice));
	std::vector<mosrx_kparams> kps(nb);
	for (int i = 0; i < nb; i++) {
		uint8_t *f; uint32_t *o; uint16_t *l; mosrx_result *r;
		CHK(hipMalloc((void **)&f, t.frames_bytes + 64));
		CHK(hipMemcpy(f, t.frames, t.frames_bytes + 64, hipMemcpyHostToDevice));
		CHK(hipMalloc((void **)&o, (size_t)n * 4));
		CHK(hipMemcpy(o, t.off, (size_t)n * 4, hipMemcpyHostToDevice));
		CHK(hipMalloc((void **)&l, (size_t)n * 2));
		CHK(hipMemcpy(l, t.len, (size_t)n * 2, hipMemcpyHostToDevice));
		CHK(hipMalloc((void **)&r, (size_t)n * 16));
		memset(&kps[i], 0, sizeof(kps[i]));
		kps[i].frames = f; kps[i].off = o; kps[i].len = l; kps[i].out = r; kps[i].tables = tables;
		kps[i].frames_bytes = (uint32_t)t.frames_bytes; kps[i].n = n; kps[i].flags = MOSRX_KF_VERIFY;
		kps[i].uni = (t.off[0] << 16) | stride;
	}
	void (*forms[])(const mosrx_kparams &) = {launch<256>, launch<128>, launch<64>};
	const char *names[] = {"256-frame workgroups (library)", "128-frame workgroups", "64-frame workgroups"};
	std::vector<mosrx_result> ref(n), got(n);
	for (int k = 0; k < 3; k++) {
		CHK(hipMemset(kps[k].out, 0xEE, (size_t)n * 16));
		forms[k](kps[k]);
		CHK(hipDeviceSynchronize());
		CHK(hipMemcpy(k ? got.data() : ref.data(), kps[k].out, (size_t)n * 16, hipMemcpyDeviceToHost));
		if (k && memcmp(ref.data(), got.data(), (size_t)n * 16)) {
			printf("records of form %d DIFFER from the library's\n", k);
			return 1;
		}
	}
	uint64_t ok = 0;
	for (uint32_t i = 0; i < n; i++)
		ok += ref[i].verdict == 1;
	printf("records equal across forms; %lu of %u verdict 1\n", (unsigned long)ok, n);
	for (int i = 0; i < iters; i++)
		for (int k = 0; k < 3; k++) {
			forms[k](kps[(i * 3 + k) % nb]);
			CHK(hipDeviceSynchronize());
		}
	printf("%d isolated launches of each form\n", iters);
	return 0;
}
