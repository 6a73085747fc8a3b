// probe_tabfill.hip — the 64 B ring's table fill (diagnostic only).  New
// mechanism tested: every wave of the SMALL tile fills the whole 2 KiB of LDS
// tables itself (2 x 16-byte loads per lane, 8 KiB of L2 reads per 256 frames,
// 2 of a lane's 9 vector loads), so that no barrier is needed; DBG 256 fills
// them once per workgroup (8 bytes per lane) behind a barrier.  One launch over
// 8M x 64 B frames (the ring's work; 3 resident copies, > 1.5 GB), 16-byte and
// 8-byte records, the forms interleaved, 3 rounds; records checked equal.
#include "../mos-networking-stack_amd/csrc/mosrx_kernels.hip"
#include "../include/mosrx_trace.h"
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <vector>

#define CHK(x) do { if ((x) != hipSuccess) { printf("HIP error %s line %d\n", #x, __LINE__); return 1; } } while (0)

template <int VAR, int DBG>
__global__ __launch_bounds__(SMALL_THREADS) void k_small(mosrx_kparams kp)
{
	classify_tile_small<VAR, MOSRX_SMALL_FRAMES, DBG>(kp, blockIdx.x);
}

typedef void (*launch_fn)(const mosrx_kparams &);
template <int VAR, int DBG>
static void launch(const mosrx_kparams &kp)
{
	hipLaunchKernelGGL((k_small<VAR, DBG>), dim3((kp.n + MOSRX_SMALL_FRAMES - 1) / MOSRX_SMALL_FRAMES),
	                   dim3(SMALL_THREADS), 0, 0, kp);
}

int main(int argc, char **argv)
{
	const uint32_t n = argc > 1 ? (uint32_t)atoi(argv[1]) : 256u * 32768u;
	const int nb = 3;
	mosrx_trace t;
	if (mosrx_trace_gen(MOSRX_TRACE_S64, n, 1, 0, &t)) {
		printf("trace_gen failed\n");
		return 1;
	}
	mosrx_params p;
	mosrx_params_default(&p);
	std::vector<uint32_t> tab(MOSRX_TAB_ALLOC_WORDS, 0);
	mosrx_rss_tables(p.rss_key, p.rss_key_len, tab.data());
	uint32_t *tables;
	CHK(hipMalloc((void **)&tables, tab.size() * 4));
	CHK(hipMemcpy(tables, tab.data(), tab.size() * 4, hipMemcpyHostToDevice));
	mosrx_kparams kps[nb];
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
	}
	struct { const char *name; launch_fn fn; size_t rec; } forms[] = {
	    {"16 B records, per-wave fill (library)", launch<0, 0>, 16},
	    {"16 B records, one fill + barrier", launch<0, 256>, 16},
	    {"8 B records, per-wave fill (library)", launch<VAR_C8, 0>, 8},
	    {"8 B records, one fill + barrier", launch<VAR_C8, 256>, 8}};
	std::vector<uint8_t> a((size_t)n * 16), b((size_t)n * 16);
	for (int k = 0; k < 4; k += 2) {
		for (int j = 0; j < 2; j++) {
			CHK(hipMemset(kps[j].out, 0xEE, (size_t)n * 16));
			forms[k + j].fn(kps[j]);
			CHK(hipDeviceSynchronize());
		}
		CHK(hipMemcpy(a.data(), kps[0].out, (size_t)n * forms[k].rec, hipMemcpyDeviceToHost));
		CHK(hipMemcpy(b.data(), kps[1].out, (size_t)n * forms[k].rec, hipMemcpyDeviceToHost));
		printf("%s: records %s\n", forms[k + 1].name, memcmp(a.data(), b.data(), (size_t)n * forms[k].rec) ? "DIFFER" : "equal");
	}
	hipEvent_t e0, e1;
	CHK(hipEventCreate(&e0));
	CHK(hipEventCreate(&e1));
	const int iters = 30;
	for (int rep = 0; rep < 3; rep++) {
		for (auto &f : forms) {
			CHK(hipDeviceSynchronize());
			CHK(hipEventRecord(e0, 0));
			for (int i = 0; i < iters; i++)
				f.fn(kps[i % nb]);
			CHK(hipEventRecord(e1, 0));
			CHK(hipEventSynchronize(e1));
			float ms;
			CHK(hipEventElapsedTime(&ms, e0, e1));
			const double bytes = (double)t.caplen_sum + (6.0 + f.rec) * n;
			printf("rep %d %-40s %8.2f us per launch (%.3f of 8 TB/s, %.1f Gpkt/s)\n", rep, f.name, ms * 1e3 / iters,
			       bytes / (ms * 1e-3 / iters) / 8e12, n / (ms * 1e-3 / iters) / 1e9);
		}
	}
	return 0;
}
