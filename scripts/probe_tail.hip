// probe_tail.hip — finer tiles at the end of a single launch (diagnostic only).
//
// A single 256K IMIX launch runs 4096 64-frame tiles in two rounds of the
// 2048 resident workgroups and ends with a drain of falling concurrency
// (DESIGN §4.4).  Here the last fraction f of the batch's frames goes into
// tiles of T2 = 32 or 16 frames (workgroups are dispatched in blockIdx order,
// so these are the last to start), the rest stays in 64-frame tiles:
//   block b <  A: frames [64 b, 64 b + 64)
//   block b >= A: frames [64 A + T2 (b - A), ... + T2)
// with the variant the library picks for the trace.  Every split is checked
// against the library's records before it is timed; forms interleave, 3 rounds.
#include "../mos-networking-stack_amd/csrc/mosrx_kernels.hip"
#include "../include/mosrx_trace.h"
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <vector>

#define CHK(x) do { if ((x) != hipSuccess) { printf("HIP error %s line %d\n", #x, __LINE__); return 1; } } while (0)

template <int VAR>
__global__ __launch_bounds__(64 * (1 + MOSRX_STREAMERS)) __attribute__((amdgpu_waves_per_eu(8)))
void k_lib(mosrx_kparams kp)
{
	classify_tile_stream<MOSRX_STREAMERS, VAR>(kp, blockIdx.x);
}

template <int VAR, uint32_t T2>
__global__ __launch_bounds__(64 * (1 + MOSRX_STREAMERS)) __attribute__((amdgpu_waves_per_eu(8)))
void k_split(mosrx_kparams kp, uint32_t A)
{
	const uint32_t b = blockIdx.x;
	const uint32_t first = b < A ? 64u * b : 64u * A + T2 * (b - A);
	const uint32_t cnt = min(b < A ? 64u : T2, kp.n - first);
	classify_span_stream<MOSRX_STREAMERS, VAR>(kp, b, first, cnt);
}

struct Form {
	const char *name;
	uint32_t t2;     // 0: the library
	double frac;     // share of the frames in T2-frame tiles
};

template <int VAR>
static void launch(const Form &f, const mosrx_kparams &kp, hipStream_t st)
{
	const uint32_t n = kp.n;
	if (!f.t2) {
		hipLaunchKernelGGL((k_lib<VAR>), dim3((n + 63) / 64), dim3(64 * (1 + MOSRX_STREAMERS)), 0, st, kp);
		return;
	}
	uint32_t A = (uint32_t)((1.0 - f.frac) * n) / 64u;
	const uint32_t rest = n - 64u * A, nb = A + (rest + f.t2 - 1) / f.t2;
	if (f.t2 == 32)
		hipLaunchKernelGGL((k_split<VAR, 32>), dim3(nb), dim3(64 * (1 + MOSRX_STREAMERS)), 0, st, kp, A);
	else if (f.t2 == 48)
		hipLaunchKernelGGL((k_split<VAR, 48>), dim3(nb), dim3(64 * (1 + MOSRX_STREAMERS)), 0, st, kp, A);
	else
		hipLaunchKernelGGL((k_split<VAR, 16>), dim3(nb), dim3(64 * (1 + MOSRX_STREAMERS)), 0, st, kp, A);
}

int main(int argc, char **argv)
{
	const int kind = argc > 1 ? atoi(argv[1]) : MOSRX_TRACE_IMIX;
	const uint32_t n = argc > 2 ? (uint32_t)atoi(argv[2]) : 262144;
	const int nb = 12;
	mosrx_trace t;
	if (mosrx_trace_gen(kind, n, 1000000, 0, &t)) {
		printf("trace_gen failed\n");
		return 1;
	}
	const int nt = t.frames_bytes / n >= 768 ? 1 : 0;
	mosrx_params p;
	mosrx_params_default(&p);
	std::vector<uint32_t> tab(MOSRX_TAB_ALLOC_WORDS, 0);
	mosrx_rss_tables(p.rss_key, p.rss_key_len, tab.data());
	for (uint32_t x = 0; x < 512; x++)
		((uint8_t *)(tab.data() + MOSRX_TAB_RSS_WORDS))[x] = (uint8_t)(x % 8);
	uint32_t *tables;
	CHK(hipMalloc((void **)&tables, tab.size() * 4));
	CHK(hipMemcpy(tables, tab.data(), tab.size() * 4, hipMemcpyHostToDevice));
	mosrx_kparams kps[nb];
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
	const double bytes = (double)t.caplen_sum + 22.0 * n;
	printf("trace kind %d n %u: %.2f MB algorithmic, variant %d\n", kind, n, bytes / 1e6, nt ? 2 : 0);
	const int sweep = argc > 3 ? atoi(argv[3]) : 0;
	const Form forms0[] = {{"library (64 only)", 0, 0},  {"tail 1/8 in 32", 32, 0.125}, {"tail 1/4 in 32", 32, 0.25},
	                       {"tail 1/2 in 32", 32, 0.5}, {"all in 32", 32, 1.0},       {"tail 1/8 in 16", 16, 0.125},
	                       {"tail 1/4 in 16", 16, 0.25}};
	// sweep 1: around the best 1500 B split of sweep 0
	const Form forms1[] = {{"library (64 only)", 0, 0},  {"tail 3/8 in 32", 32, 0.375}, {"tail 1/2 in 32", 32, 0.5},
	                       {"tail 5/8 in 32", 32, 0.625}, {"tail 3/4 in 32", 32, 0.75}, {"tail 1/2 in 48", 48, 0.5},
	                       {"all in 48", 48, 1.0},         {"tail 1/2 in 16", 16, 0.5}};
	const Form *forms = sweep ? forms1 : forms0;
	const int nforms = sweep ? 8 : 7;
	auto run = [&](const Form &f, const mosrx_kparams &kp) {
		if (nt) launch<2>(f, kp, 0); else launch<0>(f, kp, 0);
	};
	std::vector<mosrx_result> want(n), got(n);
	run(forms[0], kps[0]);
	CHK(hipDeviceSynchronize());
	CHK(hipMemcpy(want.data(), kps[0].out, n * 16, hipMemcpyDeviceToHost));
	for (int fi = 0; fi < nforms; fi++) {
		const Form &f = forms[fi];
		CHK(hipMemset(kps[1].out, 0xEE, n * 16));
		run(f, kps[1]);
		CHK(hipDeviceSynchronize());
		CHK(hipMemcpy(got.data(), kps[1].out, n * 16, hipMemcpyDeviceToHost));
		if (memcmp(got.data(), want.data(), (size_t)n * 16)) {
			printf("%s: RECORDS DIFFER\n", f.name);
			return 2;
		}
	}
	printf("every form: records equal to the library's\n");
	hipEvent_t a, b;
	CHK(hipEventCreate(&a));
	CHK(hipEventCreate(&b));
	const int iters = 200;
	for (int rep = 0; rep < 3; rep++) {
		for (int fi = 0; fi < nforms; fi++) {
			const Form &f = forms[fi];
			CHK(hipDeviceSynchronize());
			CHK(hipEventRecord(a, 0));
			for (int i = 0; i < iters; i++)
				run(f, kps[i % nb]);
			CHK(hipEventRecord(b, 0));
			CHK(hipEventSynchronize(b));
			float ms;
			CHK(hipEventElapsedTime(&ms, a, b));
			printf("rep %d %-20s back-to-back %7.2f us (%.3f of 8 TB/s)\n", rep, f.name, ms * 1e3 / iters,
			       bytes / (ms * 1e-3 / iters) / 8e12);
		}
	}
	return 0;
}
