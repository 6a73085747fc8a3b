// probe_rss.hip — forms of the header wave's Toeplitz (diagnostic only).
//
// VERDICT r2 #4 asks for the 24 nibble lookups to be replaced by 12 byte
// lookups (12 x 256 x u32 = 12 KiB of LDS).  The library's stream tile
// (classify_tile_stream, one workgroup per 64-frame tile) runs here with
//   nibble  the library: 24 nibble tables (1.5 KiB) in LDS,
//   none    no Toeplitz at all (wrong hashes): the bound on any faster form,
//   byte    12 byte tables staged in LDS by the header wave (12 KiB),
//   byte-g  the 12 byte tables read from global memory (L1 / L2), no staging,
// each with the variant the library picks for the trace (mean frame >= 768 B:
// non-temporal tails).  Every form but `none` is checked against the library
// records before it is timed; the timings interleave the forms, 3 rounds.
#include "../mos-networking-stack_amd/csrc/mosrx_kernels.hip"
#include "../include/mosrx_trace.h"
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <vector>

#define CHK(x) do { if ((x) != hipSuccess) { printf("HIP error %s line %d\n", #x, __LINE__); return 1; } } while (0)

template <int VAR, int DBG>
__global__ __launch_bounds__(64 * (1 + MOSRX_STREAMERS)) __attribute__((amdgpu_waves_per_eu(8)))
void k_tile(mosrx_kparams kp)
{
	classify_tile_stream<MOSRX_STREAMERS, VAR, DBG>(kp, blockIdx.x);
}

typedef void (*launch_fn)(const mosrx_kparams &, uint32_t, hipStream_t);
template <int VAR, int DBG>
static void launch(const mosrx_kparams &kp, uint32_t ntiles, hipStream_t st)
{
	hipLaunchKernelGGL((k_tile<VAR, DBG>), dim3(ntiles), dim3(64 * (1 + MOSRX_STREAMERS)), 0, st, kp);
}

struct Form {
	const char *name;
	launch_fn fn[2];   // [variant 0 (cached tails), variant 2 (non-temporal tails)]
	int check;
};

int main(int argc, char **argv)
{
	const int kind = argc > 1 ? atoi(argv[1]) : MOSRX_TRACE_M1500;
	const uint32_t n = argc > 2 ? (uint32_t)atoi(argv[2]) : 65536;
	const int nb = 12;                        // resident batch copies cycled (> 1.2 GB for the big traces)
	mosrx_trace t;
	if (mosrx_trace_gen(kind, n, 1000000, 0, &t)) {
		printf("trace_gen failed\n");
		return 1;
	}
	const uint32_t ntiles = (n + 63) / 64;
	const int nt = t.frames_bytes / n >= 768 ? 1 : 0;

	// tables: the library's default key, 8 queues; byte tables at MOSRX_TAB8_OFF
	mosrx_params p;
	mosrx_params_default(&p);
	std::vector<uint32_t> tab(MOSRX_TAB8_OFF + 12 * 256, 0);
	mosrx_rss_tables(p.rss_key, p.rss_key_len, tab.data());
	for (uint32_t x = 0; x < 512; x++)
		((uint8_t *)(tab.data() + MOSRX_TAB_RSS_WORDS))[x] = (uint8_t)(x % 8);
	for (int k = 0; k < 12; k++)
		for (int v = 0; v < 256; v++)
			tab[MOSRX_TAB8_OFF + 256 * k + v] = tab[(2 * k) * 16 + (v >> 4)] ^ tab[(2 * k + 1) * 16 + (v & 15)];
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
	printf("trace kind %d n %u tiles %u: %.2f MB algorithmic, variant %d\n", kind, n, ntiles, bytes / 1e6, nt ? 2 : 0);

	const Form forms[] = {
	    {"nibble (library)", {launch<0, 0>, launch<2, 0>}, 1},
	    {"none (bound)", {launch<0, 16384>, launch<2, 16384>}, 0},
	    {"byte LDS", {launch<0, 32768>, launch<2, 32768>}, 1},
	    {"byte global", {launch<0, 65536>, launch<2, 65536>}, 1},
	};
	std::vector<mosrx_result> want(n), got(n);
	hipStream_t st = 0;
	forms[0].fn[nt](kps[0], ntiles, st);
	CHK(hipDeviceSynchronize());
	CHK(hipMemcpy(want.data(), kps[0].out, n * 16, hipMemcpyDeviceToHost));
	uint32_t qs = 0;
	for (uint32_t i = 0; i < n; i++)
		qs |= 1u << (want[i].queue & 7);
	printf("library records: queues seen mask 0x%02x\n", qs);
	for (const Form &f : forms) {
		if (!f.check)
			continue;
		CHK(hipMemset(kps[1].out, 0xEE, n * 16));
		f.fn[nt](kps[1], ntiles, st);
		CHK(hipDeviceSynchronize());
		CHK(hipMemcpy(got.data(), kps[1].out, n * 16, hipMemcpyDeviceToHost));
		if (memcmp(got.data(), want.data(), (size_t)n * 16)) {
			printf("%s: RECORDS DIFFER\n", f.name);
			return 2;
		}
		printf("%s: records equal\n", f.name);
	}
	hipEvent_t a, b;
	CHK(hipEventCreate(&a));
	CHK(hipEventCreate(&b));
	const int iters = 200;
	for (int rep = 0; rep < 3; rep++) {
		for (const Form &f : forms) {
			CHK(hipDeviceSynchronize());
			CHK(hipEventRecord(a, st));
			for (int i = 0; i < iters; i++)
				f.fn[nt](kps[i % nb], ntiles, st);
			CHK(hipEventRecord(b, st));
			CHK(hipEventSynchronize(b));
			float ms, one = 0;
			CHK(hipEventElapsedTime(&ms, a, b));
			for (int i = 0; i < iters; i++) {
				float tt;
				CHK(hipEventRecord(a, st));
				f.fn[nt](kps[i % nb], ntiles, st);
				CHK(hipEventRecord(b, st));
				CHK(hipEventSynchronize(b));
				CHK(hipEventElapsedTime(&tt, a, b));
				one += tt;
			}
			printf("rep %d %-18s back-to-back %7.2f us (%.3f of 8 TB/s) | single %7.2f us (%.3f)\n", rep, f.name,
			       ms * 1e3 / iters, bytes / (ms * 1e-3 / iters) / 8e12, one * 1e3 / iters,
			       bytes / (one * 1e-3 / iters) / 8e12);
		}
	}
	return 0;
}
