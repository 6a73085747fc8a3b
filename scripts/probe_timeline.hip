// probe_timeline.hip — where a stream-tile launch spends its time (diagnostic only).
// Builds classify_tile_stream with DBG 128: every tile's header wave stamps the
// 100 MHz real-time clock at entry, descriptors ready, windows ready, parse done,
// barrier passed and records stored; the streamers at entry and at their barrier
// arrival; plus the header wave's HW_ID / XCC_ID.  The stamps force waits the
// kernel would do anyway (s_waitcnt 0), so the phases are close to the library's.
//   probe_timeline <trace kind> <frames> <resident batches>
#include "../mos-networking-stack_amd/csrc/mosrx_kernels.hip"
#include "probe_sp.h"
#include "probe_h2.h"
#include "probe_t128.h"
#include "../include/mosrx_trace.h"
#include <algorithm>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <vector>

#define CHK(x) do { if ((x) != hipSuccess) { printf("HIP error %s line %d\n", #x, __LINE__); return 1; } } while (0)

static double pct(std::vector<double> v, double q)
{
	if (v.empty()) return 0;
	std::sort(v.begin(), v.end());
	return v[std::min(v.size() - 1, (size_t)(q * v.size()))];
}

template <int DBG, int S = 3, int U = 4, int W = 8, uint32_t T = 64, int VAR = 2>
__global__ __launch_bounds__(64 * (1 + S)) __attribute__((amdgpu_waves_per_eu(W))) void k_tl(mosrx_kparams kp)
{
	classify_tile_stream<S, VAR, DBG, U, T>(kp, blockIdx.x);
}

template <int NT, int U = 4>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(8))) void k_sp(mosrx_kparams kp)
{
	classify_tile_sp<3, 2, NT, 0, U>(kp, blockIdx.x);
}

template <int NT, int U = 4>
static int plain_sp(const char *name, std::vector<mosrx_kparams> &kps, uint32_t ntiles, double bytes)
{
	const int nb = (int)kps.size();
	const uint32_t ng = (ntiles + NT - 1) / NT;
	hipEvent_t a, b;
	CHK(hipEventCreate(&a));
	CHK(hipEventCreate(&b));
	// records equal the library shape's (S13) on batch 0
	const uint32_t n = kps[0].n;
	mosrx_result *ref, *got;
	CHK(hipMalloc((void **)&ref, n * 16));
	CHK(hipMalloc((void **)&got, n * 16));
	mosrx_kparams k0 = kps[0];
	k0.out = ref;
	hipLaunchKernelGGL((k_tl<0>), dim3(ntiles), dim3(256), 0, 0, k0);
	k0.out = got;
	CHK(hipMemset(got, 0xAB, n * 16));
	hipLaunchKernelGGL((k_sp<NT, U>), dim3(ng), dim3(256), 0, 0, k0);
	CHK(hipDeviceSynchronize());
	std::vector<uint8_t> hr(n * 16), hg(n * 16);
	CHK(hipMemcpy(hr.data(), ref, n * 16, hipMemcpyDeviceToHost));
	CHK(hipMemcpy(hg.data(), got, n * 16, hipMemcpyDeviceToHost));
	uint32_t bad = 0, first = 0xFFFFFFFFu;
	for (uint32_t i = 0; i < n; i++)
		if (memcmp(&hr[16 * i], &hg[16 * i], 16)) { bad++; if (first == 0xFFFFFFFFu) first = i; }
	CHK(hipFree(ref));
	CHK(hipFree(got));
	float best = 1e9;
	for (int rep = 0; rep < 3; rep++) {
		for (int i = 0; i < nb; i++)
			hipLaunchKernelGGL((k_sp<NT, U>), dim3(ng), dim3(256), 0, 0, kps[i]);
		CHK(hipEventRecord(a, 0));
		for (int i = 0; i < 4 * nb; i++)
			hipLaunchKernelGGL((k_sp<NT, U>), dim3(ng), dim3(256), 0, 0, kps[i % nb]);
		CHK(hipEventRecord(b, 0));
		CHK(hipEventSynchronize(b));
		float ms;
		CHK(hipEventElapsedTime(&ms, a, b));
		best = std::min(best, ms / (4 * nb));
	}
	printf("%-24s back-to-back %6.2f us (%5.0f GB/s)  records %s (%u differ, first %d)\n", name, best * 1e3,
	       bytes / (best * 1e-3) / 1e9, bad ? "DIFFER" : "equal", bad, (int)first);
	return 0;
}

template <int H, int S, int W, int VAR>
__global__ __launch_bounds__(64 * (H + S)) __attribute__((amdgpu_waves_per_eu(W))) void k_h(mosrx_kparams kp)
{
	classify_tile_stream_h<H, S, VAR>(kp, blockIdx.x);
}
template <int F, int S, int U, int W, int VAR>
__global__ __launch_bounds__(64 * (1 + S)) __attribute__((amdgpu_waves_per_eu(W))) void k_f(mosrx_kparams kp)
{
	classify_tile_stream_f<F, S, VAR, U>(kp, blockIdx.x);
}

// a probe shape K (grid g, block w threads): records against the library shape
// on batch 0, then timed back to back over the resident batches
template <typename K>
static int plain_k(const char *name, K kern, uint32_t g, uint32_t w, std::vector<mosrx_kparams> &kps,
                   uint32_t ntiles, double bytes)
{
	const int nb = (int)kps.size();
	hipEvent_t a, b;
	CHK(hipEventCreate(&a));
	CHK(hipEventCreate(&b));
	const uint32_t n = kps[0].n;
	mosrx_result *ref, *got;
	CHK(hipMalloc((void **)&ref, n * 16));
	CHK(hipMalloc((void **)&got, n * 16));
	mosrx_kparams k0 = kps[0];
	k0.out = ref;
	hipLaunchKernelGGL((k_tl<0>), dim3(ntiles), dim3(256), 0, 0, k0);
	k0.out = got;
	CHK(hipMemset(got, 0xAB, n * 16));
	hipLaunchKernelGGL(kern, dim3(g), dim3(w), 0, 0, k0);
	CHK(hipDeviceSynchronize());
	std::vector<uint8_t> hr(n * 16), hg(n * 16);
	CHK(hipMemcpy(hr.data(), ref, n * 16, hipMemcpyDeviceToHost));
	CHK(hipMemcpy(hg.data(), got, n * 16, hipMemcpyDeviceToHost));
	uint32_t bad = 0, first = 0xFFFFFFFFu;
	for (uint32_t i = 0; i < n; i++)
		if (memcmp(&hr[16 * i], &hg[16 * i], 16)) { bad++; if (first == 0xFFFFFFFFu) first = i; }
	CHK(hipFree(ref));
	CHK(hipFree(got));
	float best = 1e9;
	for (int rep = 0; rep < 3; rep++) {
		for (int i = 0; i < nb; i++)
			hipLaunchKernelGGL(kern, dim3(g), dim3(w), 0, 0, kps[i]);
		CHK(hipEventRecord(a, 0));
		for (int i = 0; i < 4 * nb; i++)
			hipLaunchKernelGGL(kern, dim3(g), dim3(w), 0, 0, kps[i % nb]);
		CHK(hipEventRecord(b, 0));
		CHK(hipEventSynchronize(b));
		float ms;
		CHK(hipEventElapsedTime(&ms, a, b));
		best = std::min(best, ms / (4 * nb));
	}
	printf("%-24s back-to-back %6.2f us (%5.0f GB/s)  records %s (%u differ, first %d)\n", name, best * 1e3,
	       bytes / (best * 1e-3) / 1e9, bad ? "DIFFER" : "equal", bad, (int)first);
	return 0;
}
template <int H, int S, int W, int VAR = 0>
static int plain_h(const char *name, std::vector<mosrx_kparams> &kps, uint32_t ntiles, double bytes)
{
	return plain_k(name, k_h<H, S, W, VAR>, ntiles, 64 * (H + S), kps, ntiles, bytes);
}
template <int F, int S, int U, int W, int VAR = 0>
static int plain_f(const char *name, std::vector<mosrx_kparams> &kps, uint32_t ntiles, double bytes)
{
	return plain_k(name, k_f<F, S, U, W, VAR>, (kps[0].n + 64 * F - 1) / (64 * F), 64 * (1 + S), kps, ntiles,
	               bytes);
}

// one timing of a stream-tile variant: 4 passes over the resident batches, ms per launch
template <int S, int U, int W, int DBG, uint32_t T, int VAR>
static double time_tl(std::vector<mosrx_kparams> &kps, uint32_t ntiles64)
{
	const uint32_t ntiles = ntiles64 * (64 / T);
	const int nb = (int)kps.size();
	hipEvent_t a, b;
	if (hipEventCreate(&a) != hipSuccess || hipEventCreate(&b) != hipSuccess)
		return -1;
	for (int i = 0; i < nb; i++)
		hipLaunchKernelGGL((k_tl<DBG, S, U, W, T, VAR>), dim3(ntiles), dim3(64 * (1 + S)), 0, 0, kps[i]);
	hipEventRecord(a, 0);
	for (int i = 0; i < 4 * nb; i++)
		hipLaunchKernelGGL((k_tl<DBG, S, U, W, T, VAR>), dim3(ntiles), dim3(64 * (1 + S)), 0, 0, kps[i % nb]);
	hipEventRecord(b, 0);
	hipEventSynchronize(b);
	float ms = 0;
	hipEventElapsedTime(&ms, a, b);
	hipEventDestroy(a);
	hipEventDestroy(b);
	return ms / (4 * nb);
}

template <int S, int U, int W, int DBG = 0, uint32_t T = 64, int VAR = 2>
static int plain(const char *name, std::vector<mosrx_kparams> &kps, uint32_t ntiles64, double bytes)
{
	const uint32_t ntiles = ntiles64 * (64 / T);
	const int nb = (int)kps.size();
	hipEvent_t a, b;
	CHK(hipEventCreate(&a));
	CHK(hipEventCreate(&b));
	float best = 1e9;
	for (int rep = 0; rep < 3; rep++) {
		for (int i = 0; i < nb; i++)
			hipLaunchKernelGGL((k_tl<DBG, S, U, W, T, VAR>), dim3(ntiles), dim3(64 * (1 + S)), 0, 0, kps[i]);
		CHK(hipEventRecord(a, 0));
		for (int i = 0; i < 4 * nb; i++)
			hipLaunchKernelGGL((k_tl<DBG, S, U, W, T, VAR>), dim3(ntiles), dim3(64 * (1 + S)), 0, 0, kps[i % nb]);
		CHK(hipEventRecord(b, 0));
		CHK(hipEventSynchronize(b));
		float ms;
		CHK(hipEventElapsedTime(&ms, a, b));
		best = std::min(best, ms / (4 * nb));
	}
	printf("%-24s back-to-back %6.2f us (%5.0f GB/s)\n", name, best * 1e3, bytes / (best * 1e-3) / 1e9);
	return 0;
}

template <uint32_t T, int WEND = MOSRX_WINDOW_END_SMALL, int DBG = 0>
__global__ __launch_bounds__(T) __attribute__((amdgpu_waves_per_eu(8))) void k_small(mosrx_kparams kp)
{
	classify_tile_small<0, T, DBG, WEND>(kp, blockIdx.x);
}
template <uint32_t T, int WEND = MOSRX_WINDOW_END_SMALL, int DBG = 0>
static double time_small(std::vector<mosrx_kparams> &kps)
{
	const int nb = (int)kps.size();
	const uint32_t ng = (kps[0].n + T - 1) / T;
	hipEvent_t a, b;
	if (hipEventCreate(&a) != hipSuccess || hipEventCreate(&b) != hipSuccess)
		return -1;
	for (int i = 0; i < nb; i++)
		hipLaunchKernelGGL((k_small<T, WEND, DBG>), dim3(ng), dim3(T), 0, 0, kps[i]);
	hipEventRecord(a, 0);
	for (int i = 0; i < 2 * nb; i++)
		hipLaunchKernelGGL((k_small<T, WEND, DBG>), dim3(ng), dim3(T), 0, 0, kps[i % nb]);
	hipEventRecord(b, 0);
	hipEventSynchronize(b);
	float ms = 0;
	hipEventElapsedTime(&ms, a, b);
	hipEventDestroy(a);
	hipEventDestroy(b);
	return ms / (2 * nb);
}
// records of a SMALL variant against the library SMALL shape on batch 0
template <uint32_t T, int WEND>
static uint32_t small_diff(std::vector<mosrx_kparams> &kps)
{
	const uint32_t n = kps[0].n, ng = (n + T - 1) / T, ng0 = (n + 255) / 256;
	mosrx_result *ref, *got;
	if (hipMalloc((void **)&ref, n * 16) != hipSuccess || hipMalloc((void **)&got, n * 16) != hipSuccess)
		return 0xFFFFFFFFu;
	mosrx_kparams k0 = kps[0];
	k0.out = ref;
	hipLaunchKernelGGL((k_small<256>), dim3(ng0), dim3(256), 0, 0, k0);
	k0.out = got;
	hipMemset(got, 0xAB, n * 16);
	hipLaunchKernelGGL((k_small<T, WEND>), dim3(ng), dim3(T), 0, 0, k0);
	hipDeviceSynchronize();
	std::vector<uint8_t> hr(n * 16), hg(n * 16);
	hipMemcpy(hr.data(), ref, n * 16, hipMemcpyDeviceToHost);
	hipMemcpy(hg.data(), got, n * 16, hipMemcpyDeviceToHost);
	hipFree(ref);
	hipFree(got);
	uint32_t bad = 0;
	for (uint32_t i = 0; i < n; i++)
		bad += memcmp(&hr[16 * i], &hg[16 * i], 16) != 0;
	return bad;
}
template <uint32_t T>
static int plain_small(const char *name, std::vector<mosrx_kparams> &kps, double bytes)
{
	const int nb = (int)kps.size();
	const uint32_t ng = (kps[0].n + T - 1) / T;
	hipEvent_t a, b;
	CHK(hipEventCreate(&a));
	CHK(hipEventCreate(&b));
	float best = 1e9;
	for (int rep = 0; rep < 3; rep++) {
		for (int i = 0; i < nb; i++)
			hipLaunchKernelGGL((k_small<T>), dim3(ng), dim3(T), 0, 0, kps[i]);
		CHK(hipEventRecord(a, 0));
		for (int i = 0; i < 2 * nb; i++)
			hipLaunchKernelGGL((k_small<T>), dim3(ng), dim3(T), 0, 0, kps[i % nb]);
		CHK(hipEventRecord(b, 0));
		CHK(hipEventSynchronize(b));
		float ms;
		CHK(hipEventElapsedTime(&ms, a, b));
		best = std::min(best, ms / (2 * nb));
	}
	printf("%-24s back-to-back %6.2f us (%5.0f GB/s)\n", name, best * 1e3, bytes / (best * 1e-3) / 1e9);
	return 0;
}


int main(int argc, char **argv)
{
	const int kind = argc > 1 ? atoi(argv[1]) : MOSRX_TRACE_IMIX;
	const uint32_t n = argc > 2 ? (uint32_t)atoi(argv[2]) : 262144;
	const int nb = argc > 3 ? atoi(argv[3]) : 13;
	mosrx_trace t;
	if (mosrx_trace_gen(kind, n, 1000000, 0, &t)) {
		printf("trace_gen failed\n");
		return 1;
	}
	const uint32_t ntiles = (n + 63) / 64;
	uint32_t *tables, *stamps;
	CHK(hipMalloc((void **)&tables, MOSRX_TAB_ALLOC_WORDS * 4));
	CHK(hipMemset(tables, 0, MOSRX_TAB_ALLOC_WORDS * 4));
	CHK(hipMalloc((void **)&stamps, (size_t)ntiles * 64));
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
		kps[i] = (mosrx_kparams){f, o, l, r, tables, NULL, NULL, stamps, NULL, (uint32_t)t.frames_bytes, n,
		                         MOSRX_KF_VERIFY};
	}
	const double bytes = (double)t.caplen_sum + 22.0 * n;
	hipEvent_t a, b;
	CHK(hipEventCreate(&a));
	CHK(hipEventCreate(&b));
	// plain (DBG 0) back-to-back times over the resident batches, then stamped launches
	printf("trace kind %d n %u tiles %u: %.2f MB\n", kind, n, ntiles, bytes / 1e6);
	if (kind == MOSRX_TRACE_S64 || kind == MOSRX_TRACE_FW64) {
		if (argc > 4 && atoi(argv[4]) == 4) {
			// what bounds the SMALL tile: without the window loads / without the record stores
			std::vector<double> a, b, c;
			for (int r = 0; r < 9; r++) {
				a.push_back(time_small<256>(kps));
				b.push_back(time_small<256, MOSRX_WINDOW_END_SMALL, 2>(kps));
				c.push_back(time_small<256, MOSRX_WINDOW_END_SMALL, 4>(kps));
			}
			const char *nm[3] = {"SMALL 256 (library)", "SMALL 256 no window loads", "SMALL 256 no record stores"};
			std::vector<double> *v[3] = {&a, &b, &c};
			for (int k = 0; k < 3; k++)
				printf("%-28s median %8.2f us (%5.0f GB/s of algorithmic bytes)\n", nm[k], pct(*v[k], 0.5) * 1e3,
				       bytes / (pct(*v[k], 0.5) * 1e-3) / 1e9);
			return 0;
		}
		printf("SMALL 256 WEND 62: records %u differ\n", small_diff<256, MOSRX_WINDOW_END_STREAM>(kps));
		std::vector<double> a, b;
		for (int r = 0; r < 9; r++) {
			a.push_back(time_small<256>(kps));
			b.push_back(time_small<256, MOSRX_WINDOW_END_STREAM>(kps));
		}
		printf("SMALL 256 WEND 78 (library) median %7.2f us (%5.0f GB/s)\n", pct(a, 0.5) * 1e3,
		       bytes / (pct(a, 0.5) * 1e-3) / 1e9);
		printf("SMALL 256 WEND 62 (4 loads) median %7.2f us (%5.0f GB/s)\n", pct(b, 0.5) * 1e3,
		       bytes / (pct(b, 0.5) * 1e-3) / 1e9);
		return 0;
	}
	plain<3, 4, 8>("S13 U4 W8 (library)", kps, ntiles, bytes);
	plain<3, 4, 8, 0, 64, 0>("S13 tails cached (auto)", kps, ntiles, bytes);
	plain<3, 4, 8, 0, 64, 0>("S13 tails cached (auto)", kps, ntiles, bytes);
	if (argc > 4 && atoi(argv[4]) == 6) {
		// header wave priority (DBG 32: s_setprio 2 on the header wave), interleaved medians
		const char *names[] = {"S13 cached (library)", "S13 cached, header prio 2", "S13 nt (library)",
		                       "S13 nt, header prio 2"};
		std::vector<double> ts[4];
		for (int r = 0; r < 9; r++) {
			ts[0].push_back(time_tl<3, 4, 8, 0, 64, 0>(kps, ntiles));
			ts[1].push_back(time_tl<3, 4, 8, 32, 64, 0>(kps, ntiles));
			ts[2].push_back(time_tl<3, 4, 8, 0, 64, 2>(kps, ntiles));
			ts[3].push_back(time_tl<3, 4, 8, 32, 64, 2>(kps, ntiles));
		}
		for (int v = 0; v < 4; v++)
			printf("%-28s median %7.2f us  min %7.2f us  (%5.0f GB/s at the median)\n", names[v], pct(ts[v], 0.5) * 1e3,
			       pct(ts[v], 0.0) * 1e3, bytes / (pct(ts[v], 0.5) * 1e-3) / 1e9);
		return 0;
	}
	if (argc > 4 && atoi(argv[4]) == 5) {
		// streamer count x loads in flight: fewer streamers per tile = more tiles resident
		// (S1: 2-wave tiles, 16 per CU), interleaved rounds, median per variant
		const char *names[] = {"S3 U4 cached (library)", "S1 U8 cached", "S1 U6 cached", "S2 U6 cached",
		                       "S2 U4 cached", "S3 U4 nt (library)", "S1 U8 nt", "S2 U6 nt"};
		std::vector<double> ts[8];
		for (int r = 0; r < 7; r++) {
			ts[0].push_back(time_tl<3, 4, 8, 0, 64, 0>(kps, ntiles));
			ts[1].push_back(time_tl<1, 8, 8, 0, 64, 0>(kps, ntiles));
			ts[2].push_back(time_tl<1, 6, 8, 0, 64, 0>(kps, ntiles));
			ts[3].push_back(time_tl<2, 6, 8, 0, 64, 0>(kps, ntiles));
			ts[4].push_back(time_tl<2, 4, 8, 0, 64, 0>(kps, ntiles));
			ts[5].push_back(time_tl<3, 4, 8, 0, 64, 2>(kps, ntiles));
			ts[6].push_back(time_tl<1, 8, 8, 0, 64, 2>(kps, ntiles));
			ts[7].push_back(time_tl<2, 6, 8, 0, 64, 2>(kps, ntiles));
		}
		for (int v = 0; v < 8; v++)
			printf("%-28s median %7.2f us  min %7.2f us  (%5.0f GB/s at the median)\n", names[v], pct(ts[v], 0.5) * 1e3,
			       pct(ts[v], 0.0) * 1e3, bytes / (pct(ts[v], 0.5) * 1e-3) / 1e9);
		return 0;
	}
	if (argc > 4 && atoi(argv[4]) == 3) {
		// interleaved rounds, median and min per variant (cross-variant drift cancels)
		const char *names[] = {"cached: pend, tables first (lib)", "cached: pend, windows first",
		                       "cached: record after B, tables first", "cached: record after B, windows first",
		                       "nt: pend, tables first", "nt: pend, windows first (lib)", "nt: record after B, windows first (r2)"};
		std::vector<double> ts[7];
		for (int r = 0; r < 9; r++) {
			ts[0].push_back(time_tl<3, 4, 8, 0, 64, 0>(kps, ntiles));
			ts[1].push_back(time_tl<3, 4, 8, 4096, 64, 0>(kps, ntiles));
			ts[2].push_back(time_tl<3, 4, 8, 8192, 64, 0>(kps, ntiles));
			ts[3].push_back(time_tl<3, 4, 8, 8192 | 4096, 64, 0>(kps, ntiles));
			ts[4].push_back(time_tl<3, 4, 8, 4096, 64, 2>(kps, ntiles));
			ts[5].push_back(time_tl<3, 4, 8, 0, 64, 2>(kps, ntiles));
			ts[6].push_back(time_tl<3, 4, 8, 8192, 64, 2>(kps, ntiles));
		}
		for (int v = 0; v < 7; v++)
			printf("%-40s median %7.2f us  min %7.2f us  (%5.0f GB/s at the median)\n", names[v], pct(ts[v], 0.5) * 1e3,
			       pct(ts[v], 0.0) * 1e3, bytes / (pct(ts[v], 0.5) * 1e-3) / 1e9);
		return 0;
	}
	if (argc > 4 && atoi(argv[4]) == 2) {
		plain_h<1, 3, 8>("H1 S3 (probe copy)", kps, ntiles, bytes);
		plain_h<2, 3, 8>("H2 S3 (32 frames/hdr)", kps, ntiles, bytes);
		plain_h<2, 2, 8>("H2 S2 (32 frames/hdr)", kps, ntiles, bytes);
		plain_h<2, 6, 8>("H2 S6 (32 frames/hdr)", kps, ntiles, bytes);
	}
	plain_f<1, 3, 4, 8>("F1 S3 U4 (probe copy)", kps, ntiles, bytes);
	plain_f<2, 3, 4, 8>("F2 S3 U4 (128 frames)", kps, ntiles, bytes);
	plain<3, 4, 8, 2, 64, 0>("S13 no window loads, cached", kps, ntiles, bytes);
	plain<3, 4, 8, 1, 64, 0>("S13 no parse, cached", kps, ntiles, bytes);
	plain<3, 4, 8, 4, 64, 0>("S13 streamer loads only, cached", kps, ntiles, bytes);
	plain<3, 4, 8, 5, 64, 0>("S13 loads only (no parse, no sums)", kps, ntiles, bytes);
	plain<3, 4, 8, 7, 64, 0>("S13 stream loads + descriptors only", kps, ntiles, bytes);
	plain<3, 4, 8>("S13 U4 W8 (nt tails)", kps, ntiles, bytes);
	float ms;
	const bool after_b = argc > 5;   // timeline of the windows-after-the-barrier variant (DBG 512)
	for (int i = 0; i < 2 * nb; i++) {
		if (after_b)
			hipLaunchKernelGGL((k_tl<128 | 512>), dim3(ntiles), dim3(256), 0, 0, kps[i % nb]);
		else
			hipLaunchKernelGGL((k_tl<128>), dim3(ntiles), dim3(256), 0, 0, kps[i % nb]);
	}
	CHK(hipEventRecord(a, 0));
	if (after_b)
		hipLaunchKernelGGL((k_tl<128 | 512>), dim3(ntiles), dim3(256), 0, 0, kps[1 % nb]);
	else
		hipLaunchKernelGGL((k_tl<128>), dim3(ntiles), dim3(256), 0, 0, kps[1 % nb]);
	CHK(hipEventRecord(b, 0));
	CHK(hipEventSynchronize(b));
	CHK(hipEventElapsedTime(&ms, a, b));
	std::vector<uint32_t> st((size_t)ntiles * 16);
	CHK(hipMemcpy(st.data(), stamps, st.size() * 4, hipMemcpyDeviceToHost));
	printf("stamped launch %.2f us (event)\n", ms * 1e3);

	uint32_t t0 = 0xFFFFFFFFu, tend = 0;
	for (uint32_t i = 0; i < ntiles; i++) {
		t0 = std::min(t0, st[i * 16 + 0]);
		tend = std::max(tend, st[i * 16 + 5]);
	}
	const double us = 0.01;   // 100 MHz
	printf("first tile start -> last record stored: %.2f us\n", (tend - t0) * us);
	const char *ph[] = {"desc wait (h1-h0)", "window wait (h2-h1)", "parse (h3-h2)", "barrier wait (h4-h3)",
	                    "emit (h5-h4)"};
	for (int k = 0; k < 5; k++) {
		std::vector<double> d;
		for (uint32_t i = 0; i < ntiles; i++)
			d.push_back((double)(st[i * 16 + k + 1] - st[i * 16 + k]) * us);
		double m = 0;
		for (double x : d) m += x;
		printf("  %-22s mean %6.2f  p10 %6.2f  p50 %6.2f  p90 %6.2f us\n", ph[k], m / d.size(), pct(d, 0.1),
		       pct(d, 0.5), pct(d, 0.9));
	}
	{
		std::vector<double> life, sdone, lead;
		for (uint32_t i = 0; i < ntiles; i++) {
			const uint32_t *s = &st[i * 16];
			const uint32_t sd = std::max(s[7], std::max(s[8], s[9]));
			life.push_back((s[5] - s[0]) * us);
			sdone.push_back(((double)sd - (double)s[0]) * us);
			lead.push_back(((double)s[3] - (double)sd) * us);   // > 0: streamers waited for the header
		}
		printf("  tile lifetime           p10 %6.2f  p50 %6.2f  p90 %6.2f us\n", pct(life, .1), pct(life, .5),
		       pct(life, .9));
		printf("  streamers done (from h0) p10 %6.2f  p50 %6.2f  p90 %6.2f us\n", pct(sdone, .1), pct(sdone, .5),
		       pct(sdone, .9));
		printf("  header parse end - streamers done: p10 %6.2f p50 %6.2f p90 %6.2f us (>0: header is the long pole)\n",
		       pct(lead, .1), pct(lead, .5), pct(lead, .9));
	}
	// concurrency over time: tiles alive per 0.5 us bin, starts per bin
	const int nbin = (int)((tend - t0) * us / 0.5) + 1;
	std::vector<int> alive(nbin, 0), starts(nbin, 0);
	for (uint32_t i = 0; i < ntiles; i++) {
		const int b0 = (int)((st[i * 16] - t0) * us / 0.5), b1 = (int)((st[i * 16 + 5] - t0) * us / 0.5);
		starts[std::min(b0, nbin - 1)]++;
		for (int k = b0; k <= b1 && k < nbin; k++)
			alive[k]++;
	}
	printf("  t(us) alive starts\n");
	for (int k = 0; k < nbin; k++)
		printf("  %5.1f %5d %5d\n", k * 0.5, alive[k], starts[k]);
	// per-CU tile count spread (HW_ID cu_id bits 11:8, se_id 15:13; XCC)
	std::vector<int> percu(8 * 8 * 16 * 2, 0);
	for (uint32_t i = 0; i < ntiles; i++) {
		const uint32_t hw = st[i * 16 + 10], x = st[i * 16 + 11] & 7;
		const uint32_t cu = (hw >> 8) & 15, se = (hw >> 13) & 7, sh = (hw >> 12) & 1;
		percu[((x * 8 + se) * 2 + sh) * 16 + cu]++;
	}
	int used = 0, mx = 0, mn = 1 << 30;
	for (int c : percu)
		if (c) { used++; mx = std::max(mx, c); mn = std::min(mn, c); }
	printf("  CUs seen %d, tiles per CU min %d max %d\n", used, mn, mx);
	return 0;
}
