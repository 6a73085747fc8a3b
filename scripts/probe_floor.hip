// probe_floor.hip — the single 64 B launch's floor (diagnostic only).
// Config #2 literally is one launch over 32K frames of 64 B (bench row S64_1,
// ~4.1 us, 0.08 of 8 TB/s).  This probe times, dispatch-stamped and over
// rotating buffers (1.4 GB, past the 256 MiB Infinity Cache, as the bench),
// the stages such a launch cannot avoid, in 128 workgroups of 256 lanes (the
// SMALL tile's grid) and in 512 of 64:
//   empty        the dispatch alone
//   store        one 16-byte record per frame
//   desc+store   the descriptor load (off) then the record
//   chain16      off + len, then 16 bytes of the frame at off, then the record
//   chain80      off + len, then the 80-byte window (5 x 16 B), then the record
//   library      the library's SMALL classify kernel over config #2's trace
//                (mosrx_classify_kernel<SMALL, 0>, 128 tiles of 256 frames)
// So the library's 4.1 us can be set against the dependent round trips and
// the store drain it is made of.  Each is also timed back to back (400
// launches between one event pair), the per-launch cost when dispatches overlap.
//
//   hipcc -O3 --offload-arch=gfx950 -mllvm -amdgpu-kernarg-preload-count=7 -o scripts/probe_floor \
//     scripts/probe_floor.hip -Lmos-networking-stack_amd -lmosrx -Wl,-rpath,'$ORIGIN/../mos-networking-stack_amd'
#include "../mos-networking-stack_amd/csrc/mosrx_kernels.hip"
#include "../include/mosrx_trace.h"
#include <hip/hip_ext.h>
#include <algorithm>
#include <stdint.h>
#include <stdio.h>
#include <vector>

#define CHK(x) do { if ((x) != hipSuccess) { printf("HIP error %s line %d\n", #x, __LINE__); return 1; } } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

struct set {
	const uint8_t *frames;
	const uint32_t *off;
	const uint16_t *len;
	u32x4 *out;
};

template <int MODE>
__global__ void k_floor(set s, uint32_t n)
{
	const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
	if (MODE == 0 || i >= n)
		return;
	u32x4 r = {i, 0u, 0u, 0u};
	if (MODE >= 2)
		r.y = s.off[i];
	if (MODE >= 3) {
		const uint32_t l = s.len[i];
		const u32x4 *w = (const u32x4 *)(s.frames + (r.y & ~15u));
		r ^= w[0];
		if (MODE >= 4) {
			r ^= w[1];
			r ^= w[2];
			r ^= w[3];
			r ^= w[4];
		}
		r.w += l;
	}
	__builtin_nontemporal_store(r, &s.out[i]);
}

// the same launches back to back between one event pair: per-launch cost when dispatches overlap
template <int MODE>
static int b2b(const std::vector<set> &sets, uint32_t n, uint32_t wg, int iters, double *avg)
{
	hipEvent_t a, b;
	CHK(hipEventCreate(&a));
	CHK(hipEventCreate(&b));
	CHK(hipEventRecord(a, 0));
	for (int i = 0; i < iters; i++)
		hipLaunchKernelGGL(k_floor<MODE>, dim3((n + wg - 1) / wg), dim3(wg), 0, 0, sets[(size_t)i * 7 % sets.size()], n);
	CHK(hipEventRecord(b, 0));
	CHK(hipEventSynchronize(b));
	float ms;
	CHK(hipEventElapsedTime(&ms, a, b));
	*avg = ms * 1e3 / iters;
	CHK(hipEventDestroy(a));
	CHK(hipEventDestroy(b));
	return 0;
}

template <int MODE>
static int timed(const std::vector<set> &sets, uint32_t n, uint32_t wg, int iters, double *med)
{
	std::vector<hipEvent_t> e0(iters), e1(iters);
	for (int i = 0; i < iters; i++) {
		CHK(hipEventCreate(&e0[i]));
		CHK(hipEventCreate(&e1[i]));
	}
	for (int i = 0; i < iters; i++)
		hipExtLaunchKernelGGL(k_floor<MODE>, dim3((n + wg - 1) / wg), dim3(wg), 0, 0, e0[i], e1[i], 0,
		                      sets[(size_t)i * 7 % sets.size()], n);
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

static int lib_launch(const mosrx_kparams &kp, hipEvent_t a, hipEvent_t b)
{
	const uint32_t tiles = (kp.n + MOSRX_SMALL_FRAMES - 1) / MOSRX_SMALL_FRAMES;
	if (a)
		hipExtLaunchKernelGGL((mosrx_classify_kernel<MOSRX_KIND_SMALL, 0>), dim3(tiles), dim3(WG_THREADS(MOSRX_KIND_SMALL)),
		                      0, 0, a, b, 0, kp.off, kp.len, kp.frames, kp.tables, kp.frames_bytes, kp.n, kp.flags, kp);
	else
		hipLaunchKernelGGL((mosrx_classify_kernel<MOSRX_KIND_SMALL, 0>), dim3(tiles), dim3(WG_THREADS(MOSRX_KIND_SMALL)),
		                   0, 0, kp.off, kp.len, kp.frames, kp.tables, kp.frames_bytes, kp.n, kp.flags, kp);
	return 0;
}

static int lib_timed(const std::vector<mosrx_kparams> &kps, int iters, double *med, double *avg)
{
	std::vector<hipEvent_t> e0(iters), e1(iters);
	for (int i = 0; i < iters; i++) {
		CHK(hipEventCreate(&e0[i]));
		CHK(hipEventCreate(&e1[i]));
	}
	for (int i = 0; i < iters; i++)
		lib_launch(kps[(size_t)i * 7 % kps.size()], e0[i], e1[i]);
	CHK(hipDeviceSynchronize());
	std::vector<float> d(iters);
	for (int i = 0; i < iters; i++) {
		CHK(hipEventElapsedTime(&d[i], e0[i], e1[i]));
		CHK(hipEventDestroy(e0[i]));
		CHK(hipEventDestroy(e1[i]));
	}
	std::sort(d.begin(), d.end());
	*med = d[iters / 2] * 1e3;
	hipEvent_t a, b;
	CHK(hipEventCreate(&a));
	CHK(hipEventCreate(&b));
	CHK(hipEventRecord(a, 0));
	for (int i = 0; i < iters; i++)
		lib_launch(kps[(size_t)i * 7 % kps.size()], nullptr, nullptr);
	CHK(hipEventRecord(b, 0));
	CHK(hipEventSynchronize(b));
	float ms;
	CHK(hipEventElapsedTime(&ms, a, b));
	*avg = ms * 1e3 / iters;
	return 0;
}

int main()
{
	const uint32_t n = 32768, stride = 64;
	const int nsets = 512;
	std::vector<uint32_t> off(n);
	std::vector<uint16_t> len(n, 60);
	for (uint32_t i = 0; i < n; i++)
		off[i] = 2 + stride * i;
	std::vector<uint8_t> fr((size_t)n * stride + 64, 0x45);
	std::vector<set> sets(nsets);
	for (int k = 0; k < nsets; k++) {
		uint8_t *f; uint32_t *o; uint16_t *l; u32x4 *r;
		CHK(hipMalloc((void **)&f, fr.size()));
		CHK(hipMemcpy(f, fr.data(), fr.size(), hipMemcpyHostToDevice));
		CHK(hipMalloc((void **)&o, n * 4));
		CHK(hipMemcpy(o, off.data(), n * 4, hipMemcpyHostToDevice));
		CHK(hipMalloc((void **)&l, n * 2));
		CHK(hipMemcpy(l, len.data(), n * 2, hipMemcpyHostToDevice));
		CHK(hipMalloc((void **)&r, n * 16));
		sets[k] = {f, o, l, r};
	}
	// the library's kernel over config #2's trace (S64: 32K frames of 60 B, one flow), as bench row S64_1
	mosrx_trace t;
	if (mosrx_trace_gen(MOSRX_TRACE_S64, n, 1, 0, &t)) {
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
	std::vector<mosrx_kparams> kps(nsets);
	for (int k = 0; k < nsets; k++) {
		uint8_t *f; uint32_t *o; uint16_t *l; mosrx_result *r;
		CHK(hipMalloc((void **)&f, t.frames_bytes + 64));
		CHK(hipMemcpy(f, t.frames, t.frames_bytes + 64, hipMemcpyHostToDevice));
		CHK(hipMalloc((void **)&o, n * 4));
		CHK(hipMemcpy(o, t.off, n * 4, hipMemcpyHostToDevice));
		CHK(hipMalloc((void **)&l, n * 2));
		CHK(hipMemcpy(l, t.len, n * 2, hipMemcpyHostToDevice));
		CHK(hipMalloc((void **)&r, n * 16));
		kps[k] = (mosrx_kparams){f, o, l, r, tables, NULL, NULL, NULL, NULL, (uint32_t)t.frames_bytes, n,
		                         MOSRX_KF_VERIFY};
	}
	static const char *names[5] = {"empty", "store", "desc+store", "chain16", "chain80"};
	printf("%u frames of %u B per launch, %d rotating buffer sets\n", n, stride, nsets);
	for (int rep = 0; rep < 3; rep++) {
		for (uint32_t wg : {256u, 64u})
			for (int m = 0; m < 5; m++) {
				double med = 0, avg = 0;
				int rc = 0;
				switch (m) {
				case 0: rc = timed<0>(sets, n, wg, 400, &med) || b2b<0>(sets, n, wg, 400, &avg); break;
				case 1: rc = timed<1>(sets, n, wg, 400, &med) || b2b<1>(sets, n, wg, 400, &avg); break;
				case 2: rc = timed<2>(sets, n, wg, 400, &med) || b2b<2>(sets, n, wg, 400, &avg); break;
				case 3: rc = timed<3>(sets, n, wg, 400, &med) || b2b<3>(sets, n, wg, 400, &avg); break;
				case 4: rc = timed<4>(sets, n, wg, 400, &med) || b2b<4>(sets, n, wg, 400, &avg); break;
				}
				if (rc)
					return rc;
				printf("rep %d wg %3u %-11s stamped median %6.2f us, back to back %6.2f us per launch\n", rep, wg,
				       names[m], med, avg);
			}
		double med, avg;
		if (lib_timed(kps, 400, &med, &avg))
			return 1;
		printf("rep %d        library     stamped median %6.2f us, back to back %6.2f us per launch\n", rep, med, avg);
	}
	return 0;
}
