// probe_small_align.hip -- the SMALL tile's window loads on config #2's layout
// (diagnostic only, not the library).  Mechanism under test: the alignment of
// the per-lane 16-byte window loads.  The library loads each lane's window
// from the 4-byte-aligned address (off + 2) & ~3 (no realignment for frames at
// 2 mod 4); on a 64-byte-strided layout one of its five loads then straddles a
// 64-byte line.  Loads from off & ~15 never straddle (realigned in registers).
// Pure-read kernels over 8M frames of 60 B at a 64 B stride (start 2), each lane
// XOR-folding its window and writing an 8-byte record, as the compact ring:
//   0  lane per frame, 5 loads at (off + 2) & ~3       (the library's addresses)
//   1  lane per frame, 5 loads at off & ~15            (16-byte aligned)
//   2  lane per frame, 6 loads at off & ~15            (what a general layout needs)
//   3  wave per 64 frames, 5 contiguous 1 KiB loads     (coalesced: a bound)
// Launches of each mode alternate over two resident copies (past the 256 MiB
// Infinity Cache); per mode the median of 30 event-timed launches.
//
//   hipcc -O3 --offload-arch=gfx950 -o scripts/probe_small_align scripts/probe_small_align.hip
#include <hip/hip_runtime.h>
#include <algorithm>
#include <stdint.h>
#include <stdio.h>
#include <vector>

#define CHK(x) do { if ((x) != hipSuccess) { printf("HIP error %s line %d\n", #x, __LINE__); return 1; } } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ u32x4 ld(__amdgpu_buffer_rsrc_t r, uint32_t c)
{
	return __builtin_amdgcn_raw_buffer_load_b128(r, c, 0, 0);
}

template <int MODE>
__global__ __launch_bounds__(256) void k_win(const uint8_t *frames, uint32_t nbytes, const uint32_t *off,
                                             const uint16_t *len, u32x2 *out, uint32_t n)
{
	const uint32_t p = blockIdx.x * 256u + threadIdx.x, lane = threadIdx.x & 63u;
	const __amdgpu_buffer_rsrc_t rs =
	    __builtin_amdgcn_make_buffer_rsrc((void *)frames, (short)0, (int)((nbytes + 15u) & ~15u), 0x00020000);
	const uint32_t q = min(p, n - 1u);
	const uint32_t o = off[q];
	uint32_t l = len[q];
	asm volatile("" : "+v"(l));
	u32x4 x = {0, 0, 0, 0};
	if constexpr (MODE == 0) {
		const uint32_t b = (o + 2u) & ~3u;
#pragma unroll
		for (int m = 0; m < 5; m++)
			x ^= ld(rs, b + 16u * m);
	} else if constexpr (MODE == 1 || MODE == 2) {
		const uint32_t b = o & ~15u;
#pragma unroll
		for (int m = 0; m < (MODE == 1 ? 5 : 6); m++)
			x ^= ld(rs, b + 16u * m);
		// the realignment the library would do (v_alignbyte by the frame's phase)
		const uint32_t sh = (o & 3u) * 8u;
		x.x = __builtin_amdgcn_alignbyte(x.y, x.x, sh);
		x.y = __builtin_amdgcn_alignbyte(x.z, x.y, sh);
		x.z = __builtin_amdgcn_alignbyte(x.w, x.z, sh);
	} else {
		const uint32_t b = __builtin_amdgcn_readfirstlane(o) & ~15u;
#pragma unroll
		for (int m = 0; m < 5; m++)
			x ^= ld(rs, b + 1024u * m + 16u * lane);
	}
	if (p < n)
		__builtin_nontemporal_store((u32x2){x.x ^ x.y ^ x.z ^ x.w, l}, &out[p]);
}

template <int MODE>
static int run(const std::vector<const uint8_t *> &fr, const std::vector<const uint32_t *> &off,
               const std::vector<const uint16_t *> &len, const std::vector<u32x2 *> &out, uint32_t nbytes, uint32_t n,
               int i, float *ms)
{
	hipEvent_t a, b;
	CHK(hipEventCreate(&a));
	CHK(hipEventCreate(&b));
	const size_t s = (size_t)i % fr.size();
	CHK(hipEventRecord(a, 0));
	hipLaunchKernelGGL(k_win<MODE>, dim3((n + 255) / 256), dim3(256), 0, 0, fr[s], nbytes, off[s], len[s], out[s], n);
	CHK(hipEventRecord(b, 0));
	CHK(hipEventSynchronize(b));
	CHK(hipEventElapsedTime(ms, a, b));
	CHK(hipEventDestroy(a));
	CHK(hipEventDestroy(b));
	return 0;
}

int main()
{
	const uint32_t n = 8u << 20, stride = 64, flen = 60;
	const uint32_t nbytes = 2 + stride * n;
	std::vector<uint8_t> h(nbytes + 128);
	uint64_t z = 0x6D4F5321;
	for (auto &c : h) {
		z = z * 6364136223846793005ull + 1442695040888963407ull;
		c = (uint8_t)(z >> 56);
	}
	std::vector<uint32_t> ho(n);
	std::vector<uint16_t> hl(n, flen);
	for (uint32_t i = 0; i < n; i++)
		ho[i] = 2 + stride * i;
	const int NSET = 2;
	std::vector<const uint8_t *> fr;
	std::vector<const uint32_t *> off;
	std::vector<const uint16_t *> len;
	std::vector<u32x2 *> out;
	for (int s = 0; s < NSET; s++) {
		uint8_t *f; uint32_t *o; uint16_t *l; u32x2 *r;
		CHK(hipMalloc(&f, nbytes + 128));
		CHK(hipMalloc(&o, 4ull * n));
		CHK(hipMalloc(&l, 2ull * n));
		CHK(hipMalloc(&r, 8ull * n));
		CHK(hipMemcpy(f, h.data(), nbytes + 128, hipMemcpyHostToDevice));
		CHK(hipMemcpy(o, ho.data(), 4ull * n, hipMemcpyHostToDevice));
		CHK(hipMemcpy(l, hl.data(), 2ull * n, hipMemcpyHostToDevice));
		fr.push_back(f); off.push_back(o); len.push_back(l); out.push_back(r);
	}
	const double algo = (double)n * (flen + 6 + 8);
	const char *names[4] = {"lane, 5 x 16 B at (off+2)&~3 (library)", "lane, 5 x 16 B at off&~15",
	                        "lane, 6 x 16 B at off&~15", "wave, 5 x 1 KiB contiguous (bound)"};
	for (int rep = 0; rep < 3; rep++) {
		std::vector<float> t[4];
		for (int i = 0; i < 40; i++) {   // modes interleaved; the first 10 rounds warm the clocks
			float ms[4];
			if (run<0>(fr, off, len, out, nbytes, n, i, &ms[0]) || run<1>(fr, off, len, out, nbytes, n, i, &ms[1]) ||
			    run<2>(fr, off, len, out, nbytes, n, i, &ms[2]) || run<3>(fr, off, len, out, nbytes, n, i, &ms[3]))
				return 1;
			if (i >= 10)
				for (int m = 0; m < 4; m++)
					t[m].push_back(ms[m]);
		}
		for (int m = 0; m < 4; m++) {
			std::sort(t[m].begin(), t[m].end());
			const double med = t[m][t[m].size() / 2];
			printf("rep %d mode %d %-42s median %8.2f us  %6.0f GB/s of 74 B/frame\n", rep, m, names[m], med * 1e3,
			       algo / (med * 1e-3) / 1e9);
		}
		fflush(stdout);
	}
	return 0;
}
