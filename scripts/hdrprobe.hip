// hdrprobe.hip — VERDICT r5 next #5: is the standalone BPF kernel's 1.79x
// HBM traffic real, and what scale does FETCH_SIZE need for its access shape
// (one short header window per lane, at frame stride)?  Byte-known kernels on
// the bench's IMIX layout (60 / 590 / 1514 B frames 7:4:1, each at a 16-byte
// boundary + 2, 256K frames per batch, 12 batches cycled so no launch is
// served by the 256 MiB Infinity Cache), each reading off[] (4 B per frame)
// and writing one u32 per frame:
//   win80   5 x 16-byte loads per lane from off & ~3: the JIT's staging of the
//           bench's 8 programs (STAGE_V 5, bpf_jit.c stage_pieces)
//   sec64   4 x 16-byte loads per lane from off & ~63: one 64-byte sector
//   stream  16 bytes per lane, contiguous, over the batch's frame bytes (the
//           guide's calibrated shape: FETCH_SIZE reads 1/2 of the bytes)
// The host prints, per kernel, the distinct 64-byte sectors its loads touch
// (the bytes HBM must deliver at 64-byte granularity); rocprofv3 --pmc
// FETCH_SIZE / WRITE_SIZE runs of this program give what the counters say.
//   hipcc --offload-arch=gfx950 -O3 scripts/hdrprobe.hip -o scripts/hdrprobe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <algorithm>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

struct u4 { uint32_t x, y, z, w; };

__global__ __launch_bounds__(256) void win80(const uint8_t *fr, const uint32_t *off, uint32_t n, uint32_t *out)
{
	const uint32_t i = blockIdx.x * 256u + threadIdx.x;
	if (i >= n) return;
	const uint4 *p = (const uint4 *)(fr + (off[i] & ~3u));
	uint32_t s = 0;
#pragma unroll
	for (int m = 0; m < 5; m++) { const uint4 v = p[m]; s += v.x ^ v.y ^ v.z ^ v.w; }
	out[i] = s;
}

__global__ __launch_bounds__(256) void sec64(const uint8_t *fr, const uint32_t *off, uint32_t n, uint32_t *out)
{
	const uint32_t i = blockIdx.x * 256u + threadIdx.x;
	if (i >= n) return;
	const uint4 *p = (const uint4 *)(fr + (off[i] & ~63u));
	uint32_t s = 0;
#pragma unroll
	for (int m = 0; m < 4; m++) { const uint4 v = p[m]; s += v.x ^ v.y ^ v.z ^ v.w; }
	out[i] = s;
}

__global__ __launch_bounds__(256) void stream(const uint4 *fr, uint64_t n16, const uint32_t *off, uint32_t n,
                                              uint32_t *out)
{
	const uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x;
	uint32_t s = 0;
	for (uint64_t j = i; j < n16; j += (uint64_t)gridDim.x * 256u) { const uint4 v = fr[j]; s += v.x ^ v.y ^ v.z ^ v.w; }
	if (i < n) out[i] = s + off[i];
}

static uint64_t sectors(const std::vector<uint32_t> &off, uint32_t mask, uint32_t bytes)
{
	std::vector<uint64_t> s;
	s.reserve(off.size() * 3);
	for (uint32_t o : off) {
		const uint64_t a = o & mask;
		for (uint64_t x = a & ~63ull; x < a + bytes; x += 64) s.push_back(x);
	}
	std::sort(s.begin(), s.end());
	return (uint64_t)(std::unique(s.begin(), s.end()) - s.begin());
}

int main(int argc, char **argv)
{
	const uint32_t n = 262144, nbuf = 12, iters = argc > 1 ? atoi(argv[1]) : 24;
	const uint32_t cap[3] = {60, 590, 1514};
	std::vector<uint32_t> off(n);
	uint64_t pos = 2, seed = 12345;
	std::vector<uint8_t> cls(n);
	for (uint32_t i = 0; i < n; i += 12) {    // 7 x 60, 4 x 590, 1 x 1514 per 12, shuffled
		uint8_t g[12] = {0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2};
		for (int k = 11; k > 0; k--) {
			seed = seed * 6364136223846793005ull + 1442695040888963407ull;
			const int j = (int)((seed >> 33) % (uint64_t)(k + 1));
			std::swap(g[k], g[j]);
		}
		for (int k = 0; k < 12 && i + k < n; k++) cls[i + k] = g[k];
	}
	for (uint32_t i = 0; i < n; i++) {
		off[i] = (uint32_t)pos;
		pos = ((pos + cap[cls[i]] - 2 + 15) & ~15ull) + 2;
	}
	const uint64_t fb = (pos + 255) & ~255ull;
	std::vector<uint8_t> h(fb);
	for (uint64_t i = 0; i < fb; i++) h[i] = (uint8_t)(i * 2654435761u >> 13);
	uint8_t *d_fr[nbuf];
	uint32_t *d_off, *d_out;
	for (uint32_t b = 0; b < nbuf; b++) {
		CK(hipMalloc(&d_fr[b], fb + 256));
		CK(hipMemcpy(d_fr[b], h.data(), fb, hipMemcpyHostToDevice));
	}
	CK(hipMalloc(&d_off, n * 4));
	CK(hipMalloc(&d_out, n * 4));
	CK(hipMemcpy(d_off, off.data(), n * 4, hipMemcpyHostToDevice));
	const uint64_t s80 = sectors(off, ~3u, 80), s64 = sectors(off, ~63u, 64);
	printf("frames %u, frame bytes %llu per batch\n", n, (unsigned long long)fb);
	printf("win80: distinct 64-B sectors %llu = %.2f MB (+ off %.2f MB); algorithmic 64-B headers %.2f MB\n",
	       (unsigned long long)s80, s80 * 64 / 1e6, n * 4 / 1e6, n * 64 / 1e6);
	printf("sec64: distinct 64-B sectors %llu = %.2f MB (+ off %.2f MB)\n", (unsigned long long)s64, s64 * 64 / 1e6,
	       n * 4 / 1e6);
	printf("stream: %.2f MB (+ off %.2f MB); every kernel writes %.2f MB\n", fb / 1e6, n * 4 / 1e6, n * 4 / 1e6);
	const dim3 g((n + 255) / 256), t(256);
	for (uint32_t i = 0; i < iters; i++) {
		win80<<<g, t>>>(d_fr[i % nbuf], d_off, n, d_out);
		sec64<<<g, t>>>(d_fr[(i + 4) % nbuf], d_off, n, d_out);
		stream<<<2048, t>>>((const uint4 *)d_fr[(i + 8) % nbuf], fb / 16, d_off, n, d_out);
	}
	CK(hipDeviceSynchronize());
	printf("done (%u launches of each)\n", iters);
	return 0;
}
