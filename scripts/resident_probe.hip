// resident_probe.hip — diagnostic for DESIGN §7 #6: how fast can a resident
// kernel turn a small group around when the host posts it through pinned
// memory, against a launch + event wait per group?  One workgroup of 256
// lanes reads 256 x 64-byte frames from pinned host memory (one 16-byte load
// per lane from each of 4 frames... here: lane i reads frame i's first 64
// bytes), folds them and writes one u32 per frame back to pinned memory.
//   resident: the kernel polls a posted sequence number (system-scope
//             acquire load, s_sleep between polls), does the group, writes
//             the results, then publishes `done` (system-scope release store);
//             it leaves on a stop word, after 20000 groups, or after 2 s of
//             wall clock (s_memrealtime, 100 MHz) whatever the host does
//   launch:   the same work as one launch per group + hipEventSynchronize
// Prints the median and p99 host round trip (post -> done seen) of each.
//   hipcc --offload-arch=gfx950 -O3 scripts/resident_probe.hip -o scripts/resident_probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <algorithm>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

#define NFR 256
#define STOP 0xFFFFFFFFu
#define MAX_GROUPS 20000u
#define MAX_TICKS (2u * 100000000u)   // 2 s at 100 MHz

__device__ __forceinline__ uint32_t fold(const uint4 *p)
{
	uint32_t s = 0;
#pragma unroll
	for (int m = 0; m < 4; m++) {
		const uint4 v = p[m];
		s += v.x ^ v.y ^ v.z ^ v.w;
	}
	return s;
}

__global__ __launch_bounds__(256) void group_once(const uint8_t *frames, uint32_t *out, uint32_t seq)
{
	const uint32_t i = threadIdx.x;
	out[i] = fold(reinterpret_cast<const uint4 *>(frames + 64u * i)) + seq;
}

__global__ __launch_bounds__(256) void resident(const uint8_t *frames, uint32_t *out, uint32_t *post, uint32_t *done)
{
	__shared__ uint32_t s_seq;
	const uint32_t i = threadIdx.x;
	const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
	uint32_t last = 0, groups = 0;
	for (;;) {
		if (i == 0) {
			uint32_t v;
			for (;;) {
				v = __hip_atomic_load(post, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
				if (v != last || __builtin_amdgcn_s_memrealtime() - t0 > MAX_TICKS)
					break;
				__builtin_amdgcn_s_sleep(1);
			}
			s_seq = (v != last) ? v : STOP;   // timed out: leave
		}
		__syncthreads();
		const uint32_t seq = s_seq;
		__syncthreads();
		if (seq == STOP || ++groups > MAX_GROUPS)
			break;
		out[i] = fold(reinterpret_cast<const uint4 *>(frames + 64u * i)) + seq;
		__threadfence_system();
		__syncthreads();
		if (i == 0)
			__hip_atomic_store(done, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
		last = seq;
	}
}

static double now_us()
{
	timespec t;
	clock_gettime(CLOCK_MONOTONIC, &t);
	return t.tv_sec * 1e6 + t.tv_nsec * 1e-3;
}

static void report(const char *name, std::vector<double> &v)
{
	std::sort(v.begin(), v.end());
	printf("%s: n=%zu median %.2f us, p99 %.2f us\n", name, v.size(), v[v.size() / 2], v[v.size() * 99 / 100]);
}

int main()
{
	uint8_t *h_fr;
	uint32_t *h_out, *h_post, *h_done;
	CK(hipHostMalloc((void **)&h_fr, NFR * 64, hipHostMallocDefault));
	CK(hipHostMalloc((void **)&h_out, NFR * 4, hipHostMallocDefault));
	CK(hipHostMalloc((void **)&h_post, 64, hipHostMallocDefault));
	CK(hipHostMalloc((void **)&h_done, 64, hipHostMallocDefault));
	for (int i = 0; i < NFR * 64; i++)
		h_fr[i] = (uint8_t)(i * 131u);
	*h_post = 0;
	*h_done = 0;
	void *d_fr, *d_out, *d_post, *d_done;
	CK(hipHostGetDevicePointer(&d_fr, h_fr, 0));
	CK(hipHostGetDevicePointer(&d_out, h_out, 0));
	CK(hipHostGetDevicePointer(&d_post, h_post, 0));
	CK(hipHostGetDevicePointer(&d_done, h_done, 0));
	uint32_t expect[NFR];
	for (int i = 0; i < NFR; i++) {
		uint32_t s = 0;
		const uint32_t *w = reinterpret_cast<const uint32_t *>(h_fr + 64 * i);
		for (int m = 0; m < 4; m++)
			s += w[4 * m] ^ w[4 * m + 1] ^ w[4 * m + 2] ^ w[4 * m + 3];
		expect[i] = s;
	}
	hipStream_t st;
	CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
	hipEvent_t ev;
	CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
	// launch per group
	std::vector<double> rt;
	int bad = 0;
	for (uint32_t g = 1; g <= 3000; g++) {
		const double t = now_us();
		hipLaunchKernelGGL(group_once, dim3(1), dim3(256), 0, st, (const uint8_t *)d_fr, (uint32_t *)d_out, g);
		CK(hipEventRecord(ev, st));
		CK(hipEventSynchronize(ev));
		const double dt = now_us() - t;
		if (g > 200)
			rt.push_back(dt);
		bad += h_out[g % NFR] != expect[g % NFR] + g;
	}
	report("launch + event wait per group", rt);
	// resident
	rt.clear();
	hipLaunchKernelGGL(resident, dim3(1), dim3(256), 0, st, (const uint8_t *)d_fr, (uint32_t *)d_out,
	                   (uint32_t *)d_post, (uint32_t *)d_done);
	int timeouts = 0;
	for (uint32_t g = 1; g <= 5000 && !timeouts; g++) {
		const double t = now_us();
		__atomic_store_n(h_post, g, __ATOMIC_RELEASE);
		while (__atomic_load_n(h_done, __ATOMIC_ACQUIRE) != g)
			if (now_us() - t > 100000.0) {   // 100 ms: the kernel never saw the post
				timeouts++;
				break;
			}
		const double dt = now_us() - t;
		if (g > 200 && !timeouts)
			rt.push_back(dt);
		bad += !timeouts && h_out[g % NFR] != expect[g % NFR] + g;
	}
	__atomic_store_n(h_post, STOP, __ATOMIC_RELEASE);
	CK(hipStreamSynchronize(st));   // the kernel leaves on STOP, or by itself within 2 s
	if (!rt.empty())
		report("resident kernel, pinned doorbell", rt);
	printf("wrong results %d, timeouts %d\n", bad, timeouts);
	return bad || timeouts;
}
