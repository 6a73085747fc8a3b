// clkprobe.hip — diagnostic: the shader clock a kernel
// runs at right after the GPU idled or after an SDMA copy, against back to
// back.  One workgroup per CU spins a dependent ALU chain between two reads of
// the shader cycle counter (clock64) and the 100 MHz constant clock
// (wall_clock64); cycles / elapsed = the clock the waves saw.
//   hipcc --offload-arch=gfx950 -O2 scripts/clkprobe.hip -o scripts/clkprobe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>
#include <vector>
#include <algorithm>

__global__ void spin(unsigned long long *out, int iters)
{
	unsigned long long c0 = clock64(), r0 = wall_clock64();
	float x = threadIdx.x * 1e-3f;
	for (int i = 0; i < iters; i++)
		x = x * 1.000001f + 1e-7f;
	unsigned long long c1 = clock64(), r1 = wall_clock64();
	if (threadIdx.x == 0) {
		out[blockIdx.x * 3 + 0] = c1 - c0;
		out[blockIdx.x * 3 + 1] = r1 - r0;
		out[blockIdx.x * 3 + 2] = x > 1e30f;
	}
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

static int nblk;
static unsigned long long *d_out, *h_out;

static double mhz(int iters)
{
	spin<<<nblk, 64>>>(d_out, iters);
	CK(hipDeviceSynchronize());
	CK(hipMemcpy(h_out, d_out, nblk * 3 * 8, hipMemcpyDeviceToHost));
	std::vector<double> f;
	for (int b = 0; b < nblk; b++)
		f.push_back((double)h_out[b * 3] / ((double)h_out[b * 3 + 1] / 100.0));   // cycles per us
	std::sort(f.begin(), f.end());
	return f[f.size() / 2];
}

int main()
{
	hipDeviceProp_t p;
	CK(hipGetDeviceProperties(&p, 0));
	nblk = p.multiProcessorCount;
	CK(hipMalloc(&d_out, nblk * 3 * 8));
	CK(hipHostMalloc(&h_out, nblk * 3 * 8, 0));
	const size_t big = 100u << 20;
	void *dbuf, *hbuf;
	CK(hipMalloc(&dbuf, big));
	CK(hipHostMalloc(&hbuf, big, 0));
	memset(hbuf, 1, big);
	const int it = 2000;   // ~ a few us per launch
	for (int i = 0; i < 2000; i++)
		mhz(it);                                       // warm
	double a[6] = {0};
	const int N = 40;
	for (int i = 0; i < N; i++) a[0] += mhz(it) / N;             // back to back
	for (int i = 0; i < N; i++) { usleep(2000); a[1] += mhz(it) / N; }
	for (int i = 0; i < N; i++) { usleep(30000); a[2] += mhz(it) / N; }
	for (int i = 0; i < N; i++) { CK(hipMemcpy(dbuf, hbuf, big, hipMemcpyHostToDevice)); a[3] += mhz(it) / N; }
	for (int i = 0; i < N; i++) {
		CK(hipMemcpy(dbuf, hbuf, big, hipMemcpyHostToDevice));
		usleep(10000);
		a[4] += mhz(it) / N;
	}
	for (int i = 0; i < N; i++) a[5] += mhz(it) / N;             // back to back again
	printf("shader clock MHz (median over %d CUs, mean of %d launches): back-to-back %.0f | after 2 ms idle %.0f | "
	       "after 30 ms idle %.0f | right after a 100 MB H2D copy %.0f | 10 ms after one %.0f | back-to-back %.0f\n",
	       nblk, N, a[0], a[1], a[2], a[3], a[4], a[5]);
	return 0;
}
