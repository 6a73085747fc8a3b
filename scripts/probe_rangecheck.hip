// probe_rangecheck.hip — how gfx950 range-checks a raw buffer_load_dwordx4 that
// straddles num_records (whole load zeroed, or dword by dword?).  Diagnostic
// only; the answer decides how the classify kernel bounds its window loads.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__global__ void probe(const uint8_t *buf, uint32_t nrec, uint32_t *out)
{
	__amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void *)buf, (short)0, (int)nrec, 0x00020000);
	const uint32_t off = threadIdx.x * 4;   // offsets 0,4,...,60
	u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0);
	out[threadIdx.x * 4 + 0] = v.x;
	out[threadIdx.x * 4 + 1] = v.y;
	out[threadIdx.x * 4 + 2] = v.z;
	out[threadIdx.x * 4 + 3] = v.w;
}

int main()
{
	uint8_t h[256];
	for (int i = 0; i < 256; i++)
		h[i] = (uint8_t)(i + 1);
	uint8_t *d;
	uint32_t *o, ho[64];
	hipMalloc(&d, 256);
	hipMalloc(&o, 256);
	hipMemcpy(d, h, 256, hipMemcpyHostToDevice);
	for (uint32_t nrec : {48u, 50u}) {
		hipLaunchKernelGGL(probe, dim3(1), dim3(16), 0, 0, d, nrec, o);
		hipMemcpy(ho, o, 256, hipMemcpyDeviceToHost);
		printf("num_records=%u\n", nrec);
		for (int l = 8; l < 14; l++)
			printf("  load@%2d: %08x %08x %08x %08x\n", l * 4, ho[4 * l], ho[4 * l + 1], ho[4 * l + 2], ho[4 * l + 3]);
	}
	return 0;
}
