// mosrx_device.h — device helpers shared by the gfx950 kernels.
#ifndef MOSRX_DEVICE_H
#define MOSRX_DEVICE_H

#ifndef __HIPCC_RTC__
#include <hip/hip_runtime.h>
#endif

#include "mosrx_internal.h"

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// The resource range is frames_bytes rounded up to 16: the 16-byte chunk that
// holds the buffer's last byte is readable whole (it cannot cross a page the
// buffer does not touch), and every byte past the last frame's end is masked.
// Loads at or past the range read zero with no memory traffic; the range check
// is per dword (tested by test_buffer_end_exact on misaligned layouts).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t frame_rsrc(const uint8_t *base, uint32_t nbytes)
{
	return __builtin_amdgcn_make_buffer_rsrc((void *)base, (short)0, (int)((nbytes + 15u) & ~15u), 0x00020000);
}

// Stores of the per-frame outputs (records, side arrays): written once, read
// by the host after the launch.  MOSRX_OUT_AUX (A/B builds) picks the cache
// policy bits of a buffer store instead (gfx950: 1 sc0, 2 nt, 16 sc1).
typedef uint32_t u32x3 __attribute__((ext_vector_type(3)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
// out_store(base, i, v): element i of a per-frame output array (`base` is
// uniform: the kernel's argument).
#ifdef MOSRX_OUT_AUX
__device__ __forceinline__ __amdgpu_buffer_rsrc_t out_rsrc(const void *base)
{
	return __builtin_amdgcn_make_buffer_rsrc((void *)base, (short)0, 0x7FFFFFFF, 0x00020000);
}
__device__ __forceinline__ void out_store(u32x4 *base, uint32_t i, u32x4 v)
{
	__builtin_amdgcn_raw_buffer_store_b128(v, out_rsrc(base), 16u * i, 0, MOSRX_OUT_AUX);
}
__device__ __forceinline__ void out_store(u32x2 *base, uint32_t i, u32x2 v)
{
	__builtin_amdgcn_raw_buffer_store_b64(v, out_rsrc(base), 8u * i, 0, MOSRX_OUT_AUX);
}
__device__ __forceinline__ void out_store(uint32_t *base, uint32_t i, u32x3 v)   // 12-byte elements
{
	__builtin_amdgcn_raw_buffer_store_b96(v, out_rsrc(base), 12u * i, 0, MOSRX_OUT_AUX);
}
__device__ __forceinline__ void out_store(uint32_t *base, uint32_t i, uint32_t v)
{
	__builtin_amdgcn_raw_buffer_store_b32(v, out_rsrc(base), 4u * i, 0, MOSRX_OUT_AUX);
}
#else
__device__ __forceinline__ void out_store(u32x4 *base, uint32_t i, u32x4 v)
{
	__builtin_nontemporal_store(v, base + i);
}
__device__ __forceinline__ void out_store(u32x2 *base, uint32_t i, u32x2 v)
{
	__builtin_nontemporal_store(v, base + i);
}
__device__ __forceinline__ void out_store(uint32_t *base, uint32_t i, u32x3 v)   // 12-byte elements
{
	__builtin_nontemporal_store(v, reinterpret_cast<u32x3 *>(base + 3u * i));
}
__device__ __forceinline__ void out_store(uint32_t *base, uint32_t i, uint32_t v)
{
	__builtin_nontemporal_store(v, base + i);
}
#endif

// Capture length clipped to the batch buffer (a frame never reads past it).
__device__ __forceinline__ uint32_t eff_caplen(uint32_t o, uint32_t len, uint32_t nbytes)
{
	// select form, not a branch: a branch lets the compiler sink the len[]
	// load behind the off[] load (one more round trip before any frame byte)
	return min(len, o < nbytes ? nbytes - o : 0u);
}

#endif
