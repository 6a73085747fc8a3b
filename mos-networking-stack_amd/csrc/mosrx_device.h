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

// Capture length clipped to the batch buffer (a frame never reads past it).
__device__ __forceinline__ uint32_t eff_caplen(uint32_t o, uint32_t len, uint32_t nbytes)
{
	// select form, not a branch: a branch lets the compiler sink the len[]
	// load behind the off[] load (one more round trip before any frame byte)
	return min(len, o < nbytes ? nbytes - o : 0u);
}

#endif
