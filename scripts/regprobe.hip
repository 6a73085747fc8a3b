// regprobe.hip — register use of stream-tile variants (compile only:
// hipcc -c -Rpass-analysis=kernel-resource-usage).  Diagnostic, not shipped.
#include "../mos-networking-stack_amd/csrc/mosrx_kernels.hip"

template <int S, int DBG, int W = 6, int U = 8>
__global__ __launch_bounds__(64 * (1 + S)) __attribute__((amdgpu_waves_per_eu(W))) void k_sdbg(mosrx_kparams kp)
{
	classify_tile_stream<S, 2, DBG, U>(kp, blockIdx.x);
}
template __global__ void k_sdbg<3, 0, 8, 4>(mosrx_kparams);
template __global__ void k_sdbg<4, 0, 8, 4>(mosrx_kparams);
template __global__ void k_sdbg<2, 0, 8, 4>(mosrx_kparams);
template __global__ void k_sdbg<3, 0, 8, 8>(mosrx_kparams);
template __global__ void k_sdbg<3, 0, 1, 4>(mosrx_kparams);
