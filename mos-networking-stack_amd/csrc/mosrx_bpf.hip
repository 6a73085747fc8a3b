// mosrx_bpf.hip — batched classic-BPF evaluation on gfx950.
//
// mOS runs sfbpf_filter (bpf/sf_bpf_filter.c:214-536) per frame for every
// raw-monitor filter (ip_in.c:56-63) and stream SYN / orphan filter
// (tcp.c:42-56, 486-496).  Here one launch evaluates up to 32 programs over a
// batch, one lane per frame, and writes a match bitmask per frame.
//
// SIMT without divergence: every program accepted by mosrx_bpf_set jumps only
// forward, so a lane's program counter only grows.  The wave walks the
// instructions once in order with a UNIFORM index i; the instruction comes in
// through scalar loads, its opcode switch is a scalar branch, and the lanes
// whose own pc equals i execute it under the exec mask.  Instructions no lane
// sits on are skipped with one ballot; the walk ends when every lane returned.
// Scratch memory M[16] lives in registers: its index is the instruction's k,
// uniform, so a load/store is a uniform compare chain of v_cndmask.
//
// Packet loads: every lane first stages its frame's first STAGE_B bytes in LDS
// with one burst of 16-byte loads (one memory latency per frame instead of one
// per filter load); a load inside that window is two LDS reads + v_alignbyte,
// a deeper one goes to HBM/L2 through the batch buffer resource.  Bounds are
// checked against buflen exactly as the reference does first.

#include <errno.h>
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include "mosrx_device.h"

#define BPF_TILE 256u
#define BPF_DONE 0xFFFFFFFFu
#define STAGE_V  9u                 // 16-byte loads per frame: bytes [o & ~3, +144)
#define STAGE_DW (4u * STAGE_V)     // staged dwords per frame
#define STAGE_LD (STAGE_DW + 1u)    // LDS stride per lane (odd: conflict-free columns)
#define STAGE_B  (4u * STAGE_DW - 3u) // frame bytes guaranteed staged: [0, 141)

// opcode fields (include/bpf/sfbpf.h)
enum : uint32_t {
	B_LD = 0, B_LDX = 1, B_ST = 2, B_STX = 3, B_ALU = 4, B_JMP = 5, B_RET = 6, B_MISC = 7,
	B_W = 0, B_H = 8, B_B = 0x10,
	B_IMM = 0, B_ABS = 0x20, B_IND = 0x40, B_MEM = 0x60, B_LEN = 0x80, B_MSH = 0xa0,
	B_ADD = 0, B_SUB = 0x10, B_MUL = 0x20, B_DIV = 0x30, B_OR = 0x40, B_AND = 0x50, B_LSH = 0x60,
	B_RSH = 0x70, B_NEG = 0x80,
	B_JA = 0, B_JEQ = 0x10, B_JGT = 0x20, B_JGE = 0x30, B_JSET = 0x40,
	B_K = 0, B_X = 8, B_A = 0x10, B_TAX = 0, B_TXA = 0x80,
};

// Little-endian dword of buffer bytes [a, a+4); a may be unaligned.
__device__ __forceinline__ uint32_t ld_le32(__amdgpu_buffer_rsrc_t rs, uint32_t a)
{
	const uint32_t a4 = a & ~3u;
	const uint32_t lo = __builtin_amdgcn_raw_buffer_load_b32(rs, a4, 0, 0);
	const uint32_t hi = __builtin_amdgcn_raw_buffer_load_b32(rs, a4 + 4u, 0, 0);
	return __builtin_amdgcn_alignbyte(hi, lo, a & 3u);
}
// Little-endian dword of frame bytes [k, k+4) (k + 4 <= STAGE_B + 3 staged):
// from the lane's LDS window when inside it, else from memory.
__device__ __forceinline__ uint32_t fr_le32(const uint32_t *win, uint32_t sh, __amdgpu_buffer_rsrc_t rs,
                                            uint32_t o, uint32_t k, uint32_t size)
{
	if (k + size <= STAGE_B) {
		const uint32_t a = sh + k;
		return __builtin_amdgcn_alignbyte(win[(a >> 2) + 1u], win[a >> 2], a & 3u);
	}
	return ld_le32(rs, o + k);
}

// M[k] with k uniform (< 16, checked at set)
__device__ __forceinline__ uint32_t mem_get(const uint32_t (&M)[16], uint32_t k)
{
	uint32_t r = 0;
#pragma unroll
	for (uint32_t q = 0; q < 16; q++)
		r = (k == q) ? M[q] : r;
	return r;
}
__device__ __forceinline__ void mem_put(uint32_t (&M)[16], uint32_t k, uint32_t v)
{
#pragma unroll
	for (uint32_t q = 0; q < 16; q++)
		M[q] = (k == q) ? v : M[q];
}

__device__ __forceinline__ uint32_t be32(uint32_t le) { return __builtin_bswap32(le); }
__device__ __forceinline__ uint32_t be16(uint32_t le) { return ((le & 0xFFu) << 8) | ((le >> 8) & 0xFFu); }

__global__ __launch_bounds__(BPF_TILE) void mosrx_bpf_kernel(const mosrx_bparams bp)
{
	__shared__ uint32_t s_win[STAGE_LD * BPF_TILE];
	const uint32_t t = threadIdx.x;
	const uint32_t p = blockIdx.x * BPF_TILE + t;
	const bool live = p < bp.n;
	const __amdgpu_buffer_rsrc_t rs = frame_rsrc(bp.frames, bp.frames_bytes);

	uint32_t o = 0, cap = 0, lip = 0;
	if (live) {
		o = bp.off[p];
		cap = eff_caplen(o, bp.len[p], bp.frames_bytes);
	}
	// stage bytes [o & ~3, +144) of the frame (out-of-range dwords read 0)
	uint32_t *win = s_win + STAGE_LD * t;
	const uint32_t sh = o & 3u;
	{
		const uint32_t base = live ? (o & ~3u) : bp.frames_bytes + 16u;
		u32x4 v[STAGE_V];
#pragma unroll
		for (uint32_t m = 0; m < STAGE_V; m++)
			v[m] = __builtin_amdgcn_raw_buffer_load_b128(rs, base + 16u * m, 0, 0);
#pragma unroll
		for (uint32_t m = 0; m < STAGE_V; m++) {
			win[4 * m + 0] = v[m].x; win[4 * m + 1] = v[m].y; win[4 * m + 2] = v[m].z; win[4 * m + 3] = v[m].w;
		}
	}
	// datagram length for the SYN/orphan call sites: 14 + tot_len of an IPv4
	// frame whose datagram lies inside the capture
	if (cap >= 18u && (fr_le32(win, sh, rs, o, 12u, 2u) & 0xFFFFu) == 0x0008u) {
		lip = 14u + be16(fr_le32(win, sh, rs, o, 16u, 2u));
		if (lip > cap)
			lip = 0;
	}

	uint32_t match = 0;
	for (uint32_t j = 0; j < bp.nprog; j++) {
		const bool ipm = (bp.ip_mode >> j) & 1u;
		const uint32_t L = ipm ? lip : cap;
		const bool act = live && (!ipm || lip != 0u);
		const uint32_t plen = bp.prog_len[j];
		if (plen == 0) {                       // no filter: sfbpf_filter(NULL) = ~0
			match |= act ? (1u << j) : 0u;
			continue;
		}
		const uint2 *prog = reinterpret_cast<const uint2 *>(bp.insns + bp.prog_off[j]);
		uint32_t pc = act ? 0u : BPF_DONE, A = 0, X = 0, ret = 0;
		uint32_t M[16];
#pragma unroll
		for (int q = 0; q < 16; q++)
			M[q] = 0;
		for (uint32_t i = 0; i < plen; i++) {
			if (__ballot(pc == i) == 0) {
				if (__ballot(pc != BPF_DONE) == 0)
					break;
				continue;
			}
			const uint2 w = prog[i];                               // scalar load
			const uint32_t code = w.x & 0xFFFFu, jt = (w.x >> 16) & 0xFFu, jf = w.x >> 24, k = w.y;
			const bool e = (pc == i);
			uint32_t npc = i + 1u;
			bool oob = false;                                      // bounds check failed: return 0
			switch (code) {
			case B_RET | B_K: ret = e ? k : ret; npc = BPF_DONE; break;
			case B_RET | B_A: ret = e ? A : ret; npc = BPF_DONE; break;
			case B_LD | B_W | B_ABS:
				oob = (uint64_t)k + 4u > L;
				if (e && !oob) A = be32(fr_le32(win, sh, rs, o, k, 4u));
				break;
			case B_LD | B_H | B_ABS:
				oob = (uint64_t)k + 2u > L;
				if (e && !oob) A = be16(fr_le32(win, sh, rs, o, k, 2u));
				break;
			case B_LD | B_B | B_ABS:
				oob = k >= L;
				if (e && !oob) A = fr_le32(win, sh, rs, o, k, 1u) & 0xFFu;
				break;
			case B_LD | B_W | B_LEN: if (e) A = L; break;
			case B_LDX | B_W | B_LEN: if (e) X = L; break;
			case B_LD | B_W | B_IND: {
				const uint32_t kk = X + k;
				oob = (uint64_t)kk + 4u > L;
				if (e && !oob) A = be32(fr_le32(win, sh, rs, o, kk, 4u));
				break;
			}
			case B_LD | B_H | B_IND: {
				const uint32_t kk = X + k;
				oob = (uint64_t)kk + 2u > L;
				if (e && !oob) A = be16(fr_le32(win, sh, rs, o, kk, 2u));
				break;
			}
			case B_LD | B_B | B_IND: {
				const uint32_t kk = X + k;
				oob = kk >= L;
				if (e && !oob) A = fr_le32(win, sh, rs, o, kk, 1u) & 0xFFu;
				break;
			}
			case B_LDX | B_MSH | B_B:
				oob = k >= L;
				if (e && !oob) X = (fr_le32(win, sh, rs, o, k, 1u) & 0xFu) << 2;
				break;
			case B_LD | B_IMM: if (e) A = k; break;
			case B_LDX | B_IMM: if (e) X = k; break;
			case B_LD | B_MEM: if (e) A = mem_get(M, k); break;
			case B_LDX | B_MEM: if (e) X = mem_get(M, k); break;
			case B_ST: if (e) mem_put(M, k, A); break;
			case B_STX: if (e) mem_put(M, k, X); break;
			case B_JMP | B_JA: npc = i + 1u + k; break;
			case B_JMP | B_JGT | B_K: npc = i + 1u + ((A > k) ? jt : jf); break;
			case B_JMP | B_JGE | B_K: npc = i + 1u + ((A >= k) ? jt : jf); break;
			case B_JMP | B_JEQ | B_K: npc = i + 1u + ((A == k) ? jt : jf); break;
			case B_JMP | B_JSET | B_K: npc = i + 1u + ((A & k) ? jt : jf); break;
			case B_JMP | B_JGT | B_X: npc = i + 1u + ((A > X) ? jt : jf); break;
			case B_JMP | B_JGE | B_X: npc = i + 1u + ((A >= X) ? jt : jf); break;
			case B_JMP | B_JEQ | B_X: npc = i + 1u + ((A == X) ? jt : jf); break;
			case B_JMP | B_JSET | B_X: npc = i + 1u + ((A & X) ? jt : jf); break;
			case B_ALU | B_ADD | B_X: if (e) A += X; break;
			case B_ALU | B_SUB | B_X: if (e) A -= X; break;
			case B_ALU | B_MUL | B_X: if (e) A *= X; break;
			case B_ALU | B_DIV | B_X:
				oob = (X == 0u);                              // division by X == 0 returns 0
				if (e && !oob) A /= X;
				break;
			case B_ALU | B_AND | B_X: if (e) A &= X; break;
			case B_ALU | B_OR | B_X: if (e) A |= X; break;
			case B_ALU | B_LSH | B_X: if (e) A <<= (X & 31u); break;   // x86 shift semantics
			case B_ALU | B_RSH | B_X: if (e) A >>= (X & 31u); break;
			case B_ALU | B_ADD | B_K: if (e) A += k; break;
			case B_ALU | B_SUB | B_K: if (e) A -= k; break;
			case B_ALU | B_MUL | B_K: if (e) A *= k; break;
			case B_ALU | B_DIV | B_K: if (e) A /= k; break;           // k != 0 (mosrx_bpf_set)
			case B_ALU | B_AND | B_K: if (e) A &= k; break;
			case B_ALU | B_OR | B_K: if (e) A |= k; break;
			case B_ALU | B_LSH | B_K: if (e) A <<= (k & 31u); break;
			case B_ALU | B_RSH | B_K: if (e) A >>= (k & 31u); break;
			case B_ALU | B_NEG: if (e) A = 0u - A; break;
			case B_MISC | B_TAX: if (e) X = A; break;
			case B_MISC | B_TXA: if (e) A = X; break;
			default: oob = true; break;                               // rejected at set
			}
			if (e) {
				if (oob) {
					ret = 0;
					npc = BPF_DONE;
				}
				pc = npc;
			}
		}
		match |= ret ? (1u << j) : 0u;
	}
	if (live)
		bp.match[p] = match;
}

extern "C" int mosrx_launch_bpf(const mosrx_bparams *bp, void *stream)
{
	if (!bp || bp->n == 0)
		return bp ? 0 : -EINVAL;
	if (bp->nprog > MOSRX_BPF_MAX_PROGS)
		return -EINVAL;
	const uint32_t grid = (bp->n + BPF_TILE - 1u) / BPF_TILE;
	void *e0, *e1;
	if (mosrx__stamp_take(&e0, &e1))   // dispatch-stamped timing (mosrx_time_op_dispatch)
		hipExtLaunchKernelGGL(mosrx_bpf_kernel, dim3(grid), dim3(BPF_TILE), 0, (hipStream_t)stream,
		                      (hipEvent_t)e0, (hipEvent_t)e1, 0, *bp);
	else
		hipLaunchKernelGGL(mosrx_bpf_kernel, dim3(grid), dim3(BPF_TILE), 0, (hipStream_t)stream, *bp);
	return hipGetLastError() == hipSuccess ? 0 : -EIO;
}
