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
// Scratch memory M[16] lives in LDS (one column per lane, conflict-free).
//
// Packet loads read the frame bytes from HBM/L2 through the batch buffer
// resource (two dword loads + v_alignbyte for an unaligned word), after the
// same bounds checks the reference makes against buflen.

#include <errno.h>

#include "mosrx_device.h"

#define BPF_TILE 256u
#define BPF_DONE 0xFFFFFFFFu

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
__device__ __forceinline__ uint32_t be32(uint32_t le) { return __builtin_bswap32(le); }
__device__ __forceinline__ uint32_t be16(uint32_t le) { return ((le & 0xFFu) << 8) | ((le >> 8) & 0xFFu); }

__global__ __launch_bounds__(BPF_TILE) void mosrx_bpf_kernel(const mosrx_bparams bp)
{
	__shared__ uint32_t s_mem[16 * BPF_TILE];
	const uint32_t t = threadIdx.x;
	const uint32_t p = blockIdx.x * BPF_TILE + t;
	const bool live = p < bp.n;
	const __amdgpu_buffer_rsrc_t rs = frame_rsrc(bp.frames, bp.frames_bytes);

	uint32_t o = 0, cap = 0, lip = 0;
	if (live) {
		o = bp.off[p];
		cap = eff_caplen(o, bp.len[p], bp.frames_bytes);
	}
	// datagram length for the SYN/orphan call sites: 14 + tot_len of an IPv4
	// frame whose datagram lies inside the capture
	if (cap >= 18u && (ld_le32(rs, o + 12u) & 0xFFFFu) == 0x0008u) {
		lip = 14u + be16(ld_le32(rs, o + 16u));
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
		uint32_t pc = act ? 0u : BPF_DONE, A = 0, X = 0, ret = 0, memw = 0;
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
				if (e && !oob) A = be32(ld_le32(rs, o + k));
				break;
			case B_LD | B_H | B_ABS:
				oob = (uint64_t)k + 2u > L;
				if (e && !oob) A = be16(ld_le32(rs, o + k));
				break;
			case B_LD | B_B | B_ABS:
				oob = k >= L;
				if (e && !oob) A = ld_le32(rs, o + k) & 0xFFu;
				break;
			case B_LD | B_W | B_LEN: if (e) A = L; break;
			case B_LDX | B_W | B_LEN: if (e) X = L; break;
			case B_LD | B_W | B_IND: {
				const uint32_t kk = X + k;
				oob = (uint64_t)kk + 4u > L;
				if (e && !oob) A = be32(ld_le32(rs, o + kk));
				break;
			}
			case B_LD | B_H | B_IND: {
				const uint32_t kk = X + k;
				oob = (uint64_t)kk + 2u > L;
				if (e && !oob) A = be16(ld_le32(rs, o + kk));
				break;
			}
			case B_LD | B_B | B_IND: {
				const uint32_t kk = X + k;
				oob = kk >= L;
				if (e && !oob) A = ld_le32(rs, o + kk) & 0xFFu;
				break;
			}
			case B_LDX | B_MSH | B_B:
				oob = k >= L;
				if (e && !oob) X = (ld_le32(rs, o + k) & 0xFu) << 2;
				break;
			case B_LD | B_IMM: if (e) A = k; break;
			case B_LDX | B_IMM: if (e) X = k; break;
			case B_LD | B_MEM: if (e) A = ((memw >> k) & 1u) ? s_mem[k * BPF_TILE + t] : 0u; break;
			case B_LDX | B_MEM: if (e) X = ((memw >> k) & 1u) ? s_mem[k * BPF_TILE + t] : 0u; break;
			case B_ST: if (e) { s_mem[k * BPF_TILE + t] = A; memw |= 1u << k; } break;
			case B_STX: if (e) { s_mem[k * BPF_TILE + t] = X; memw |= 1u << k; } break;
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
	hipLaunchKernelGGL(mosrx_bpf_kernel, dim3(grid), dim3(BPF_TILE), 0, (hipStream_t)stream, *bp);
	return hipGetLastError() == hipSuccess ? 0 : -EIO;
}
