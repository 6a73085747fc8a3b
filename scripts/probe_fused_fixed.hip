// probe_fused_fixed.hip — where the fused classify + BPF tile's fixed cost
// comes from (diagnostic only).  The IMIX ring fused with one trivial program
// (`ret #1`) costs ~5 us more than plain classification while its code differs
// by ~40 instructions.  Here both forms of the library's stream
// tile are built by hipcc in one binary, with the trivial set's generated hook
// (scripts/probe_fused/mosrx_bpf_hook.h):
//   plain       classify_tile_stream<3, 0>          (the library's IMIX variant)
//   fused       classify_tile_stream<3, VAR_BPF>    (hook + 4-byte mask per frame)
//   fused, masks not stored (DBG 131072); plain + a constant mask stored (DBG 262144);
//   fused with the masks stored through the cache (DBG 524288)
// one 256K IMIX batch per launch and a ring of 8 batches per launch (the
// batch-queue kernel), dispatch-stamped medians.  If hipcc's fused form costs
// what the hipRTC module does, the cost is the tile's; if not, the module path.
//
//   hipcc -O3 --offload-arch=gfx950 -mllvm -amdgpu-kernarg-preload-count=7 -I scripts/probe_fused \
//     -o scripts/probe_fused_fixed scripts/probe_fused_fixed.hip -Lmos-networking-stack_amd -lmosrx \
//     -Wl,-rpath,'$ORIGIN/../mos-networking-stack_amd'
#define MOSRX_RTC_BPF 1
#include "../mos-networking-stack_amd/csrc/mosrx_kernels.hip"
#include "../include/mosrx_trace.h"
#include <algorithm>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <vector>

#define CHK(x) do { if ((x) != hipSuccess) { printf("HIP error %s line %d\n", #x, __LINE__); return 1; } } while (0)
#define S 3
#define WG (64 * (1 + S))

__global__ __launch_bounds__(WG) __attribute__((amdgpu_waves_per_eu(8))) void k_plain(mosrx_kparams kp)
{
	classify_tile_stream<S, 0>(kp, blockIdx.x);
}

__global__ __launch_bounds__(WG) __attribute__((amdgpu_waves_per_eu(8))) void k_fused(mosrx_kparams kp)
{
	classify_tile_stream<S, VAR_BPF>(kp, blockIdx.x);
}

__global__ __launch_bounds__(WG) __attribute__((amdgpu_waves_per_eu(8))) void k_fused_nostore(mosrx_kparams kp)
{
	classify_tile_stream<S, VAR_BPF, 131072>(kp, blockIdx.x);
}

__global__ __launch_bounds__(WG) __attribute__((amdgpu_waves_per_eu(8))) void k_fused_cached(mosrx_kparams kp)
{
	classify_tile_stream<S, VAR_BPF, 524288>(kp, blockIdx.x);
}

__global__ __launch_bounds__(WG) __attribute__((amdgpu_waves_per_eu(8))) void k_plain_store(mosrx_kparams kp)
{
	classify_tile_stream<S, 0, 262144>(kp, blockIdx.x);
}

__global__ __launch_bounds__(WG) __attribute__((amdgpu_waves_per_eu(8)))
void kq_plain(const mosrx_qdesc *desc, uint32_t tpb, uint32_t nb, mosrx_qparams qp)
{
	queue_tile<MOSRX_KIND_S13, 0>(desc, tpb, nb, qp);
}

__global__ __launch_bounds__(WG) __attribute__((amdgpu_waves_per_eu(8)))
void kq_fused(const mosrx_qdesc *desc, uint32_t tpb, uint32_t nb, mosrx_qparams qp)
{
	queue_tile<MOSRX_KIND_S13, VAR_BPF>(desc, tpb, nb, qp);
}

static int stamped(int f, const std::vector<mosrx_kparams> &kps, const std::vector<mosrx_qdesc *> &rings,
                   uint32_t tiles, uint32_t rtiles, uint32_t tpb, uint32_t rb, const mosrx_qparams &qp, int iters,
                   double *med)
{
	std::vector<hipEvent_t> e0(iters), e1(iters);
	for (int i = 0; i < iters; i++) {
		CHK(hipEventCreate(&e0[i]));
		CHK(hipEventCreate(&e1[i]));
	}
	for (int i = 0; i < iters; i++) {
		const mosrx_kparams &kp = kps[i % kps.size()];
		const mosrx_qdesc *d = rings[i % rings.size()];
		switch (f) {
		case 0: hipExtLaunchKernelGGL(k_plain, dim3(tiles), dim3(WG), 0, 0, e0[i], e1[i], 0, kp); break;
		case 1: hipExtLaunchKernelGGL(k_fused, dim3(tiles), dim3(WG), 0, 0, e0[i], e1[i], 0, kp); break;
		case 4: hipExtLaunchKernelGGL(k_fused_nostore, dim3(tiles), dim3(WG), 0, 0, e0[i], e1[i], 0, kp); break;
		case 6: hipExtLaunchKernelGGL(k_fused_cached, dim3(tiles), dim3(WG), 0, 0, e0[i], e1[i], 0, kp); break;
		case 5: hipExtLaunchKernelGGL(k_plain_store, dim3(tiles), dim3(WG), 0, 0, e0[i], e1[i], 0, kp); break;
		case 2: hipExtLaunchKernelGGL(kq_plain, dim3(rtiles), dim3(WG), 0, 0, e0[i], e1[i], 0, d, tpb, rb, qp); break;
		case 3: hipExtLaunchKernelGGL(kq_fused, dim3(rtiles), dim3(WG), 0, 0, e0[i], e1[i], 0, d, tpb, rb, qp); break;
		}
	}
	CHK(hipDeviceSynchronize());
	std::vector<float> d(iters);
	for (int i = 0; i < iters; i++) {
		CHK(hipEventElapsedTime(&d[i], e0[i], e1[i]));
		CHK(hipEventDestroy(e0[i]));
		CHK(hipEventDestroy(e1[i]));
	}
	std::sort(d.begin(), d.end());
	*med = d[iters / 2] * 1e3;
	return 0;
}

int main(int argc, char **argv)
{
	const uint32_t n = argc > 1 ? (uint32_t)atoi(argv[1]) : 262144;
	const int nb = 24, rb = 8;   // 24 resident batches (~2.3 GB), rings of 8
	mosrx_trace t;
	if (mosrx_trace_gen(MOSRX_TRACE_IMIX, n, 1000000, 0, &t)) {
		printf("trace_gen failed\n");
		return 1;
	}
	mosrx_params p;
	mosrx_params_default(&p);
	uint32_t tab[MOSRX_TAB_ALLOC_WORDS];
	memset(tab, 0, sizeof(tab));
	mosrx_rss_tables(p.rss_key, p.rss_key_len, tab);
	uint32_t *tables;
	CHK(hipMalloc((void **)&tables, sizeof(tab)));
	CHK(hipMemcpy(tables, tab, sizeof(tab), hipMemcpyHostToDevice));
	const uint32_t tiles = (n + 63) / 64;
	std::vector<mosrx_kparams> kps(nb);
	std::vector<mosrx_qdesc> hd(nb);
	for (int i = 0; i < nb; i++) {
		uint8_t *f; uint32_t *o, *m; uint16_t *l; mosrx_result *r;
		CHK(hipMalloc((void **)&f, t.frames_bytes + 64));
		CHK(hipMemcpy(f, t.frames, t.frames_bytes + 64, hipMemcpyHostToDevice));
		CHK(hipMalloc((void **)&o, n * 4));
		CHK(hipMemcpy(o, t.off, n * 4, hipMemcpyHostToDevice));
		CHK(hipMalloc((void **)&l, n * 2));
		CHK(hipMemcpy(l, t.len, n * 2, hipMemcpyHostToDevice));
		CHK(hipMalloc((void **)&r, n * 16));
		CHK(hipMalloc((void **)&m, n * 4));
		kps[i] = (mosrx_kparams){f, o, l, r, tables, NULL, NULL, m, NULL, (uint32_t)t.frames_bytes, n,
		                         MOSRX_KF_VERIFY};
		memset(&hd[i], 0, sizeof(hd[i]));
		hd[i].frames = f;
		hd[i].off = o;
		hd[i].len = l;
		hd[i].out = r;
		hd[i].bmatch = m;
		hd[i].frames_bytes = (uint32_t)t.frames_bytes;
		hd[i].n = n;
		hd[i].tile_base = (uint32_t)(i % rb) * tiles;
	}
	std::vector<mosrx_qdesc *> rings;
	for (int i = 0; i < nb; i += rb) {
		mosrx_qdesc *d;
		CHK(hipMalloc((void **)&d, rb * sizeof(mosrx_qdesc)));
		CHK(hipMemcpy(d, &hd[i], rb * sizeof(mosrx_qdesc), hipMemcpyHostToDevice));
		rings.push_back(d);
	}
	mosrx_qparams qp;
	memset(&qp, 0, sizeof(qp));
	qp.tables = tables;
	qp.nb = rb;
	qp.flags = MOSRX_KF_VERIFY;
	qp.tpb = tiles;
	// the fused records equal the plain ones, the masks are the set's (8 x ret #1 -> 0xFF for IPv4 frames in
	// datagram mode, 0x55 bits frame mode: checked for non-zero here, the library's tests pin them)
	std::vector<mosrx_result> a(n), b(n);
	std::vector<uint32_t> mk(n);
	hipLaunchKernelGGL(k_plain, dim3(tiles), dim3(WG), 0, 0, kps[0]);
	CHK(hipDeviceSynchronize());
	CHK(hipMemcpy(a.data(), kps[0].out, n * 16, hipMemcpyDeviceToHost));
	CHK(hipMemset(kps[0].out, 0xEE, n * 16));
	hipLaunchKernelGGL(k_fused, dim3(tiles), dim3(WG), 0, 0, kps[0]);
	CHK(hipDeviceSynchronize());
	CHK(hipMemcpy(b.data(), kps[0].out, n * 16, hipMemcpyDeviceToHost));
	CHK(hipMemcpy(mk.data(), kps[0].bmatch, n * 4, hipMemcpyDeviceToHost));
	if (memcmp(a.data(), b.data(), (size_t)n * 16)) {
		printf("fused records differ from plain\n");
		return 2;
	}
	uint32_t zero = 0;
	for (uint32_t i = 0; i < n; i++)
		zero += mk[i] == 0;
	const double bytes = (double)t.caplen_sum + 22.0 * n;
	printf("IMIX %u frames per batch, %u tiles; %.2f MB algorithmic per batch; masks zero for %u frames\n", n, tiles,
	       bytes / 1e6, zero);
	static const char *names[7] = {"single, plain", "single, fused (trivial)", "ring of 8, plain",
	                               "ring of 8, fused (trivial)", "single, fused, masks not stored",
	                               "single, plain + constant masks", "single, fused, cached mask stores"};
	for (int rep = 0; rep < 3; rep++)
		for (int f = 0; f < 7; f++) {
			double med;
			if (stamped(f, kps, rings, tiles, tiles * rb, tiles, rb, qp, 128, &med))
				return 1;
			const double by = bytes * (f == 2 || f == 3 ? rb : 1);
			printf("rep %d %-28s stamped median %8.2f us (%.3f of 8 TB/s)\n", rep, names[f], med,
			       by / (med * 1e-6) / 8e12);
		}
	return 0;
}
