/*
 * mosrx_ctx.h — host-side context layout shared by the C host files
 * (mosrx_api.c, bpf_api.c).  Not part of the ABI.
 */
#ifndef MOSRX_CTX_H
#define MOSRX_CTX_H

#define __HIP_PLATFORM_AMD__ 1
#include <hip/hip_runtime_api.h>

#include "mosrx_internal.h"

#define HIPCHK(x) do { if ((x) != hipSuccess) return -EIO; } while (0)

#define MOSRX_BPF_JIT_CACHE 16   /* compiled program sets kept per context */

/* pipeline slots for the end-to-end path (double-buffered H2D | kernel | D2H) */
#define NSLOT MOSRX_NSLOT

struct slot {
	uint8_t *d_frames;
	uint32_t *d_off;
	uint16_t *d_len;
	mosrx_result *d_res;
	uint32_t *d_fh;
	mosrx_tcpinfo *d_ti;
	uint32_t *d_cnt;
	uint64_t cap_frames;
	uint32_t cap_n;
	hipStream_t stream;
	hipEvent_t done;
	uint32_t *h_cnt;   /* MOSRX_R_COUNT, pinned: a D2H copy into pageable memory blocks the host */
	hipEvent_t kev0, kev1;     /* around the kernel of the last submit (when the context times) */
	mosrx_qdesc *h_qdesc;      /* MOSRX_MAX_GROUP, pinned: a group's batch table */
	mosrx_qdesc *d_qdesc;
	int timed;
	int busy;
};

struct mosrx_ctx {
	int device;
	hipStream_t stream;
	mosrx_params params;
	uint32_t kflags;
	uint32_t *d_tables;
	struct slot slot[NSLOT];
	uint32_t h_cnt[MOSRX_R_COUNT];   /* counters of the last waited batch */
	hipEvent_t ev0, ev1;
	int variant;                     /* kernel cache-policy variant (mosrx_set_variant) */
	mosrx_bpf_insn *d_bpf;           /* installed BPF programs (MOSRX_BPF_MAX_INSNS), NULL until set */
	mosrx_bparams bpf;               /* program table of the installed set */
	hipFunction_t bpf_fn;            /* compiled form of the installed set (bpf_jit.c), NULL: interpreter */
	int bpf_engine_req;              /* MOSRX_BPF_ENGINE_* for the next mosrx_bpf_set */
	char bpf_jit_log[512];           /* hipRTC log of the last failed compile */
	hipFunction_t bpf_fs, bpf_fm;    /* fused classify + BPF kernels (S13 / SMALL tiles), NULL: none */
	hipFunction_t bpf_fr;            /* the S13 one with cached tail loads (batches of small frames) */
	struct { uint64_t key; hipModule_t mod, fmod; hipFunction_t fn, fs, fm, fr; } jit[MOSRX_BPF_JIT_CACHE];
	uint32_t njit;
	hipStream_t xs[MOSRX_MAX_STREAMS];   /* timing streams (mosrx_time_op), created on first use */
	hipEvent_t xdone[MOSRX_MAX_STREAMS];
	uint32_t nxs;
	int timing;                      /* record kernel events on the end-to-end path (mosrx_set_timing) */
	float last_kernel_ms;            /* kernel time of the last waited submit, -1 if not timed */
};

int mosrx__check_batch(const mosrx_batch *b, int dev);
int mosrx__bpf_jit_build(mosrx_ctx *c, const mosrx_bpf_insn *insns);
int mosrx__bpf_jit_launch(mosrx_ctx *c, const mosrx_bparams *bp, hipStream_t s);
int mosrx__bpf_jit_source(const mosrx_bpf_insn *insns, const mosrx_bparams *t, char **out);
void mosrx__bpf_jit_free(mosrx_ctx *c);
int mosrx__bpf_jit_compile(const char *src, char *log, size_t logsz, size_t *code_size);
int mosrx__bpf_jit_compile_fused(const mosrx_bpf_insn *insns, const mosrx_bparams *t, char *log, size_t logsz,
                                 size_t *code_size);
int mosrx__bpf_jit_hook_source(const mosrx_bpf_insn *insns, const mosrx_bparams *t, char **out);
int mosrx__bpf_fused_launch(mosrx_ctx *c, const mosrx_kparams *kp, int small, hipStream_t s);
int mosrx__slot_reserve(mosrx_ctx *c, struct slot *s, uint64_t frames_bytes, uint32_t n);

/* The variant a launch of `n` frames in `bytes` runs: the context's, with the
 * tail loads cached instead of non-temporal for batches of small frames when
 * the context runs the library default (mosrx_api.c). */
int mosrx__tail_variant(const mosrx_ctx *c, uint64_t bytes, uint64_t n);

#endif
