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
#define MOSRX_BPF_POOL 8         /* device buffers the interpreter's instructions rotate over */

/* The fused classify + BPF kernels of a compiled set (bpf_jit.c k_fused_main):
 * one batch as the stream tile (non-temporal / cached tails) or the SMALL tile,
 * the same three over a batch queue, and those three with 8-byte records. */
#define MOSRX_BPF_NFUSED 9
enum { FU_S = 0, FU_SR = 1, FU_M = 2, FU_QS = 3, FU_QSR = 4, FU_QM = 5, FU_QS8 = 6, FU_QSR8 = 7, FU_QM8 = 8 };
struct mosrx_jit_entry {
	uint64_t key;                          /* set_hash of the set */
	hipModule_t mod, fmod;
	hipFunction_t fn;                      /* the set's own kernel; NULL: the compile failed */
	hipFunction_t fu[MOSRX_BPF_NFUSED];    /* fused kernels; NULL: none (two launches) */
};
struct mosrx_bpf_worker;                   /* the context's compile thread (bpf_jit.c) */

/* pipeline slots for the end-to-end path (double-buffered H2D | kernel | D2H) */
#define NSLOT MOSRX_NSLOT

struct slot {
	uint8_t *d_frames;
	uint32_t *d_off;
	uint16_t *d_len;
	mosrx_result *d_res;
	uint32_t *d_fh;
	mosrx_tcpinfo *d_ti;
	uint32_t *d_match;         /* BPF match masks (the group submit with a set installed) */
	uint32_t *d_cnt;
	uint64_t cap_frames;
	uint32_t cap_n;
	hipStream_t stream;
	hipEvent_t done;
	uint32_t *h_cnt;   /* MOSRX_CNT_WORDS, pinned: a D2H copy into pageable memory blocks the host */
	/* The counters only grow: a submit adds to d_cnt and copies it back into
	 * h_cnt, and the wait takes the batch's counts as h_cnt - h_prev (u32
	 * arithmetic, so wrapping is harmless), then keeps h_cnt as h_prev.  No
	 * memset (a blit kernel and a dependent dispatch) per submit; cnt_dirty: the
	 * device words are not h_prev (first use, a submit that failed after its
	 * launch), and the next submit zeroes both. */
	uint32_t *h_prev;
	int cnt_dirty;
	int counted;               /* the last submit made reason counts (mosrx_set_counters) */
	hipEvent_t kev0, kev1;     /* around the kernel of the last submit (when the context times) */
	mosrx_qdesc *h_qdesc;      /* MOSRX_MAX_GROUP, pinned: a group's batch table */
	mosrx_tx_check *h_txc;     /* pinned: the TX pass's check records (mosrx_tx_csum_host), h_txc_n of them */
	uint32_t h_txc_n;
	mosrx_qdesc *d_qdesc;
	const mosrx_qdesc *hq_dev; /* h_qdesc's device address (a direct group's batch table), NULL: none */
	int direct;                /* the last group submit was direct (mosrx_set_direct) */
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
	mosrx_bpf_insn *d_bpf;           /* installed BPF programs (MOSRX_BPF_MAX_INSNS), NULL until set:
	                                  * one of the pool's buffers */
	mosrx_bpf_insn *d_bpf_pool[MOSRX_BPF_POOL];
	int bpf_pool_used[MOSRX_BPF_POOL];   /* a launch may have read it since it was written */
	uint32_t bpf_pool_next;
	mosrx_bparams bpf;               /* program table of the installed set */
	hipFunction_t bpf_fn;            /* compiled form of the installed set (bpf_jit.c), NULL: interpreter */
	int bpf_engine_req;              /* MOSRX_BPF_ENGINE_* for the next mosrx_bpf_set */
	char bpf_jit_log[512];           /* hipRTC log of the last failed compile */
	hipFunction_t bpf_fu[MOSRX_BPF_NFUSED];   /* fused classify + BPF kernels, NULL: none */
	struct mosrx_jit_entry jit[MOSRX_BPF_JIT_CACHE];
	uint32_t njit;
	uint64_t bpf_key;                /* set_hash of the installed set */
	int bpf_pending;                 /* its compile is outstanding (the interpreter runs it meanwhile) */
	struct mosrx_bpf_worker *bw;
	hipStream_t xs[MOSRX_MAX_STREAMS];   /* timing streams (mosrx_time_op), created on first use */
	hipEvent_t xdone[MOSRX_MAX_STREAMS];
	uint32_t nxs;
	/* callers' streams a launch reading the installed set went to since the last
	 * drain, each with an event recorded after that launch (mosrx__note_stream);
	 * foreign_streams: more of them than the table holds, so the drain falls back
	 * to a device-wide sync */
#define MOSRX_FOREIGN 8
	hipStream_t fstream[MOSRX_FOREIGN];
	hipEvent_t fev[MOSRX_FOREIGN];
	uint32_t nfs;
	int foreign_streams;
	int timing;                      /* record kernel events on the end-to-end path (mosrx_set_timing) */
	int no_counters;                 /* group submits make no reason counts (mosrx_set_counters) */
	uint64_t direct_max;             /* largest direct group, input bytes (mosrx_set_direct); 0: none */
	uint32_t direct_frames;          /*   and its most frames */
	float last_kernel_ms;            /* kernel time of the last waited submit, -1 if not timed */
};

int mosrx__check_batch(const mosrx_batch *b, int dev);
void *mosrx__host_dev_of(const void *p, uint64_t len, int device);
int mosrx__bpf_jit_request(mosrx_ctx *c, const mosrx_bpf_insn *insns);
int mosrx__bpf_jit_wait(mosrx_ctx *c);
void mosrx__bpf_poll(mosrx_ctx *c);
int mosrx__bpf_fused_queue_launch(mosrx_ctx *c, const mosrx_qparams *qp, uint32_t total_tiles, int small,
                                  int variant, hipStream_t s);
/* The installed set's standalone kernel (compiled, else the interpreter) over a
 * device-resident batch, match masks into match[n]. */
int mosrx__bpf_launch_dev(mosrx_ctx *c, const uint8_t *frames, uint64_t frames_bytes, const uint32_t *off,
                          const uint16_t *len, uint32_t n, uint32_t *match, hipStream_t s);
int mosrx__bpf_jit_launch(mosrx_ctx *c, const mosrx_bparams *bp, hipStream_t s);
int mosrx__bpf_jit_source(const mosrx_bpf_insn *insns, const mosrx_bparams *t, char **out);
void mosrx__bpf_jit_free(mosrx_ctx *c);
int mosrx__bpf_jit_compile(const char *src, char *log, size_t logsz, size_t *code_size);
int mosrx__bpf_jit_compile_fused(const mosrx_bpf_insn *insns, const mosrx_bparams *t, char *log, size_t logsz,
                                 size_t *code_size);
int mosrx__bpf_jit_hook_source(const mosrx_bpf_insn *insns, const mosrx_bparams *t, char **out);
int mosrx__bpf_fused_launch(mosrx_ctx *c, const mosrx_kparams *kp, int small, hipStream_t s);
int mosrx__slot_reserve(mosrx_ctx *c, struct slot *s, uint64_t frames_bytes, uint32_t n);
/* A launch that reads the installed BPF set (its staged instructions or its
 * compiled module) was just made on stream s: when s is not one of the
 * context's own streams (a caller's stream), an event recorded on s after it
 * lets mosrx__drain wait for exactly that work. */
void mosrx__note_stream(mosrx_ctx *c, hipStream_t s);
/* Every launch that may still read a staged instruction buffer or a compiled
 * module has finished: the context's own streams synchronised, and the events
 * noted on callers' streams since the last drain (the whole device only when
 * more streams were used than the table holds).  Before a buffer is rewritten
 * or a module unloaded. */
int mosrx__drain(mosrx_ctx *c);

/* The variant a launch of `n` frames in `bytes` runs: the context's, with the
 * tail loads cached instead of non-temporal for batches of small frames when
 * the context runs the library default (mosrx_api.c). */
int mosrx__tail_variant(const mosrx_ctx *c, uint64_t bytes, uint64_t n);

#endif
