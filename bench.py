#!/usr/bin/env python3
"""bench.py — device-resident throughput of the MI355X rx classifier.

The hot path: mOS's ProcessPacket checks + ip_fast_csum + TCPCalcChecksum +
Toeplitz RSS / queue map, over batches of frames already resident in HBM.

One STEP = one rx round over the resident batches of one rx ring: R batches of
the workload's batch size (each batch its own frames, descriptors and records),
classified by ONE launch of the batch-queue kernel (mosrx_queue_run), which is
how gpu_module_func services a group of received batches (cfg.group).  The
headline workload is BASELINE config #3 (1500 B MTU TCP segments, 1M flows,
batch 64K, R = 8); the same run measures config #2 (64 B, 1 flow, batch 32K,
R = 256) and config #4 (IMIX, batch 256K, R = 8), the single-batch launches
of each (`*_1`: one kernel per batch, 2 batches in flight), the §8f rows, the
CPU baselines (the oracle, mOS's own compiled per-frame functions and mOS's
whole ProcessPacket on this host's cores, config #1 included), the box's
streaming-read rate, and the end-to-end / backend rates (one rx loop per mTCP
thread, 1-8 threads).

Multi-GPU (torchrun, one process per GPU): the job is one sequence of batches
split round-robin over the GPUs (mosrx.shard_plan), no
collective on the data path (`scaling: weak`); gloo carries only the barrier
and the max-over-ranks of the timed region.

Each rank keeps >= 1.2 GB of distinct resident batches and cycles over them, so
no timed pass is served from the 256 MiB Infinity Cache.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W]
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import struct
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "mos-networking-stack_amd"))

import numpy as np  # noqa: E402

import mosrx  # noqa: E402  (loads libmosrx.so before torch so one HIP runtime is used)

METRIC = "Mpkts/s + GB/s device-resident checksum+RSS classify, 64B & 1500B batches"
HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md)
DESC_BYTES, RESULT_BYTES = 6, 16
RESIDENT_BYTES = 1200 << 20    # working set per rank: well past the 256 MiB Infinity Cache

# key: (trace kind, batch, batches per step (ring) or 0 (one launch per batch), label)
WORKLOADS = {
    "M1500": (mosrx.TRACE_M1500, 65_536, 8, "1xMI355X 1500B MTU TCP segments, 1M distinct 5-tuples, batch=64K (BASELINE config #3)"),
    "S64": (mosrx.TRACE_S64, 32_768, 256, "1xMI355X 64B TCP, 1 flow, batch=32K (BASELINE config #2), full verdict"),
    "S64_hdr": (mosrx.TRACE_S64, 32_768, 256, "config #2 header parse + IP cksum + RSS only (skip_tcp_csum), "
                                              "8-byte records (mosrx_result8)"),
    "S64_hdr16": (mosrx.TRACE_S64, 32_768, 256, "config #2 header-only as S64_hdr, 16-byte records"),
    # the full verdict (TCP checksum included) with the 8-byte records the drop-in path
    # hands mOS (gpu_module_func cfg.compact)
    "S64_c8": (mosrx.TRACE_S64, 32_768, 256, "config #2 full verdict, 8-byte records (mosrx_result8)"),
    # the same frames packed back to back (60-byte stride, every frame at a different
    # alignment) instead of at 16-byte boundary + 2: the inter-frame pad is the 64 B
    # rows' only traffic beyond the algorithmic bytes (diagnostic row)
    "S64_hdr_packed": (mosrx.TRACE_S64, 32_768, 256, "config #2 header-only, 8-byte records, frames packed back to "
                                                     "back (60 B stride)"),
    # the full verdict with 8-byte records on the layout the drop-in backend stages small
    # frames in (back to back, mosrx_source_fill)
    "S64_c8_packed": (mosrx.TRACE_S64, 32_768, 256, "config #2 full verdict, 8-byte records, frames packed back "
                                                    "to back as the backend stages them (60 B stride)"),
    "IMIX": (mosrx.TRACE_IMIX, 262_144, 8, "IMIX 60/590/1514 7:4:1, 1M flows, batch=256K (BASELINE config #4)"),
    # one kernel launch per batch, two batches in flight (two rx queues)
    "M1500_1": (mosrx.TRACE_M1500, 65_536, 0, "config #3, one launch per 64K batch"),
    "S64_1": (mosrx.TRACE_S64, 32_768, 0, "config #2, one launch per 32K batch"),
    "IMIX_1": (mosrx.TRACE_IMIX, 262_144, 0, "config #4, one launch per 256K batch"),
    # SURVEY.md §8f rows measured on the same traces (one launch per batch)
    "M1500_fh": (mosrx.TRACE_M1500, 65_536, 0, "config #3 classify + flow-table hash (HashFlow of FindStream's tuple)"),
    "M1500_ti": (mosrx.TRACE_M1500, 65_536, 0, "config #3 classify + pkt_info TCP fields (FillPacketContextTCPInfo)"),
    "M1500_tx": (mosrx.TRACE_M1500, 65_536, 0, "config #3 TX checksum rewrite (MOS_UPDATE_IP|TCP_CHKSUM), in place"),
    "M1500_txc": (mosrx.TRACE_M1500, 65_536, 0, "config #3 TX checksums as 8-byte records, frames untouched "
                  "(mosrx_tx_csum_dev_checks)"),
    "IMIX_bpf": (mosrx.TRACE_IMIX, 262_144, 0, "config #4 batched BPF, 8 mOS filter programs (sfbpf_compile output)"),
    "IMIX_cls_bpf": (mosrx.TRACE_IMIX, 262_144, 0, "config #4 classify + the 8 BPF programs fused in one pass"),
    # the fused pass over a ring (the batch queue: gpu_module_func's groups with filters installed)
    "IMIX_cls_bpf_ring": (mosrx.TRACE_IMIX, 262_144, 8, "config #4 classify + 8 BPF programs fused, one batch-queue "
                                                         "launch over 8 batches"),
    "S64_cls_bpf_ring": (mosrx.TRACE_S64, 32_768, 256, "config #2 classify + 8 BPF programs fused, one batch-queue "
                                                       "launch over 256 batches"),
}
DEFAULT_WORKLOADS = ("M1500,S64,S64_c8,S64_c8_packed,S64_hdr,S64_hdr16,S64_hdr_packed,IMIX,M1500_1,S64_1,IMIX_1,M1500_fh,M1500_ti,"
                     "M1500_tx,M1500_txc,IMIX_bpf,IMIX_cls_bpf,IMIX_cls_bpf_ring,S64_cls_bpf_ring")
OPS = {"M1500_fh": mosrx.OP_CLASSIFY_FH, "M1500_ti": mosrx.OP_CLASSIFY_TI, "M1500_tx": mosrx.OP_TX_CSUM,
       "M1500_txc": mosrx.OP_TX_CHECKS,
       "IMIX_bpf": mosrx.OP_BPF, "IMIX_cls_bpf": mosrx.OP_CLASSIFY_BPF}
# filter expressions whose compiled programs (tests/golden/bpf.npz, mOS's own compiler) the BPF row runs
BPF_BENCH = [("tcp", 0), ("tcp port 80", 0), ("tcp[tcpflags] & tcp-syn != 0", 1), ("net 192.168.0.0/16 and tcp", 1),
             ("host 10.0.0.1 and port 80", 0), ("ip[8] < 64", 1), ("tcp[((tcp[12:1] & 0xf0) >> 2):4] = 0x47455420", 1),
             ("portrange 1000-2000", 0)]
# rows whose records are the 8-byte mosrx_result8 (the drop-in path's compact form)
COMPACT = ("S64_hdr", "S64_hdr_packed", "S64_c8", "S64_c8_packed", "c8")
PREWARM_S = 0.3
STREAMS = 2      # rx batches in flight per GPU for the one-launch-per-batch rows
# the layout hint the resident batches are handed over with (mosrx_batch.layout): "auto" =
# their own fixed stride when they have one (the 64 B traces), None = none (A/B runs)
HINT = "auto"
DISTINCT = 8     # distinct batch contents generated per rank (the rest are resident copies of them)


_T0 = time.time()


def progress(msg: str):
    """One line on stderr per leg (a long run keeps writing while it works)."""
    print(f"[bench +{time.time() - _T0:.0f}s] {msg}", file=sys.stderr, flush=True)


def dist_env():
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    return ws, rank, local


class Dist:
    """Barrier, max and gather over ranks (gloo, CPU): the timed regions' bounds and
    the reduction of the per-rank figures; nothing on the data path."""

    def __init__(self, ws: int, rank: int):
        self.ws, self.rank, self.pg = ws, rank, None
        if ws > 1:
            import torch.distributed as dist
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            dist.init_process_group("gloo", rank=rank, world_size=ws)
            self.dist = dist

    def barrier(self):
        if self.ws > 1:
            self.dist.barrier()

    def max(self, x: float) -> float:
        if self.ws == 1:
            return x
        import torch
        t = torch.tensor([x], dtype=torch.float64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def gather(self, x: list[float]) -> list[list[float]]:
        """Every rank's vector x (same length on all ranks), in rank order."""
        if self.ws == 1:
            return [list(x)]
        import torch
        t = torch.zeros(self.ws, len(x), dtype=torch.float64)
        t[self.rank] = torch.tensor(x, dtype=torch.float64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.SUM)
        return t.tolist()

    def leg(self, fn):
        """Run one end-to-end leg on every rank at once (each rank on its own GPU
        and host thread) and reduce it.  fn(sync) sets its leg up, calls sync()
        right before and right after its timed region -- a barrier, so every
        rank's timed region starts together -- and returns this rank's `frames`,
        `bytes` and `seconds` (the timed region).  Returns (this rank's dict, the
        job's aggregate)."""
        r = fn(self.barrier)
        rows = self.gather([float(r["frames"]), float(r["bytes"]), float(r["seconds"])])
        return r, aggregate(rows)

    def close(self):
        if self.ws > 1:
            self.dist.destroy_process_group()


def aggregate(rows: list[list[float]]) -> dict:
    """The job's rate from per-rank (frames, bytes, wall seconds) of legs run at the
    same time on every rank: everything all ranks moved over the longest rank's
    wall time (the job ends with its last rank), and each rank's own rate."""
    frames = sum(r[0] for r in rows)
    nbytes = sum(r[1] for r in rows)
    wall = max(r[2] for r in rows)
    per = [r[0] / r[2] / 1e6 if r[2] > 0 else 0.0 for r in rows]
    return {"ranks": len(rows), "frames": int(frames), "seconds": round(wall, 4),
            "mpkts": round(frames / wall / 1e6, 2) if wall > 0 else None,
            "gbps": round(nbytes / wall / 1e9, 2) if wall > 0 else None,
            "per_rank_mpkts": {"min": round(min(per), 2), "max": round(max(per), 2)}}


def job_seed(kind: int, b: int) -> int:
    """Seed of the job's batch b: batch 0 is the default seeded trace of the config
    (BASELINE.md §3), every later batch its own deterministic content."""
    return 0 if b == 0 else ((mosrx.TRACE_SEED_BASE + kind) ^ (b * 0x9E3779B97F4A7C15)) & (2**64 - 1) or 1


def job_batches(nbatches: int, world: int, rank: int) -> list[int]:
    """The batches of the job this rank classifies: config #5's round-robin split."""
    return mosrx.shard_plan(nbatches, world, rank)


def algo_bytes(tr: mosrx.Trace, key: str = "") -> int:
    """B_i = caplen_i + 6 (offset+len descriptor) + 16 (result record).
    Flow hash: + 4 B per frame; pkt_info fields: + 12 B.  TX rewrite: caplen + 6 read,
    4 B written (no records).  BPF: the 6-byte descriptor + 4-byte mask + 64 header
    bytes per frame (the line a filter reads; deeper loads are extra)."""
    if key.endswith("_tx"):
        return tr.caplen_sum + tr.n * (DESC_BYTES + 4)
    if key.endswith("_txc"):       # the 8-byte check record per frame
        return tr.caplen_sum + tr.n * (DESC_BYTES + 8)
    if "_cls_bpf" in key:          # the classify bytes + the 4-byte match mask (8-byte records: _c8)
        return tr.caplen_sum + tr.n * (DESC_BYTES + (8 if key.endswith("_c8") else RESULT_BYTES) + 4)
    if key in COMPACT:                         # 8-byte compact records
        return tr.caplen_sum + tr.n * (DESC_BYTES + 8)
    if key.endswith("_bpf"):
        return tr.n * (DESC_BYTES + 4) + int(np.minimum(tr.len, 64).astype(np.int64).sum())
    extra = 4 if key.endswith("_fh") else 12 if key.endswith("_ti") else 0
    return tr.caplen_sum + tr.n * (DESC_BYTES + RESULT_BYTES + extra)


def bpf_bench_programs():
    z = np.load(os.path.join(ROOT, "tests", "golden", "bpf.npz"))
    names = [str(x) for x in z["names"]]
    progs = []
    for expr, mode in BPF_BENCH:
        j = names.index(expr)
        progs.append((z["insns"][z["prog_off"][j]:z["prog_off"][j] + z["prog_len"][j]], mode))
    return progs


def load_pmc(key: str):
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as fh:
            d = json.load(fh)
        return d.get(key)
    except (OSError, ValueError):
        return None


def prewarm(fn, seconds: float = PREWARM_S):
    """Untimed GPU work before a workload's warmup steps: the MI355X's clocks
    ramp over the first ~100 ms of load, and a few ms of steps alone measured
    ~9 % slow (gpurun_out r01: 22.4 us per 1500 B launch after 2 ms, 20.5 after 20 ms)."""
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        fn()


def median_of(fn, reps: int = 5) -> float:
    """Median of `reps` repetitions of a per-launch timing."""
    return float(np.median([fn() for _ in range(reps)]))


def kernel_duration(stamped, back_to_back: float):
    """(ms, method) of one launch for the roofline: the kernel's own duration
    from dispatch-stamped events (median of 5) when the operation is one kernel
    and the runtime stamps it, else the back-to-back figure."""
    try:
        if stamped() is not None:
            return median_of(stamped), "dispatch-stamped (hipExtLaunchKernel events), median of 5"
    except mosrx.MosrxError as e:
        print(f"[bench] dispatch-stamped timing unavailable ({e}): back-to-back figure used", file=sys.stderr)
    return back_to_back, "HIP events around back-to-back launches, median of 5"


def stamp_floor(ctx, db, iters, timing):
    """ms the dispatch stamp reads for an empty kernel with db's classify grid
    (median of 5), when the row's own figure is dispatch-stamped; else None."""
    if not timing.startswith("dispatch-stamped"):
        return None
    return median_of(lambda: ctx.probe_stamp_floor(db, iters))


def pack_uniform(t: mosrx.Trace) -> mosrx.Trace:
    """Trace t with its frames packed back to back (all frames one length, as in the
    64 B traces): frame i at 2 + i * len instead of at a 16-byte boundary + 2."""
    ln = int(t.len[0])
    assert (t.len == ln).all() and (np.diff(t.off.astype(np.int64)) == int(t.off[1]) - int(t.off[0])).all()
    stride = int(t.off[1]) - int(t.off[0])
    rows = t.frames[int(t.off[0]):int(t.off[0]) + stride * t.n].reshape(t.n, stride)[:, :ln]
    p = mosrx.Trace.__new__(mosrx.Trace)
    p.n = t.n
    p.frames = np.zeros(2 + ln * t.n + 64, np.uint8)
    p.frames[2:2 + ln * t.n] = rows.reshape(-1)
    p.off = (2 + ln * np.arange(t.n, dtype=np.uint64)).astype(np.uint32)
    p.len = t.len.copy()
    p.frames_bytes = 2 + ln * t.n
    p.max_len, p.caplen_sum = t.max_len, t.caplen_sum
    return p


def resident_batches(ctx, key, world, rank, nres):
    """`nres` resident batches of this rank's share of the job: the contents of its
    first job batches (seeded per job batch; DISTINCT of them for a ring, 2 for the
    one-launch rows), cycled over distinct HBM buffers.  Returns (device batches,
    traces used, their job batch indices)."""
    kind, batch, ring, _ = WORKLOADS[key]
    nd = min(DISTINCT, ring) if ring else 2
    mine = job_batches(world * nd, world, rank)[:nd]
    trs = [mosrx.Trace(kind, batch, seed=job_seed(kind, b)) for b in mine]
    if key.endswith("_packed"):
        trs = [pack_uniform(t) for t in trs]
    dbs = [ctx.upload(t.frames, t.off, t.len, frames_bytes=t.frames_bytes, max_len=t.max_len, hint=HINT)
           for t in (trs[i % len(trs)] for i in range(nres))]
    return dbs, trs, mine


def measure(ctx, dist, key, steps, warmup, rank):
    kind, batch, ring, label = WORKLOADS[key]
    params = mosrx.default_params(skip_tcp_csum=1 if key.startswith("S64_hdr") else 0)
    ctx.set_params(params)
    probe = mosrx.Trace(kind, batch)
    per_batch = max(probe.frames_bytes, 1)
    if ring:
        nres = max(2 * ring, -(-RESIDENT_BYTES // per_batch))
        nres = -(-nres // ring) * ring                     # whole rings
    else:
        nres = min(256, max(2, -(-RESIDENT_BYTES // per_batch)))
    dbs, trs, mine = resident_batches(ctx, key, dist.ws, rank, nres)
    tr = trs[0]
    ab = algo_bytes(tr, key)
    if key in OPS:
        op = OPS[key]
        arg = mosrx.TX_IP_CSUM | mosrx.TX_TCP_CSUM if op in (mosrx.OP_TX_CSUM, mosrx.OP_TX_CHECKS) else 0
        if op in (mosrx.OP_BPF, mosrx.OP_CLASSIFY_BPF):
            ctx.bpf_set(bpf_bench_programs())
        step_fn = lambda k, ns: ctx.time_op(op, dbs, k, ns, arg, kernels=False)[0]   # noqa: E731
        prewarm(lambda: step_fn(200, STREAMS))
        if warmup:
            step_fn(warmup, STREAMS)
        ctx.device_sync()
        dist.barrier()
        t0 = time.perf_counter()
        dev_ms = step_fn(steps, STREAMS)
        ctx.device_sync()
        wall = time.perf_counter() - t0     # this rank's region; the max over ranks below
        dist.barrier()
        wall_max = dist.max(wall)
        kk = 500
        # the kernel's own duration (each launch stamped by its dispatch, as
        # rocprofv3 reports it); ops of more than one launch: back to back
        kern_b2b = median_of(lambda: step_fn(kk, 1) / kk)
        kern_ms, timing = kernel_duration(lambda: ctx.time_op_dispatch(op, dbs, kk, arg), kern_b2b)
        kern_iso = None
        floor_ms = stamp_floor(ctx, dbs[0], kk, timing)
        frames_per_step, ab_step = batch, ab
        method = f"one launch per batch, batch i on stream i % {STREAMS}"
    elif ring:
        # each step = ONE queue launch over `ring` distinct resident batches (an rx
        # ring serviced at once, gpu_module_func cfg.group); several rings over
        # disjoint resident copies cycle so the working set stays past the L3
        if "_cls_bpf" in key:
            ctx.bpf_set(bpf_bench_programs())   # (compiled before the queues run)
        compact = key in COMPACT
        qs = [ctx.queue_ex(dbs[i:i + ring], match="_cls_bpf" in key, compact=compact)
              for i in range(0, len(dbs), ring)]
        prewarm(lambda: qs[0].time(8, qs[1:], kernels=False))
        if warmup:
            qs[0].time(warmup, qs[1:], kernels=False)
        ctx.device_sync()
        dist.barrier()
        t0 = time.perf_counter()
        dev_ms, _ = qs[0].time(steps, qs[1:], kernels=False)
        ctx.device_sync()
        wall = time.perf_counter() - t0     # this rank's region; the max over ranks below
        dist.barrier()
        wall_max = dist.max(wall)
        kk = max(16, 4 * len(qs))
        kern_b2b = median_of(lambda: qs[0].time(kk, qs[1:], kernels=False)[0] / kk)
        kern_ms, timing = kernel_duration(lambda: qs[0].time_dispatch(kk, qs[1:]), kern_b2b)
        floor_ms = None
        _, kern_iso = qs[0].time(min(kk, 32), qs[1:])
        for q in qs:
            q.destroy()
        frames_per_step, ab_step = batch * ring, ab * ring
        method = f"one batch-queue launch per step over {ring} resident batches" + (
            " (fused classify + BPF queue kernel)" if "_cls_bpf" in key else
            ", 8-byte records" if compact else "")
    else:
        prewarm(lambda: ctx.time_dev_streams(dbs, 200, STREAMS))
        if warmup:
            ctx.time_dev_streams(dbs, warmup, STREAMS)
        ctx.device_sync()
        dist.barrier()
        t0 = time.perf_counter()
        # K back-to-back batches, batch i on stream i % STREAMS (independent rx
        # batches overlap launch and drain); HIP events on the kernel streams
        dev_ms = ctx.time_dev_streams(dbs, steps, STREAMS)
        ctx.device_sync()
        wall = time.perf_counter() - t0     # this rank's region; the max over ranks below
        dist.barrier()
        wall_max = dist.max(wall)
        # roofline: the kernel's own duration over 500 back-to-back launches on
        # ONE stream, each launch stamped by its dispatch (hipExtLaunchKernel: the
        # figure rocprofv3's kernel trace reports), median of 5 such runs; kept
        # beside it: events around the 500 launches (dispatch gaps included) and
        # around each single launch (dispatch included)
        kk = 500
        kern_b2b = median_of(lambda: ctx.time_dev_streams(dbs, kk, 1) / kk)
        kern_ms, timing = kernel_duration(lambda: ctx.time_op_dispatch(mosrx.OP_CLASSIFY, dbs, kk), kern_b2b)
        kern_iso = ctx.time_dev_kernels(dbs, kk)
        floor_ms = stamp_floor(ctx, dbs[0], kk, timing)
        frames_per_step, ab_step = batch, ab
        method = f"one launch per batch, batch i on stream i % {STREAMS}"
    for d in dbs:
        d.free()
    n = dist.ws
    # each rank's own device rate over its timed steps (HIP events on its kernel stream)
    per_rank = [r[0] for r in dist.gather([ab_step * steps / (dev_ms * 1e-3) / 1e9 if dev_ms > 0 else 0.0])]
    out = {
        "workload": label,
        "batch": batch,
        "batches_per_step": ring or 1,
        "method": method,
        "frames_bytes_per_batch": tr.frames_bytes,
        "algo_bytes_per_batch": ab,
        "resident_batches": len(dbs),
        "resident_bytes": int(sum(t.frames_bytes for t in (trs[i % len(trs)] for i in range(len(dbs))))),
        "job_batches": mine,
        "wall_s": wall_max,
        "ms_per_step": 1e3 * wall_max / steps,
        "gbps": n * ab_step * steps / wall_max / 1e9,
        "mpkts": n * frames_per_step * steps / wall_max / 1e6,
        "device_ms_per_step": dev_ms / steps,
        "kernel_ms": kern_ms,
        "kernel_ms_back_to_back": kern_b2b,
        "kernel_ms_isolated": kern_iso,
        "per_rank_device_gbps": {"min": round(min(per_rank), 1), "max": round(max(per_rank), 1)},
    }
    achieved = ab_step / (kern_ms * 1e-3) / 1e9
    pmc = load_pmc(key)
    out["roofline"] = {
        "bound": "hbm",
        "achieved": round(achieved, 1),
        "peak": HBM_PEAK_GBS,
        "unit": "GB/s",
        "frac": round(achieved / HBM_PEAK_GBS, 4),
        "traffic": (pmc or {}).get("hbm_bytes_per_launch"),
        # the launch duration behind `achieved` (the kernel's own duration, each
        # of the back-to-back launches stamped by its dispatch, median of 5), and
        # the timed region's own device time per step (HIP events around the K
        # timed steps)
        "launch_us": round(kern_ms * 1e3, 3),
        "launch_timing": timing,
        "launch_us_back_to_back": round(kern_b2b * 1e3, 3),
        "timed_region_device_us_per_step": round(1e3 * dev_ms / steps, 3),
    }
    if floor_ms is not None:
        # the stamp's own reading for an empty kernel of this launch's grid: a short
        # launch's stamped figure is stated against it (rocprofv3's trace in profiles/)
        out["roofline"]["stamp_floor_us"] = round(floor_ms * 1e3, 3)
        out["roofline"]["launch_us_over_empty"] = round((kern_ms - floor_ms) * 1e3, 3)
    if pmc:
        out["roofline"]["traffic_source"] = pmc.get("source")
    return out, tr


def cpu_share():
    """Threads one GPU's share of the host may use: the process's CPU affinity,
    capped by the share the environment states (MOSRX_CPU_THREADS /
    OMP_NUM_THREADS: 16 per GPU on the pool's boxes, whose nproc shows the whole
    machine).  Returns (threads, affinity size, the stated cap or None)."""
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    cap = os.environ.get("MOSRX_CPU_THREADS") or os.environ.get("OMP_NUM_THREADS")
    cap = int(cap) if cap else None
    return (max(1, min(aff, cap)) if cap else aff), aff, cap


def cpu_quota():
    """CPUs' worth of time the process's cgroup may use (cpu.max / cfs quota), or
    None when unlimited: a thread count above it measures the quota, not the cores."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as fh:
            q, per = fh.read().split()[:2]
        return None if q == "max" else int(q) / int(per)
    except (OSError, ValueError):
        pass
    try:
        with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as fh:
            q = int(fh.read())
        with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as fh:
            per = int(fh.read())
        return None if q <= 0 else q / per
    except (OSError, ValueError):
        return None


def host_model():
    try:
        with open("/proc/cpuinfo") as fh:
            return next((ln.split(":", 1)[1].strip() for ln in fh if ln.startswith("model name")), "")
    except OSError:
        return ""


def cpu_baseline(tr: mosrx.Trace, key: str, min_s: float = 3.0, shares: bool = True, ws: int = 1,
                 host_cpus=None):
    """The oracle (bit-exact C restatement, oracle/mosrx_oracle.c) on this host's cores:
    one core (`value`), one GPU's share of the host (`per_gpu_share`: the threads a
    rank may use, e.g. 16 of 256 CPUs on the pool's 1-GPU boxes), and for a job of
    `ws` GPUs the whole job's share (`job_share`: ws x that, over the CPUs the
    process had before its NUMA binding, `host_cpus`) -- the host-core figure the
    ws-GPU line stands next to.  One pthread per core over disjoint trace slices,
    as mOS shards per core.  Reported baseline only; never the measured product path."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_py as O
    p = O.params(skip_tcp_csum=1 if key.startswith("S64_hdr") else 0)
    ab = algo_bytes(tr, key)

    if key in OPS or "_cls_bpf" in key:
        return cpu_baseline_row(tr, key, min_s, O)

    def run(nt):
        reps, t0 = 0, time.perf_counter()
        while True:
            O.classify(tr.frames, tr.off, tr.len, p, nthreads=nt)
            reps += 1
            el = time.perf_counter() - t0
            if el >= min_s:
                return reps, el

    def leg(nt, what):
        rn, en = run(nt)
        return {"value": round(rn * ab / en / 1e9, 3), "unit": "GB/s", "cores": nt, "kind": "port",
                "mpkts": round(rn * tr.n / en / 1e6, 3),
                "sample": f"{rn} passes over one {tr.n}-frame batch, {nt} pthreads over disjoint slices "
                          f"({en:.1f} s); {what}; host nproc {os.cpu_count()}"}

    r1, e1 = run(1)
    gb1 = r1 * ab / e1 / 1e9
    out = {
        "value": round(gb1, 3), "unit": "GB/s", "cores": 1, "kind": "port",
        "mpkts": round(r1 * tr.n / e1 / 1e6, 3),
        "sample": f"{r1} passes over one {tr.n}-frame batch of this workload ({e1:.1f} s), "
                  f"oracle/mosrx_oracle.c mo_classify, 1 thread; host '{host_model()}', nproc {os.cpu_count()}",
    }
    if not shares:
        return out
    nt, aff, cap = cpu_share()
    out["per_gpu_share"] = leg(nt, f"one GPU's share of the host: {nt} of {os.cpu_count()} CPUs "
                                   f"(affinity {aff}, stated share {cap})")
    out["per_gpu_share"]["host_cpus"] = os.cpu_count()
    out["per_gpu_share"]["cpu_quota"] = cpu_quota()
    if ws > 1 and host_cpus:
        # the job's share: ws GPUs' worth of threads over the CPUs the job's process had
        # before its NUMA binding (rank 0 alone runs this, after every GPU leg)
        nj = max(1, min(len(host_cpus), (cap or len(host_cpus)) * ws))
        quota = cpu_quota()
        if quota:                  # (a one-GPU box rehearsing N ranks has one GPU's quota)
            nj = max(1, min(nj, int(quota)))
        # the whole host: every CPU the process had, as far as the
        # cgroup quota lets threads run at once; only when that is more than the job's share
        nh = max(1, min(len(host_cpus), int(quota) if quota else len(host_cpus)))
        mine = os.sched_getaffinity(0)
        try:
            os.sched_setaffinity(0, host_cpus)
            out["job_share"] = leg(nj, f"the {ws}-GPU job's share of the host: {nj} of {os.cpu_count()} CPUs")
            if nh > nj:
                out["whole_host"] = leg(nh, f"every CPU the job may run on: {nh} of {os.cpu_count()} CPUs")
        finally:
            os.sched_setaffinity(0, mine)
        out["job_share"]["host_cpus"] = os.cpu_count()
        out["job_share"]["cpu_quota"] = quota
        if "whole_host" in out:
            out["whole_host"]["host_cpus"] = os.cpu_count()
            out["whole_host"]["cpu_quota"] = quota
    return out


def cpu_reference(tr: mosrx.Trace, key: str, seconds: float, process_packet: bool = False, forward: int = 0,
                  threads: int = 1):
    """mOS's own compiled functions on one host core, when the reference build
    travelled with the tree; else None.  A reported baseline, never the
    measured path.  Default: `mosref --time` = ref_frame, i.e. the header
    checks of eth_in.c / ip_in.c / tcp.c, ip_fast_csum, TCPCalcChecksum,
    GetRSSHash, GetRSSCPUCore per frame (the GPU record's scope).
    process_packet: `mosref --time-pp` = mOS's whole ProcessPacket per frame as
    the rx loop calls it (checks + checksums + FindStream on an empty flow
    table; no RSS, which the NIC computes in mOS).  forward: mos.conf `forward`
    under which ProcessPacket runs (1: its ForwardIPPacket / ForwardEthernetFrame
    calls are recorded by the harness, not transmitted).  threads > 1 (`--time`
    only): one pthread per disjoint slice of the trace, as mOS shards its frames
    over one mTCP thread per core (core.c:1369-1466)."""
    exe = os.path.join(ROOT, "oracle", "_ref", "mosref")
    if not os.access(exe, os.X_OK):
        return None
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import tempfile
    import pktlib
    with tempfile.TemporaryDirectory() as td:
        path = os.path.join(td, "trace.mrxt")
        pktlib.write_ref_trace(path, tr.frames[:tr.frames_bytes], tr.off, tr.len, forward=forward)
        try:
            cmd = [exe, "--time-pp" if process_packet else "--time", path, str(seconds)]
            if threads > 1 and not process_packet:
                cmd.append(str(threads))
            out = subprocess.run(cmd, capture_output=True, text=True, timeout=seconds + 60)
            r = json.loads(out.stdout.strip().splitlines()[-1])
        except (OSError, ValueError, IndexError, subprocess.TimeoutExpired):
            return None
    el = r["seconds"]
    what = (f"ProcessPacket per frame (oracle/_ref/mosref --time-pp; checks + checksums + FindStream, "
            f"no RSS; forward={forward}" + (": the Forward* calls recorded, not transmitted)" if forward else ")")
            if process_packet else
            "ip_fast_csum + TCPCalcChecksum + GetRSSHash + GetRSSCPUCore + header checks "
            "(oracle/_ref/mosref --time: ref_frame, not ProcessPacket)")
    nt = int(r.get("threads", 1))
    # every thread's frames over the longest thread's time (mosref reports the rate)
    return {"value": round(algo_bytes(tr, key) / tr.n * r["mpkts"] * 1e6 / 1e9, 3), "unit": "GB/s", "cores": nt,
            "kind": "reference", "mpkts": round(r["mpkts"], 3),
            "sample": f"{r['passes']} slice passes over one {tr.n}-frame batch ({el:.1f} s), mOS core/src {what}, "
                      f"{nt} thread(s)" + (" over disjoint slices" if nt > 1 else "")}


def cpu_baseline_row(tr: mosrx.Trace, key: str, min_s: float, O):
    """The oracle for a §8f row (flow hash / pkt_info / TX rewrite / BPF), one thread."""
    ab = algo_bytes(tr, key)
    progs = bpf_bench_programs() if "_bpf" in key else None
    reps, t0 = 0, time.perf_counter()
    while True:
        if key.endswith("_fh") or key.endswith("_ti"):
            O.classify_ex(tr.frames, tr.off, tr.len, O.params())
        elif key.endswith("_tx") or key.endswith("_txc"):
            O.tx_csum(tr.frames, tr.off, tr.len, mosrx.TX_IP_CSUM | mosrx.TX_TCP_CSUM)
        elif "_cls_bpf" in key:
            O.classify(tr.frames, tr.off, tr.len, O.params())
            O.bpf_eval(progs, tr.frames, tr.off, tr.len)
        else:
            O.bpf_eval(progs, tr.frames, tr.off, tr.len)
        reps += 1
        el = time.perf_counter() - t0
        if el >= min_s:
            break
    fn = ("mo_classify + mo_bpf_eval" if "_cls_bpf" in key else
          {"_fh": "mo_classify_ex", "_ti": "mo_classify_ex", "_tx": "mo_tx_csum", "txc": "mo_tx_csum",
           "bpf": "mo_bpf_eval"}[key[-3:]])
    return {"value": round(reps * ab / el / 1e9, 3), "unit": "GB/s", "cores": 1, "kind": "port",
            "mpkts": round(reps * tr.n / el / 1e6, 3),
            "sample": f"{reps} passes over one {tr.n}-frame batch ({el:.1f} s), oracle {fn}, 1 thread"}


MOS_CONF = """mos {{
	forward = {forward}
	netdev {{
		lo 0x0001
	}}
	mos_log = {log}/
	arp_table {{
		0.0.0.0/0 02:00:00:00:00:aa
	}}
	route_table {{
		0.0.0.0/0 lo
	}}
	nic_forward_table {{
		lo lo
	}}
	max_concurrency = 20000
	tcp_tw_interval = 0
	tcp_timeout = -1
}}
"""


def orphan_segments(n: int, size: int = 1460, seed: int = 3) -> mosrx.Trace:
    """`n` TCP data segments (ACK|PSH, `size` payload bytes) of 256 flows that
    never opened a connection: every one takes mOS's orphan path, so the
    per-frame cost left after the checks is small (no stream to track)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import pktlib
    rng = np.random.default_rng(seed)
    pay = rng.integers(0, 256, size, dtype=np.uint8).tobytes()
    frames = [pktlib.tcp_frame(f"10.1.{i % 256}.7", "192.168.7.7", 2000 + i % 256, 80, pay, flags=0x18,
                               seq=i * size) for i in range(n)]
    buf, off, ln = pktlib.pack_frames(frames)
    t = mosrx.Trace.__new__(mosrx.Trace)
    t.frames, t.off, t.len, t.n = buf, off, ln, n
    t.frames_bytes = int(off[-1]) + int(ln[-1])
    return t


def cpu_rx_loop_leg(tr: mosrx.Trace, loops: int, forward: int, reps: int = 5, timeout: float = 60.0,
                    exe: str | None = None, monitors: int = 1):
    """mOS's own rx loop on one host core (oracle/_ref/mos_app: mtcp_init, an
    mTCP thread in RunMainLoop, one stream monitor socket, gpu_module_func as
    the I/O module): the per-frame CPU time of core.c:902-907 (timed per batch)
    with mOS's ProcessPacket on every frame ("pp") and with csrc/mos_rx.c
    taking the checks from the GPU records ("gpu"), on the same frames,
    alternated `reps` times (medians, with min / max).  What mOS sends goes
    nowhere (MOSAPP_NO_TX: no pcap dump) and the time spent in get_wptr -- the
    TX buffer's flush to the source every 64 frames, the harness's sink -- is
    taken out of the figures (`*_excl_tx`; the raw ones are kept beside them).
    The difference is the CPU time per frame the GPU saves inside mOS.
    `monitors` 0: mOS with no monitor socket (no stream tracking, no
    callbacks: ProcessPacket plus the loop).  A reported baseline; None when
    the binary did not travel with the tree."""
    exe = exe or os.path.join(ROOT, "oracle", "_ref", "mos_app")
    if not os.access(exe, os.X_OK):
        return None
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import tempfile
    import pktlib
    ns = {"pp": [], "gpu": []}
    raw = {"pp": [], "gpu": []}
    frames = 0
    with tempfile.TemporaryDirectory() as td:
        trace = os.path.join(td, "t.mrxt")
        pktlib.write_ref_trace(trace, tr.frames[:tr.frames_bytes], tr.off, tr.len, forward=forward)
        for rep in range(reps):
            for mode in ("pp", "gpu"):
                d = os.path.join(td, f"{mode}{rep}")
                os.makedirs(os.path.join(d, "log"))
                conf = os.path.join(d, "mos.conf")
                with open(conf, "w") as fh:
                    fh.write(MOS_CONF.format(log=os.path.join(d, "log"), forward=forward))
                env = dict(os.environ, MOSAPP_QUIET="1", MOSAPP_LOOPS=str(loops), MOSAPP_BATCH="8192",
                           MOSAPP_NO_TX="1", MOSAPP_MONITORS=str(monitors))
                try:
                    r = subprocess.run([exe, mode, conf, trace, d], capture_output=True, text=True, timeout=timeout,
                                       env=env)
                    st = json.loads(r.stdout.strip().splitlines()[-1])
                except (OSError, ValueError, IndexError, subprocess.TimeoutExpired):
                    return None
                ns[mode].append(st["rx_ns_per_frame_excl_tx"])
                raw[mode].append(st["rx_ns_per_frame"])
                frames = st["rx_frames_timed"]
    pp, gp = float(np.median(ns["pp"])), float(np.median(ns["gpu"]))
    saved = [a - b for a, b in zip(ns["pp"], ns["gpu"])]           # per alternated pair
    return {"processpacket_ns_per_frame": round(pp, 1), "gpu_records_ns_per_frame": round(gp, 1),
            "saved_ns_per_frame": round(pp - gp, 1),
            "saved_ns_per_frame_pairs": {"median": round(float(np.median(saved)), 1),
                                         "min": round(min(saved), 1), "max": round(max(saved), 1)},
            "spread_ns": {k: [round(min(v), 1), round(max(v), 1)] for k, v in ns.items()},
            "frames": frames, "excluded": "get_wptr (TX buffer flushes), no TX dump",
            "runs_ns": {k: [round(x, 1) for x in v] for k, v in ns.items()},
            "runs_ns_incl_tx": {k: [round(x, 1) for x in v] for k, v in raw.items()},
            "sample": f"{tr.n} frames x {loops} through mOS's RunMainLoop on one core ({monitors} stream monitor(s), "
                      f"forward={forward}), oracle/_ref/mos_app pp vs gpu, {reps} alternated runs each, medians; "
                      f"TX flushes excluded"}


def measure_fw64(ctx, seconds: float):
    """BASELINE config #1: simple_firewall's rx path on ONE core, 10 000 x 60 B
    frames of one flow, the firewall's stack state (num_msp=1, forward=1,
    num_queues=1, i40e map).  The CPU baseline is the sample
    itself: mOS's samples/simple_firewall compiled unmodified over the ENABLE_GPU
    build with gpu_module_func replaying the trace (oracle/_ref/simple_firewall,
    cpu_simple_firewall below: its rx loop on one core with mOS's ProcessPacket,
    and with the GPU records); beside it mOS's own compiled per-frame functions
    (mosref --time), ProcessPacket alone and the oracle, all on one core, and the
    GPU classifying the same 10K batch."""
    tr = mosrx.Trace(mosrx.TRACE_FW64, 10_000)
    out = {"workload": "config #1: simple_firewall state, 1 core, 10k x 64B (60 B caplen), one flow",
           "batch": tr.n, "algo_bytes_per_batch": algo_bytes(tr)}
    ref = cpu_reference(tr, "FW64", seconds)
    port = cpu_baseline(tr, "FW64", min_s=seconds, shares=False)
    if ref:
        port["reference"] = ref
    # mOS's ProcessPacket itself in the firewall's state, forward = 1: every
    # segment of the flow takes the orphan path to ForwardIPPacket (tcp.c:507-510),
    # which the harness records instead of transmitting (no route / ARP tables)
    ref = cpu_reference(tr, "FW64", seconds, process_packet=True, forward=1)
    if ref:
        port["reference_processpacket"] = ref
    sf = cpu_simple_firewall()
    if sf:
        port["simple_firewall"] = sf
    out["cpu_baseline"] = port
    ctx.set_params(mosrx.default_params())
    db = ctx.upload(tr.frames, tr.off, tr.len, frames_bytes=tr.frames_bytes, max_len=tr.max_len)
    k = ctx.time_dev_streams([db], 500, 1) / 500
    db.free()
    out["gpu_device_resident"] = {"kernel_ms": k, "mpkts": tr.n / (k * 1e-3) / 1e6,
                                  "method": "500 back-to-back launches over the resident 10K batch"}
    out["e2e_boundary"] = measure_fw64_boundary(tr)
    return out


def cpu_simple_firewall(loops: int = 20, reps: int = 3, timeout: float = 120.0):
    """BASELINE config #1 through the reference's own application, on one core:
    mOS's samples/simple_firewall (unmodified, oracle/_ref/simple_firewall: the
    ENABLE_GPU build of INTEGRATION.md §2, gpu_module_func replaying a pcap file
    of config #1's 10K x 60 B trace and the rule flows of
    tests/test_simple_firewall.py, `loops` times), `-n 1`.  Per-frame CPU time of
    RunMainLoop's rx loop (core.c:902-907, timed per batch by oracle/sf_glue.c)
    with mOS's ProcessPacket on every frame ("pp": the reference's CPU path) and
    with the consumer of the GPU records ("gpu"), alternated `reps` times,
    medians.  A reported baseline; None when the binary did not travel."""
    exe = os.path.join(ROOT, "oracle", "_ref", "simple_firewall")
    if not os.access(exe, os.X_OK):
        return None
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import tempfile
    import pathlib
    import test_simple_firewall as SF
    frames = SF.firewall_frames()
    ns = {"pp": [], "gpu": []}
    with tempfile.TemporaryDirectory() as td:
        for rep in range(reps):
            for mode in ("pp", "gpu"):
                tmp = pathlib.Path(td) / f"r{rep}"
                tmp.mkdir(exist_ok=True)
                try:
                    r = SF.run_sample(exe, mode, tmp, frames, loops=loops, linger_ms=0)
                except (AssertionError, OSError, ValueError, subprocess.TimeoutExpired) as e:
                    print(f"[bench] simple_firewall leg failed: {str(e)[:300]}", file=sys.stderr)
                    return None
                ns[mode].append(r["result"]["rx_ns_per_frame"])
    pp, gp = float(np.median(ns["pp"])), float(np.median(ns["gpu"]))
    return {"value": round(1e3 / pp, 3), "unit": "Mpkt/s", "cores": 1, "kind": "reference",
            "processpacket_ns_per_frame": round(pp, 1), "gpu_records_ns_per_frame": round(gp, 1),
            "gpu_records_mpkts": round(1e3 / gp, 3),
            "runs_ns": {k: [round(x, 1) for x in v] for k, v in ns.items()},
            "sample": f"mOS samples/simple_firewall unmodified (-n 1) over gpu_module_func replaying "
                      f"{len(frames)} frames x {loops} (config #1's 10K x 60 B flow + rule flows), rx loop "
                      f"per-frame CPU time (core.c:902-907) with ProcessPacket (value) and with the GPU records, "
                      f"{reps} alternated runs, medians"}


def measure_fw64_boundary(tr: mosrx.Trace, loops: int = 50):
    """Config #1 end to end through the drop-in boundary on one host thread: the
    10K trace replayed from a pcap file by the libpcap-free pcap source,
    gpu_module_func in simple_firewall's state, RunMainLoop's rx loop with the
    ForwardEthernetFrame consumer sending every accepted frame out through the
    source's TX (a pcap dump).  libpcap and raw sockets are not available to the
    bench (no CAP_NET_RAW on the box), so the file stands in for the wire."""
    import tempfile
    with tempfile.TemporaryDirectory() as d:
        path, out = os.path.join(d, "fw.pcap"), os.path.join(d, "tx.pcap")
        with open(path, "wb") as fh:
            fh.write(struct.pack("<IHHiIII", 0xA1B2C3D4, 2, 4, 0, 0, 65535, 1))
            for i, (o, n) in enumerate(zip(tr.off.tolist(), tr.len.tolist())):
                fh.write(struct.pack("<IIII", i, 0, n, n) + bytes(tr.frames[o:o + n]))
        src = mosrx.lib().mosrx_source_pcap(path.encode(), loops)
        mosrx.source_tx_pcap(src, out)
        be = mosrx.GpuBackend([src], params=mosrx.default_params(), batch=tr.n, cpu=15, timing=True)
        try:
            fwd = be.forwarder([0])
            t0 = time.perf_counter()
            st = be.run_loop(forward=fwd)
            dt = time.perf_counter() - t0
            ms = be.stats()
        finally:
            be.close()
    return {"mpkts": st.rx_packets / dt / 1e6, "frames": int(st.rx_packets), "forwarded": int(fwd.forwarded),
            "seconds": round(dt, 3), "device_us_per_batch": round(1e3 * ms.kernel_ms / max(ms.kernel_launches, 1), 3),
            "method": f"pcap file ({loops} replays of the 10K trace) -> gpu_module_func (simple_firewall state) -> "
                      f"mosrx_rx_loop + mosrx_forward_frame -> source TX (pcap dump), one host thread"}


def measure_e2e(ctx, tr: mosrx.Trace, iters: int, sync=lambda: None):
    """End-to-end host->HBM->host rate (pinned staging, 2 slots); recorded in DESIGN.md.
    sync() brackets the timed region (the ranks' barrier in a multi-GPU job)."""
    ctx.set_params(mosrx.default_params())
    # one pinned staging block per slot, frames | off | len, the frames in the
    # gpu_module backend's staging layout (mosrx_source_fill: frames of up to
    # 128 bytes back to back): the library moves it over PCIe in one copy
    src = mosrx.mem_source(tr.frames, tr.off, tr.len, loops=1, mode=mosrx.SRC_FILL)
    mf = max(int(tr.max_len), 64)
    cap = tr.frames_bytes + 2 * mf + 4096      # the fill keeps a largest frame's room past its last frame
    staged = np.zeros(cap, np.uint8)
    soff = np.zeros(tr.n, np.uint32)
    slen = np.zeros(tr.n, np.uint16)
    end = C.c_uint64(0)
    got = mosrx.lib().mosrx_source_fill(src, staged.ctypes.data, cap, soff.ctypes.data, slen.ctypes.data, tr.n,
                                         mf, C.byref(end))
    mosrx.lib().mosrx_source_close(src)
    assert got == tr.n, got
    fb = int(end.value)
    fa = (fb + 15) & ~15
    bufs, outs, batches = [], [], []
    for _ in range(2):
        pb, ab = ctx.host_alloc(fa + tr.n * 6)
        ab[:fb] = staged[:fb]
        ab[fa:fa + tr.n * 4].view(np.uint32)[:] = soff
        ab[fa + tr.n * 4:].view(np.uint16)[:] = slen
        pr, _ = ctx.host_alloc(tr.n * 16)
        bufs += [pb, pr]
        outs.append(pr)
        # the staged 64 B frames sit at one stride (back to back): handed over with that hint
        batches.append(mosrx.with_hint(mosrx.Batch(pb, fb, pb + fa, pb + fa + tr.n * 4, tr.n, tr.max_len),
                                       mosrx.uniform_layout(soff) if HINT else None))
    ctx.time_host(batches, outs, 8)             # warm: both slots, pinned pages mapped
    sync()
    t0 = time.perf_counter()
    ms = ctx.time_host(batches, outs, iters)
    wall = time.perf_counter() - t0
    sync()
    for p in bufs:
        ctx.host_free(p)
    ab = algo_bytes(tr)
    return {"gbps": ab * iters / (ms * 1e-3) / 1e9, "mpkts": tr.n * iters / (ms * 1e-3) / 1e6,
            "ms_per_batch": ms / iters, "frames": tr.n * iters, "bytes": ab * iters, "seconds": wall,
            "method": "pinned hipHostMalloc staging (one block: frames | off | len, the backend's layout: "
                      "mosrx_source_fill), one H2D copy, kernel, D2H records; 2 streams"}


_BACKEND_TRACES = {}


def backend_trace(key: str, n: int) -> mosrx.Trace:
    """The backend legs' trace of n frames (generated once per size: the auto
    groups' traces are 1.3-2.3 GB)."""
    if (key, n) not in _BACKEND_TRACES:
        _BACKEND_TRACES[(key, n)] = mosrx.Trace({"S64": mosrx.TRACE_S64, "M1500": mosrx.TRACE_M1500,
                                                 "IMIX": mosrx.TRACE_IMIX}[key], n)
    return _BACKEND_TRACES[(key, n)]


def measure_backend(tr: mosrx.Trace, key: str, frames_target: int, cpu: int, group: int = 1, bpf=None,
                    compact: bool = True, sync=lambda: None, group_bytes: int = 0, group_max_us: int | None = None,
                    direct_kb: int | None = None):
    """The drop-in boundary's own rate: mosrx_rx_loop (RunMainLoop's rx section,
    core.c:897-909) over gpu_module_func (io_module.h:63-78) fed by an in-memory
    source replaying the trace — per group of batches: source -> pinned
    staging, H2D, ONE classify launch, D2H records, then the per-frame get_rptr
    + NETSTAT walk on the host, with the next group in flight while this one is
    consumed.  The kernels are timed by their dispatch-stamped durations (per batch);
    the host loop's rate is reported beside it.  Never the bench value."""
    ctx_batch = {"S64": 32_768, "M1500": 65_536, "IMIX": 262_144}[key]
    if group != 1:
        # a group's batches must be distinct frames: replaying one batch would let
        # the group's copy carry it once and the kernel re-read it from cache
        # (group 0 = the module's default, auto: as many batches per launch as are
        # ready, up to MOSRX_GROUP_AUTO_BYTES of frames -- ~500 of 64 B, 10 of 1500 B; more
        # distinct batches than a launch takes, so no launch holds the same frames twice)
        nb = group or {"S64": 640, "M1500": 20, "IMIX": 24}[key]
        tr = backend_trace(key, ctx_batch * nb)
    # warm-up (staging sized, module loaded): two launches' worth of frames, on top of
    # the timed part's frames_target
    warm = 2 * ctx_batch * (group or (512 if key == "S64" else 12))
    loops = max(1, -(-(frames_target + warm) // tr.n))
    src = mosrx.mem_source(tr.frames, tr.off, tr.len, loops=loops)
    cap = {} if group_max_us is None else {"group_max_us": group_max_us}
    if direct_kb is not None:
        cap["direct_kb"] = direct_kb
    be = mosrx.GpuBackend([src], batch=ctx_batch, max_frame=2048, pipeline=True, cpu=cpu, gpu_base=cpu,
                          group=group, timing=True, bpf=bpf, compact=compact, group_bytes=group_bytes, **cap)
    try:
        be.run_loop(max_pkts=warm)
        st0 = be.stats()
        sync()
        t0 = time.perf_counter()
        st = be.run_loop()
        dt = time.perf_counter() - t0
        sync()
        st1 = be.stats()
    finally:
        be.close()
    n = int(st.rx_packets)
    nb = n / tr.n
    launches = st1.kernel_launches - st0.kernel_launches
    kms = st1.kernel_ms - st0.kernel_ms
    batches = st1.rx_batches - st0.rx_batches
    dev_us = 1e3 * kms / max(batches, 1)
    # records: 8 bytes in compact mode (the module's configuration inside mOS), filters or not
    akey = ("_cls_bpf" if bpf else "") + ("_c8" if compact else "") if bpf else "c8" if compact else ""
    ab = algo_bytes(tr, akey) * (ctx_batch / tr.n)
    return {"mpkts": n / dt / 1e6, "gbps": nb * algo_bytes(tr, akey) / dt / 1e9, "frames": n,
            "bytes": int(nb * algo_bytes(tr, akey)),
            "seconds": dt, "filters": len(bpf) if bpf else 0,
            "records": 8 if compact else 16,
            "distinct_frames": tr.n,
            "group": group if group else "auto", "batches_per_launch": round(batches / max(launches, 1), 2),
            "kernel_launches": int(launches), "batches": int(batches),
            "direct_launches": int(st1.rx_direct_groups - st0.rx_direct_groups),
            "device_us_per_batch": round(dev_us, 3),
            "device_roofline_frac": round(ab / (dev_us * 1e-6) / 1e9 / HBM_PEAK_GBS, 4) if dev_us > 0 else None,
            "method": f"mosrx_rx_loop over gpu_module_func (pipelined, "
                      f"{group if group else 'auto (MOSRX_GROUP_AUTO)'} batch(es) per launch, "
                      f"{'8-byte records (cfg.compact)' if compact else '16-byte records'}"
                      f"{', ' + str(len(bpf)) + ' monitor filters installed: the fused classify + BPF queue kernel' if bpf else ''}), "
                      f"in-memory source replaying {tr.n} distinct frames; every batch crosses PCIe; device "
                      f"time = each kernel launch's dispatch-stamped duration (its frames were just copied in)"}


def measure_backend_latency(key: str, group: int, rate_mpkts: float, cpu: int, seconds: float = 0.6,
                            group_max_us: int = 0, warm_s: float = 0.15, direct_kb: int | None = None):
    """Per-frame residency on the drop-in path: the backend
    as measure_backend runs it (8-byte records, pipelined), fed by a paced source
    (mosrx_source_paced: frame k arrives at t0 + k / rate, none is handed out
    before it arrives, as a NIC ring fills at line rate) at `rate_mpkts`, the rx
    loop polling (idle_us 0, as mOS's poll-mode loop does) with the census
    consumer of the saturated legs.  Per frame: recv -> verdict available (its
    batch returned by recv_pkts with records) and recv -> consumed (that plus its
    share of the batch's walk), from the rx loop's probe (two clock reads per
    batch, mosrx_rx_loop_opts.probe) after `warm_s` of warm-up.  Never the bench
    value."""
    batch = {"S64": 32_768, "M1500": 65_536, "IMIX": 262_144}[key]
    kind = {"S64": mosrx.TRACE_S64, "M1500": mosrx.TRACE_M1500, "IMIX": mosrx.TRACE_IMIX}[key]
    tr = mosrx.Trace(kind, batch * {"S64": 64, "M1500": 4, "IMIX": 2}[key])
    rate = rate_mpkts * 1e6
    src = mosrx.paced_source(mosrx.mem_source(tr.frames, tr.off, tr.len, loops=0), rate)
    be = mosrx.GpuBackend([src], batch=batch, max_frame=2048, pipeline=True, cpu=cpu, gpu_base=cpu,
                          group=group, compact=True, group_max_us=group_max_us, direct_kb=direct_kb)
    probe = mosrx.LatencyProbe()
    probe.src = src
    probe.skip = int(rate * warm_s)
    try:
        t0 = time.perf_counter()
        st = be.run_loop(idle_rounds=0, idle_us=0, max_us=int((seconds + warm_s) * 1e6), probe=probe)
        dt = time.perf_counter() - t0
        ms = be.stats()
    finally:
        be.close()
    n = int(st.rx_packets)
    t0n, nspf, rel = C.c_uint64(), C.c_double(), C.c_uint64()
    out = {"offered_mpkts": round(rate_mpkts, 2), "delivered_mpkts": round(n / dt / 1e6, 2),
           "frames_recorded": int(probe.recorded),
           "avail_us": probe.percentiles("avail", (50, 99, 99.9)),
           "consumed_us": probe.percentiles("done", (50, 99, 99.9)),
           "avail_max_us": round(probe.avail_max_ns / 1e3, 1), "consumed_max_us": round(probe.done_max_ns / 1e3, 1),
           "groups": int(ms.rx_groups), "mean_group_frames": round(ms.rx_frames / max(ms.rx_groups, 1), 1),
           "max_group_frames": int(ms.max_group_frames), "group": group if group else "auto",
           "group_max_us": group_max_us, "direct_groups": int(ms.rx_direct_groups)}
    return out


def measure_backend_threads(key: str, nthreads: int, group: int, frames_per_thread: int, device: int):
    """mOS's per-core layout at the boundary: `nthreads` mTCP threads, each with
    its own context (core.c:1282-1349), its own source of distinct frames (as one
    PACKET_FANOUT socket per thread would be, mosrx_gpu_module_bind_source) and
    its own rx loop (mosrx_rx_loop_ex) on its own host thread, all on one GPU.
    Aggregate = frames of all threads / wall time from the common start to the
    last thread's end.  ctypes releases the GIL, so the loops run in parallel."""
    import ctypes as C
    import threading
    batch = {"S64": 32_768, "M1500": 65_536, "IMIX": 262_144}[key]
    kind = {"S64": mosrx.TRACE_S64, "M1500": mosrx.TRACE_M1500, "IMIX": mosrx.TRACE_IMIX}[key]
    traces = [mosrx.Trace(kind, batch * group, seed=0x51 + i) for i in range(nthreads)]
    L = mosrx.lib()
    m = mosrx.gpu_module()
    cfg = mosrx.ModuleCfg()
    L.mosrx_gpu_module_cfg_default(C.byref(cfg))
    srcs = [mosrx.mem_source(t.frames, t.off, t.len, loops=max(1, frames_per_thread // t.n)) for t in traces]
    cfg.num_ifs, cfg.src[0], cfg.batch, cfg.max_frame = 1, srcs[0], batch, 2048
    cfg.gpu_base, cfg.ngpu, cfg.pipeline, cfg.group = device, 1, 1, group
    mosrx._chk(L.mosrx_gpu_module_configure(C.byref(cfg)), "mosrx_gpu_module_configure")
    mosrx._VOIDFN(m.load_module_upper_half)()
    cpus = list(range(32, 32 + nthreads))
    objs = [C.c_uint64(0xFACE0000 + c) for c in cpus]
    ctxs = [C.addressof(o) for o in objs]
    stats = [mosrx.RxStats() for _ in cpus]
    rcs, ends = [None] * nthreads, [0.0] * nthreads
    try:
        for c, x, s in zip(cpus, ctxs, srcs):
            mosrx._chk(L.mosrx_gpu_module_bind(x, c), "mosrx_gpu_module_bind")
            mosrx._chk(L.mosrx_gpu_module_bind_source(c, 0, s), "mosrx_gpu_module_bind_source")
        for x in ctxs:
            mosrx._CTXFN(m.init_handle)(x)
        warm = mosrx.RxLoopOpts(2 * batch * group, 1, 0, 0)
        for i in range(nthreads):                 # staging sized, kernels loaded
            mosrx._chk(L.mosrx_rx_loop_ex(C.addressof(m), ctxs[i], 1, C.byref(warm), None, None,
                                          C.byref(mosrx.RxStats())), "mosrx_rx_loop_ex")
        opts = mosrx.RxLoopOpts(0, 1, 0, 0)
        go = threading.Barrier(nthreads + 1)

        def run(i):
            go.wait()
            rcs[i] = L.mosrx_rx_loop_ex(C.addressof(m), ctxs[i], 1, C.byref(opts), None, None, C.byref(stats[i]))
            ends[i] = time.perf_counter()

        th = [threading.Thread(target=run, args=(i,)) for i in range(nthreads)]
        for t in th:
            t.start()
        go.wait()
        t0 = time.perf_counter()
        for t in th:
            t.join(300)
        dt = max(ends) - t0
    finally:
        for x in ctxs:
            mosrx._CTXFN(m.destroy_handle)(x)
        for s in srcs:
            L.mosrx_source_close(s)
    if rcs != [0] * nthreads:
        raise RuntimeError(f"rx loops returned {rcs}")
    n = sum(int(s.rx_packets) for s in stats)
    ab = sum(algo_bytes(t) * int(s.rx_packets) / t.n for t, s in zip(traces, stats))
    return {"threads": nthreads, "group": group, "mpkts": round(n / dt / 1e6, 2), "gbps": round(ab / dt / 1e9, 2),
            "frames": n, "seconds": round(dt, 3),
            "per_thread_mpkts": [round(int(s.rx_packets) / (e - t0) / 1e6, 1) for s, e in zip(stats, ends)],
            "method": f"{nthreads} mTCP threads x (own context, own in-memory source of distinct frames, own "
                      f"mosrx_rx_loop_ex over gpu_module_func, {group} batch(es) per launch), one GPU"}


def main():
    global STREAMS, HINT
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--workloads", default=DEFAULT_WORKLOADS)
    ap.add_argument("--streams", type=int, default=STREAMS,
                    help="batches in flight for the one-launch-per-batch rows (1 = strictly serial launches)")
    ap.add_argument("--no-hint", action="store_true",
                    help="hand the resident batches over without their layout hint (A/B of MOSRX_BATCH_UNIFORM)")
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline legs")
    ap.add_argument("--no-e2e", action="store_true", help="skip the end-to-end (PCIe) and backend legs")
    ap.add_argument("--detail", default=os.path.join(ROOT, "gpurun_out", "bench_detail.json"),
                    help="where the full record (every row and leg) is written")
    args = ap.parse_args()
    STREAMS = args.streams
    if args.no_hint:
        HINT = None

    ws, rank, local = dist_env()
    if ws != args.gpus:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE {ws}", file=sys.stderr)
    dist = Dist(ws, rank)
    # MOSRX_BENCH_DEVICE pins every rank to one device: a rehearsal of the
    # multi-rank path on a one-GPU box, never a result
    device = int(os.environ.get("MOSRX_BENCH_DEVICE", local))
    # each rank on its GPU's NUMA node before its first GPU call (mOS binds
    # every mTCP thread to its core's node, cpu.c:56-87): the host side of the batches it
    # stages and waits for stays node-local
    host_cpus = os.sched_getaffinity(0) if hasattr(os, "sched_getaffinity") else None
    numa = mosrx.bind_to_gpu_node(device)
    ctx = mosrx.Context(device)
    keys = [k for k in args.workloads.split(",") if k]
    results, traces = {}, {}
    for k in keys:
        results[k], traces[k] = measure(ctx, dist, k, args.steps, args.warmup, rank)
        if rank == 0:
            r = results[k]
            print(f"[bench] {k}: {r['gbps']:.1f} GB/s {r['mpkts']:.1f} Mpkts/s "
                  f"kernel {r['kernel_ms']*1e3:.1f} us roofline {r['roofline']['frac']:.3f}",
                  file=sys.stderr, flush=True)
    e2e = None
    if not args.no_e2e and any(k in traces for k in ("M1500", "S64", "IMIX")):
        # every leg runs on every rank at once, between barriers (Dist.leg), each rank
        # on its own GPU and host thread; e2e[...] is this rank's figure (rank 0's in
        # the record), e2e["aggregate"][...] the job's: all ranks' frames over the
        # longest rank's wall time
        e2e, agg = {}, {}
        for k, iters in (("M1500", 60), ("S64", 800)):
            if k in traces:
                e2e[k], agg[k] = dist.leg(lambda sync: measure_e2e(ctx, traces[k], iters, sync))
                progress(f"e2e {k}: {e2e[k]['gbps']:.1f} GB/s {e2e[k]['mpkts']:.1f} Mpkt/s")
        # the gpu_module_func backend itself (host thread = this rank), the module's
        # configuration inside mOS: auto groups, 8-byte records (cfg.compact)
        # (frames through each leg: enough that the timed part holds several launches after the
        # warm-up's pipelined group -- an IMIX auto group is 3 batches of 100 MB)
        target = {"S64": 128_000_000, "M1500": 6_000_000, "IMIX": 40_000_000}
        be, be_agg = {}, {}
        legs = [(k, dict(frames_target=target[k], group=0)) for k in ("M1500", "S64", "IMIX")]
        legs += [("S64_rec16", dict(frames_target=128_000_000, group=0, compact=False)),   # 16-byte records
                 ("S64_group1", dict(frames_target=16_000_000, group=1)),      # one launch per batch
                 # auto groups of half the default bytes (256 MiB of frames per launch, round 4's default)
                 ("S64_auto512", dict(frames_target=64_000_000, group=0, group_bytes=512 << 20)),
                 ("S64_group128", dict(frames_target=32_000_000, group=128)),
                 # 8 monitor filters installed (mtcp_bind_monitor_filter): auto groups through the
                 # fused classify + BPF queue kernel's 8-byte-record (_c8) form, as without filters
                 ("S64_bpf", dict(frames_target=128_000_000, group=0, bpf=bpf_bench_programs())),
                 ("IMIX_bpf", dict(frames_target=40_000_000, group=0, bpf=bpf_bench_programs())),
                 ("S64_group8", dict(frames_target=32_000_000, group=8)),
                 ("M1500_group1", dict(frames_target=2_000_000, group=1)),
                 ("M1500_group8", dict(frames_target=4_000_000, group=8))]
        for name, kw in legs:
            k = name.split("_")[0]
            if k in traces:
                be[name], be_agg[name] = dist.leg(lambda sync: measure_backend(traces[k], k, cpu=device, sync=sync,
                                                                               **kw))
                progress(f"backend {name}: {be[name]['mpkts']:.1f} Mpkt/s, device frac "
                         f"{be[name]['device_roofline_frac']}, {be[name]['batches_per_launch']} batches per launch")
        _BACKEND_TRACES.clear()
        e2e["backend"] = be
        agg["backend"] = be_agg
        # per-frame residency on the drop-in path (paced arrivals at 25 / 50 / 90 % of each
        # configuration's saturated rate above; one GPU's host side: single-rank runs only)
        if ws == 1:
            lat = {}
            for k in ("S64", "M1500"):
                for g, name in ((0, k), (1, f"{k}_group1"), (8, f"{k}_group8")):
                    if name not in be:
                        continue
                    for load in (0.25, 0.5, 0.9):
                        r = lat[f"{name}@{int(load * 100)}"] = measure_backend_latency(k, g, load * be[name]["mpkts"],
                                                                                      cpu=device)
                        progress(f"latency {name} at {int(load * 100)} %: {r['delivered_mpkts']} Mpkt/s, avail "
                                 f"{r['avail_us']}")
            # the same light-load points with every group copied (cfg.direct_kb 0): what the
            # copy-free small groups gain, in the same run (the detail record only)
            for k, g, name in (("S64", 0, "S64"), ("M1500", 1, "M1500_group1")):
                if name in be:
                    r = lat[f"{name}@25_copied"] = measure_backend_latency(k, g, 0.25 * be[name]["mpkts"], cpu=device,
                                                                           direct_kb=0)
                    progress(f"latency {name} at 25 %, every group copied: avail {r['avail_us']}")
            e2e["backend_latency"] = lat
        e2e["aggregate"] = agg
        # one mTCP thread per core, each with its own context / source / rx loop
        # (one GPU's host side: single-rank runs only)
        if ws == 1:
            mt = {}
            if "S64" in traces:
                mt["S64"] = [measure_backend_threads("S64", t, 32, 32 * 2 ** 20, device) for t in (1, 2, 4, 8)]
            if "M1500" in traces:
                mt["M1500"] = [measure_backend_threads("M1500", t, 1, 2_000_000, device) for t in (1, 2, 4)]
            e2e["backend_threads"] = mt
            progress("backend threads: " + ", ".join(f"{k} {[r['mpkts'] for r in v]}" for k, v in mt.items()))
    # the last barrier of the GPU legs: from here rank 0 alone runs the host-core
    # baselines, with no other rank's timed region in flight, and the others wait
    dist.barrier()
    cpu = None
    if rank == 0 and not args.no_cpu:
        head = "M1500" if "M1500" in traces else keys[0]
        cpu = cpu_baseline(traces[head], head, min_s=10.0, ws=ws, host_cpus=host_cpus)
        progress(f"cpu baseline (port): {cpu['value']} GB/s on 1 core, "
                 f"{(cpu.get('per_gpu_share') or {}).get('value')} on one GPU's share")
        ref = cpu_reference(traces[head], head, 10.0)
        if ref:
            cpu["reference"] = ref
        # mOS's own code on one GPU's share of the host cores, beside
        # the port's per_gpu_share: one pthread per disjoint slice
        nt = cpu_share()[0]
        if nt > 1:
            ref = cpu_reference(traces[head], head, 10.0, threads=nt)
            if ref:
                ref["host_cpus"] = os.cpu_count()
                ref["cpu_quota"] = cpu_quota()
                cpu["reference_share"] = ref
        ref = cpu_reference(traces[head], head, 5.0, process_packet=True)
        if ref:
            cpu["reference_processpacket"] = ref
        progress("cpu baseline (mOS's own code) done")
        # mOS's whole rx loop with and without the GPU records (the CPU the GPU saves inside mOS)
        # 1500 B orphans under a monitor that forwards nothing: little besides the checks per frame
        rx = cpu_rx_loop_leg(orphan_segments(8192), 16, forward=0)
        if rx:
            cpu["mos_rx_loop_M1500"] = rx
        # config #1: simple_firewall's state (forward = 1), its one flow tracked as a stream
        rx = cpu_rx_loop_leg(mosrx.Trace(mosrx.TRACE_FW64, 10_000), 20, forward=1)
        if rx:
            cpu["mos_rx_loop_FW64"] = rx
        # the same frames through a bare mOS (no monitor: no stream tracking, no callbacks)
        rx = cpu_rx_loop_leg(mosrx.Trace(mosrx.TRACE_FW64, 10_000), 20, forward=1, monitors=0)
        if rx:
            cpu["mos_rx_loop_FW64_bare"] = rx
        progress("mOS rx-loop legs done")
        for k in keys:
            if k != head:
                results[k]["cpu_baseline"] = cpu_baseline(traces[k], k, min_s=2.0, shares=False)
                if k in ("S64", "IMIX"):
                    ref = cpu_reference(traces[k], k, 2.0)
                    if ref:
                        results[k]["cpu_baseline"]["reference"] = ref
        results["FW64"] = measure_fw64(ctx, 2.0)
        progress("config #1 (simple_firewall) legs done")
    read_ceiling = None
    if rank == 0:
        # the box's streaming-read rate over a >= 1.5 GB working set (no Infinity-
        # Cache hits), with 128 MiB launches (the single-batch rows' size: their ramp
        # and drain included) and 768 MiB launches (the ring rows' size, ~805 MB)
        read_ceiling = {"launch_128MiB": round(ctx.probe_read_bw(128 << 20, 12, 96), 1),
                        "launch_768MiB": round(ctx.probe_read_bw(768 << 20, 3, 48), 1)}
    ctx.close()
    dist.barrier()   # the other ranks wait here while rank 0 runs the host legs
    dist.close()
    if rank != 0:
        return
    head = "M1500" if "M1500" in results else keys[0]
    h = results[head]
    detail = {
        "metric": METRIC,
        "value": round(h["gbps"], 2),
        "unit": "GB/s",
        "mpkts_per_s": round(h["mpkts"], 2),
        "n_gpus": ws,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(h["ms_per_step"], 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (seeded splitmix64 traces, BASELINE.md §3; one job trace split round-robin over ranks)",
        "config": {"workload": h["workload"], "batch": h["batch"],
                   "batches_per_step": h["batches_per_step"],
                   "step": h["method"],
                   "algo_bytes_per_batch": h["algo_bytes_per_batch"],
                   "parallelism": f"replicas x{ws}: the job's batches round-robin per GPU (shard_plan), no collectives",
                   "resident_batches": h["resident_batches"],
                   "resident_bytes": h["resident_bytes"]},
        "roofline": h["roofline"],
        "read_probe_gbps": read_ceiling,
        "numa": numa,
        # the headline kernel's rate against the box's own streaming-read probe for
        # launches of the ring's size: a comparison with a simple read-only kernel, not a
        # ceiling (the classify kernel has read above it on some boxes)
        "vs_read_probe": (round(h["roofline"]["achieved"] / read_ceiling["launch_768MiB"], 4)
                                 if read_ceiling and read_ceiling.get("launch_768MiB") else None),
        "cpu_baseline": cpu,
        "secondary": {k: {kk: (round(vv, 4) if isinstance(vv, float) else vv) for kk, vv in r.items()}
                      for k, r in results.items() if k != head},
        "e2e": e2e,
    }
    # the full record (every row's method, the e2e / backend legs, CPU samples)
    # goes to a file and to stderr; stdout carries ONE compact headline line the
    # driver parses (round 2's 21 KB line was cut by the driver's stdout tail)
    path = args.detail
    try:
        os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
        with open(path, "w") as fh:
            json.dump(detail, fh, indent=1)
    except OSError as e:
        print(f"[bench] could not write {path}: {e}", file=sys.stderr)
    print("[bench-detail] " + json.dumps(detail), file=sys.stderr, flush=True)
    print(json.dumps(headline_line(detail, h, head, results, e2e)), flush=True)


def _compact_cpu(c):
    """One CPU baseline leg without its nested legs, sample text shortened."""
    if not c:
        return None
    out = {k: c[k] for k in ("value", "unit", "cores", "kind", "mpkts") if k in c}
    out["sample"] = c.get("sample", "")[:120]
    return out


def headline_line(detail, h, head, results, e2e):
    """The driver's record: the contract's fields, roofline, cpu_baseline and a
    short per-row summary.  Kept well under 4 KB."""
    rf = h["roofline"]
    cpu = detail["cpu_baseline"]
    cpu_line = None
    if cpu:
        cpu_line = _compact_cpu(cpu)
        for leg in ("per_gpu_share", "job_share", "whole_host", "reference", "reference_share",
                    "reference_processpacket"):
            if cpu.get(leg):
                # (host_cpus / cpu_quota once, on the per-GPU share; every leg's in the detail record)
                keys = ("value", "unit", "cores", "kind", "mpkts") + (
                    ("host_cpus", "cpu_quota") if leg == "per_gpu_share" else ())
                cpu_line[leg] = {k: cpu[leg][k] for k in keys if k in cpu[leg]}
        for leg in ("mos_rx_loop_M1500",):   # (config #1's rx-loop legs: the detail record and FW64 below)
            if cpu.get(leg):
                cpu_line[leg] = {k: cpu[leg][k] for k in ("processpacket_ns_per_frame", "gpu_records_ns_per_frame",
                                                          "saved_ns_per_frame")}
    sec = {}
    for k, r in results.items():
        if k == head:
            continue
        if k == "FW64":
            cb = r.get("cpu_baseline") or {}
            sec[k] = {"gpu_mpkts": round(r["gpu_device_resident"]["mpkts"], 1),
                      "cpu_port_mpkts": cb.get("mpkts"),
                      "cpu_ref_processpacket_mpkts": (cb.get("reference_processpacket") or {}).get("mpkts"),
                      "cpu_simple_firewall_mpkts": (cb.get("simple_firewall") or {}).get("value"),
                      "simple_firewall_gpu_records_mpkts": (cb.get("simple_firewall") or {}).get("gpu_records_mpkts"),
                      "boundary_mpkts": round(r["e2e_boundary"]["mpkts"], 2)}
            continue
        # [Mpkt/s, launch us, roofline frac]; GB/s and the per-rank spread: the detail record
        sec[k] = [round(r["mpkts"], 1), round(r["roofline"]["launch_us"], 2), round(r["roofline"]["frac"], 3)]
        if "stamp_floor_us" in r["roofline"]:
            sec[k].append(round(r["roofline"]["stamp_floor_us"], 2))
    e2e_line = None
    if e2e:
        e2e_line = {k: {"gbps": round(v["gbps"], 1), "mpkts": round(v["mpkts"], 1)}
                    for k, v in e2e.items() if k in ("M1500", "S64")}
        be = e2e.get("backend") or {}
        e2e_line["backend"] = {k: {"mpkts": round(v["mpkts"], 1), "dev_frac": v.get("device_roofline_frac")}
                               for k, v in be.items()
                               if k not in ("S64_group128", "M1500_group8", "S64_auto512", "S64_group8")}
        # the job's end-to-end rates: every rank's legs at once, all frames over the longest wall
        # (at N = 1 the same as the rank's own)
        ag = e2e.get("aggregate") if detail["n_gpus"] > 1 else None
        ag = ag or {}
        if ag:
            e2e_line["aggregate"] = {k: {kk: v[kk] for kk in ("ranks", "mpkts", "gbps", "per_rank_mpkts")}
                                     for k, v in ag.items() if k in ("M1500", "S64")}
            e2e_line["aggregate"]["backend"] = {k: {kk: v[kk] for kk in ("mpkts", "per_rank_mpkts")}
                                                for k, v in (ag.get("backend") or {}).items()
                                                if k in ("M1500", "S64", "IMIX")}
        if e2e.get("consumer"):
            e2e_line["consumer"] = e2e["consumer"]
        if e2e.get("backend_latency"):
            # recv -> verdict available, p50 / p99 us, at 25 / 50 / 90 % of the saturated rate
            # (groups of 8: the detail record)
            e2e_line["latency_fields"] = ("offered Mpkt/s, recv->verdict p50 us, p99 us (detail: consumed, groups "
                                          "of 8, every group copied)")
            e2e_line["latency"] = {k: [round(v["offered_mpkts"], 1), round(v["avail_us"].get("p50_us", 0)),
                                       round(v["avail_us"].get("p99_us", 0))]
                                   for k, v in e2e["backend_latency"].items()
                                   if "group8" not in k and "copied" not in k}
    return {
        "metric": detail["metric"],
        "value": detail["value"],
        "unit": detail["unit"],
        "mpkts_per_s": detail["mpkts_per_s"],
        "n_gpus": detail["n_gpus"],
        "steps": detail["steps"],
        "warmup": detail["warmup"],
        "ms_per_step": detail["ms_per_step"],
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (seeded splitmix64 traces, BASELINE.md §3)",
        "config": {"workload": h["workload"], "batch": h["batch"], "batches_per_step": h["batches_per_step"],
                   "algo_bytes_per_batch": h["algo_bytes_per_batch"],
                   "parallelism": detail["config"]["parallelism"]},
        "roofline": {k: rf[k] for k in ("bound", "achieved", "peak", "unit", "frac", "traffic", "launch_us",
                                         "launch_timing")},
        "per_rank_device_gbps": h["per_rank_device_gbps"],
        "read_probe_gbps": detail["read_probe_gbps"],
        "vs_read_probe": detail["vs_read_probe"],
        "cpu_baseline": cpu_line,
        "secondary_fields": "Mpkt/s, launch us, frac[, 1-launch rows: empty-kernel stamp us]",
        "secondary": sec,
        "e2e": e2e_line,
        "detail": "full record: stderr line '[bench-detail]' and --detail file",
    }


if __name__ == "__main__":
    main()
