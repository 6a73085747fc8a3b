#!/usr/bin/env python3
"""bench.py — device-resident throughput of the MI355X rx classifier.

One "step" = one pass of the hot path (mOS ProcessPacket checks + ip_fast_csum
+ TCPCalcChecksum + Toeplitz RSS / queue map) over one batch per GPU, inputs
already resident in HBM.  The headline workload is BASELINE config #3
(1500 B MTU TCP segments, 1M flows, batch 64K) whose GB/s the north star
prices against the HBM roofline; the same run also measures config #2
(64 B, 1 flow, batch 32K; Mpkts/s) and config #4 (IMIX, batch 256K).

Multi-GPU (torchrun, one process per GPU): batches are split round-robin over
the GPUs with no collective on the data path (`scaling: weak`); gloo carries
only the barrier and the max-over-ranks of the timed region.

Each rank cycles over several copies of its batch at distinct HBM addresses so
the working set exceeds the 256 MiB Infinity Cache: every timed pass reads HBM.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W]
"""
from __future__ import annotations

import argparse
import json
import os
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
L3_BYTES = 256 << 20

WORKLOADS = {
    # key: (trace kind, batch, label)
    "M1500": (mosrx.TRACE_M1500, 65_536, "1xMI355X 1500B MTU TCP segments, 1M distinct 5-tuples, batch=64K (BASELINE config #3)"),
    "S64": (mosrx.TRACE_S64, 32_768, "1xMI355X 64B TCP, 1 flow, batch=32K (BASELINE config #2), full verdict"),
    "S64_hdr": (mosrx.TRACE_S64, 32_768, "config #2 header parse + IP cksum + RSS only (skip_tcp_csum)"),
    "IMIX": (mosrx.TRACE_IMIX, 262_144, "IMIX 60/590/1514 7:4:1, 1M flows, batch=256K (BASELINE config #4)"),
    "S64_queue": (mosrx.TRACE_S64, 32_768, "config #2, 64 batches of 32K per launch (device batch queue)"),
    "M1500_queue": (mosrx.TRACE_M1500, 65_536, "config #3, 4 batches of 64K per launch (device batch queue)"),
    # SURVEY.md §8f rows measured on the same traces
    "M1500_fh": (mosrx.TRACE_M1500, 65_536, "config #3 classify + flow-table hash (HashFlow of FindStream's tuple)"),
    "M1500_tx": (mosrx.TRACE_M1500, 65_536, "config #3 TX checksum rewrite (MOS_UPDATE_IP|TCP_CHKSUM), in place"),
    "IMIX_bpf": (mosrx.TRACE_IMIX, 262_144, "config #4 batched BPF, 8 mOS filter programs (sfbpf_compile output)"),
    "IMIX_cls_bpf": (mosrx.TRACE_IMIX, 262_144, "config #4 classify + the 8 BPF programs fused in one pass"),
}
OPS = {"M1500_fh": mosrx.OP_CLASSIFY_FH, "M1500_tx": mosrx.OP_TX_CSUM, "IMIX_bpf": mosrx.OP_BPF,
       "IMIX_cls_bpf": mosrx.OP_CLASSIFY_BPF}
# filter expressions whose compiled programs (tests/golden/bpf.npz, mOS's own compiler) the BPF row runs
BPF_BENCH = [("tcp", 0), ("tcp port 80", 0), ("tcp[tcpflags] & tcp-syn != 0", 1), ("net 192.168.0.0/16 and tcp", 1),
             ("host 10.0.0.1 and port 80", 0), ("ip[8] < 64", 1), ("tcp[((tcp[12:1] & 0xf0) >> 2):4] = 0x47455420", 1),
             ("portrange 1000-2000", 0)]
QUEUE_DEPTH = {"S64_queue": 64, "M1500_queue": 4}   # resident batches per queue launch
PREWARM_S = 0.3
STREAMS = 2   # rx batches in flight per GPU (scripts/tune_streams.py: 2 beats 1 and 4)


def dist_env():
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    return ws, rank, local


class Dist:
    """Barrier + max-reduce over ranks (gloo, CPU); nothing on the data path."""

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

    def close(self):
        if self.ws > 1:
            self.dist.destroy_process_group()


def algo_bytes(tr: mosrx.Trace, key: str = "") -> int:
    """B_i = caplen_i + 6 (offset+len descriptor) + 16 (result record).
    Flow hash: + 4 B per frame.  TX rewrite: caplen + 6 read, 4 B written (no records).
    BPF: the 6-byte descriptor + 4-byte mask + 64 header bytes per frame (the
    line a filter reads; deeper loads are extra)."""
    if key.endswith("_tx"):
        return tr.caplen_sum + tr.n * (DESC_BYTES + 4)
    if key.endswith("_cls_bpf"):   # the classify bytes + the 4-byte match mask
        return tr.caplen_sum + tr.n * (DESC_BYTES + RESULT_BYTES + 4)
    if key.endswith("_bpf"):
        return tr.n * (DESC_BYTES + 4) + int(np.minimum(tr.len, 64).astype(np.int64).sum())
    extra = 4 if key.endswith("_fh") else 0
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


def measure(ctx, dist, key, steps, warmup, rank):
    kind, batch, label = WORKLOADS[key]
    params = mosrx.default_params(skip_tcp_csum=1 if key == "S64_hdr" else 0)
    ctx.set_params(params)
    # rank r owns the batches b = r, r+N, ... of the job's round-robin split; the
    # synthetic content differs per rank (seed), the shape does not.
    tr = mosrx.Trace(kind, batch, seed=0 if rank == 0 else 0x6D4F5321 + kind + 1000 * rank)
    ncopy = max(2, -(-2 * L3_BYTES // max(tr.frames_bytes, 1)))
    ncopy = min(max(ncopy, 2 * QUEUE_DEPTH.get(key, 1)), 256)
    dbs = [ctx.upload(tr.frames, tr.off, tr.len, frames_bytes=tr.frames_bytes, max_len=tr.max_len)
           for _ in range(ncopy)]
    ab = algo_bytes(tr, key)
    if key in OPS:
        op = OPS[key]
        arg = mosrx.TX_IP_CSUM | mosrx.TX_TCP_CSUM if op == mosrx.OP_TX_CSUM else 0
        if op in (mosrx.OP_BPF, mosrx.OP_CLASSIFY_BPF):
            ctx.bpf_set(bpf_bench_programs())
        prewarm(lambda: ctx.time_op(op, dbs, 200, STREAMS, arg, kernels=False))
        if warmup:
            ctx.time_op(op, dbs, warmup, STREAMS, arg, kernels=False)
        ctx.device_sync()
        dist.barrier()
        t0 = time.perf_counter()
        dev_ms, _ = ctx.time_op(op, dbs, steps, STREAMS, arg, kernels=False)
        ctx.device_sync()
        dist.barrier()
        wall = time.perf_counter() - t0
        wall_max = dist.max(wall)
        kk = 500
        kern_ms = median_of(lambda: ctx.time_op(op, dbs, kk, 1, arg, kernels=False)[0] / kk)
        _, kern_iso = ctx.time_op(op, dbs, kk, 1, arg, total=False)
    elif key.endswith("_queue"):
        # each step = one launch over `depth` distinct resident batches
        depth = QUEUE_DEPTH[key]
        # several queues over disjoint batch copies: the working set exceeds the L3
        qs = [ctx.queue(dbs[i:i + depth]) for i in range(0, len(dbs) - depth + 1, depth)]
        ab *= depth
        batch *= depth
        prewarm(lambda: qs[0].time(20, qs[1:], kernels=False))
        if warmup:
            qs[0].time(warmup, qs[1:], kernels=False)
        ctx.device_sync()
        dist.barrier()
        t0 = time.perf_counter()
        dev_ms, _ = qs[0].time(steps, qs[1:], kernels=False)
        ctx.device_sync()
        dist.barrier()
        wall = time.perf_counter() - t0
        wall_max = dist.max(wall)
        kk = min(steps, 64)
        kern_ms = median_of(lambda: qs[0].time(kk, qs[1:], kernels=False)[0] / kk)
        _, kern_iso = qs[0].time(kk, qs[1:])
        for q in qs:
            q.destroy()
    else:
        # warmup (untimed)
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
        dist.barrier()
        wall = time.perf_counter() - t0
        wall_max = dist.max(wall)
        # roofline: average launch duration on ONE stream, HIP events around
        # 500 back-to-back launches on the launch stream (the figure rocprofv3's
        # kernel trace reports), median of 5 such runs; the isolated figure
        # (events around each single launch, dispatch included) is kept beside it
        kk = 500
        kern_ms = median_of(lambda: ctx.time_dev_streams(dbs, kk, 1) / kk)
        kern_iso = ctx.time_dev_kernels(dbs, kk)
    for d in dbs:
        d.free()
    n = dist.ws
    out = {
        "workload": label,
        "batch": batch,
        "frames_bytes_per_batch": tr.frames_bytes,
        "algo_bytes_per_batch": ab,
        "resident_copies": ncopy,
        "wall_s": wall_max,
        "ms_per_step": 1e3 * wall_max / steps,
        "gbps": n * ab * steps / wall_max / 1e9,
        "mpkts": n * batch * steps / wall_max / 1e6,
        "device_ms_per_batch": dev_ms / steps,
        "kernel_ms": kern_ms,
        "kernel_ms_isolated": kern_iso,
    }
    achieved = ab / (kern_ms * 1e-3) / 1e9
    pmc = load_pmc(key)
    out["roofline"] = {
        "bound": "hbm",
        "achieved": round(achieved, 1),
        "peak": HBM_PEAK_GBS,
        "unit": "GB/s",
        "frac": round(achieved / HBM_PEAK_GBS, 4),
        "traffic": (pmc or {}).get("hbm_bytes_per_launch"),
    }
    if pmc:
        out["roofline"]["traffic_source"] = pmc.get("source")
    return out, tr


def cpu_baseline(tr: mosrx.Trace, key: str, min_s: float = 3.0):
    """The oracle (bit-exact C restatement, oracle/mosrx_oracle.c) on this host's cores.

    Reported baseline only; never the measured product path."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_py as O
    p = O.params(skip_tcp_csum=1 if key == "S64_hdr" else 0)
    ab = algo_bytes(tr, key)
    cores_avail = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
    cores_all = max(1, min(16, cores_avail))

    if key in OPS:
        return cpu_baseline_row(tr, key, min_s, O)

    def run(nt):
        reps, t0 = 0, time.perf_counter()
        while True:
            O.classify(tr.frames, tr.off, tr.len, p, nthreads=nt)
            reps += 1
            el = time.perf_counter() - t0
            if el >= min_s:
                return reps, el

    r1, e1 = run(1)
    rn, en = run(cores_all)
    model = ""
    try:
        with open("/proc/cpuinfo") as fh:
            model = next((ln.split(":", 1)[1].strip() for ln in fh if ln.startswith("model name")), "")
    except OSError:
        pass
    gb1, gbn = r1 * ab / e1 / 1e9, rn * ab / en / 1e9
    return {
        "value": round(gb1, 3), "unit": "GB/s", "cores": 1, "kind": "port",
        "mpkts": round(r1 * tr.n / e1 / 1e6, 3),
        "sample": f"{r1} passes over one {tr.n}-frame batch of this workload ({e1:.1f} s), "
                  f"oracle/mosrx_oracle.c mo_classify, 1 thread; host '{model}', nproc {os.cpu_count()}",
        "all_cores": {"value": round(gbn, 3), "unit": "GB/s", "cores": cores_all,
                      "mpkts": round(rn * tr.n / en / 1e6, 3),
                      "sample": f"{rn} passes, {cores_all} pthreads over disjoint slices ({en:.1f} s)"},
    }


def cpu_reference(tr: mosrx.Trace, key: str, seconds: float):
    """mOS's own compiled functions (oracle/_ref/mosref --time: the header checks,
    ip_fast_csum, TCPCalcChecksum, GetRSSHash, GetRSSCPUCore per frame) on one
    host core, when the reference build travelled with the tree; else None.
    A reported baseline beside the port, never the measured path."""
    exe = os.path.join(ROOT, "oracle", "_ref", "mosref")
    if not os.access(exe, os.X_OK):
        return None
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import tempfile
    import pktlib
    with tempfile.TemporaryDirectory() as td:
        path = os.path.join(td, "trace.mrxt")
        pktlib.write_ref_trace(path, tr.frames[:tr.frames_bytes], tr.off, tr.len)
        try:
            out = subprocess.run([exe, "--time", path, str(seconds)], capture_output=True, text=True,
                                 timeout=seconds + 60)
            r = json.loads(out.stdout.strip().splitlines()[-1])
        except (OSError, ValueError, IndexError, subprocess.TimeoutExpired):
            return None
    el = r["seconds"]
    return {"value": round(algo_bytes(tr, key) * r["passes"] / el / 1e9, 3), "unit": "GB/s", "cores": 1,
            "kind": "reference", "mpkts": round(r["mpkts"], 3),
            "sample": f"{r['passes']} passes over one {tr.n}-frame batch ({el:.1f} s), mOS core/src "
                      f"ip_fast_csum + TCPCalcChecksum + GetRSSHash + GetRSSCPUCore + header checks "
                      f"(oracle/_ref/mosref --time), 1 thread"}


def cpu_baseline_row(tr: mosrx.Trace, key: str, min_s: float, O):
    """The oracle for a §8f row (flow hash / TX rewrite / BPF), one thread."""
    ab = algo_bytes(tr, key)
    progs = bpf_bench_programs() if key.endswith("_bpf") else None
    reps, t0 = 0, time.perf_counter()
    while True:
        if key.endswith("_fh"):
            O.classify_fh(tr.frames, tr.off, tr.len, O.params())
        elif key.endswith("_tx"):
            O.tx_csum(tr.frames, tr.off, tr.len, mosrx.TX_IP_CSUM | mosrx.TX_TCP_CSUM)
        elif key.endswith("_cls_bpf"):
            O.classify(tr.frames, tr.off, tr.len, O.params())
            O.bpf_eval(progs, tr.frames, tr.off, tr.len)
        else:
            O.bpf_eval(progs, tr.frames, tr.off, tr.len)
        reps += 1
        el = time.perf_counter() - t0
        if el >= min_s:
            break
    fn = ("mo_classify + mo_bpf_eval" if key.endswith("_cls_bpf") else
          {"_fh": "mo_classify_fh", "_tx": "mo_tx_csum", "bpf": "mo_bpf_eval"}[key[-3:]])
    return {"value": round(reps * ab / el / 1e9, 3), "unit": "GB/s", "cores": 1, "kind": "port",
            "mpkts": round(reps * tr.n / el / 1e6, 3),
            "sample": f"{reps} passes over one {tr.n}-frame batch ({el:.1f} s), oracle {fn}, 1 thread"}


def measure_e2e(ctx, tr: mosrx.Trace, iters: int):
    """End-to-end host->HBM->host rate (pinned staging, 2 slots); recorded in DESIGN.md."""
    ctx.set_params(mosrx.default_params())
    # one pinned staging block per slot, frames | off | len (as the gpu_module
    # backend stages a batch): the library moves it over PCIe in one copy
    fb = tr.frames_bytes
    fa = (fb + 15) & ~15
    bufs, outs, batches = [], [], []
    for _ in range(2):
        pb, ab = ctx.host_alloc(fa + tr.n * 6)
        ab[:fb] = tr.frames[:fb]
        ab[fa:fa + tr.n * 4].view(np.uint32)[:] = tr.off
        ab[fa + tr.n * 4:].view(np.uint16)[:] = tr.len
        pr, _ = ctx.host_alloc(tr.n * 16)
        bufs += [pb, pr]
        outs.append(pr)
        batches.append(mosrx.Batch(pb, fb, pb + fa, pb + fa + tr.n * 4, tr.n, tr.max_len))
    ctx.time_host(batches, outs, 8)             # warm: both slots, pinned pages mapped
    ms = ctx.time_host(batches, outs, iters)
    for p in bufs:
        ctx.host_free(p)
    ab = algo_bytes(tr)
    return {"gbps": ab * iters / (ms * 1e-3) / 1e9, "mpkts": tr.n * iters / (ms * 1e-3) / 1e6,
            "ms_per_batch": ms / iters,
            "method": "pinned hipHostMalloc staging (one block: frames | off | len), one H2D copy, kernel, D2H records; 2 streams"}


def measure_backend(tr: mosrx.Trace, key: str, frames_target: int, cpu: int):
    """The drop-in boundary's own rate: mosrx_rx_loop (RunMainLoop's rx section,
    core.c:897-909) over gpu_module_func (io_module.h:63-78) fed by an in-memory
    source replaying the trace — per batch: source -> pinned staging, H2D,
    classify, D2H records, then the per-frame get_rptr + NETSTAT walk on the
    host, with batch k+1 in flight while k is consumed.  Recorded in DESIGN.md;
    never the bench value."""
    ctx_batch = {"S64": 32_768, "M1500": 65_536, "IMIX": 262_144}[key]
    loops = max(1, frames_target // tr.n)
    src = mosrx.mem_source(tr.frames, tr.off, tr.len, loops=loops)
    be = mosrx.GpuBackend([src], batch=ctx_batch, max_frame=2048, pipeline=True, cpu=cpu, gpu_base=cpu)
    try:
        be.run_loop(max_pkts=2 * ctx_batch)            # warm-up: staging sized, module loaded
        t0 = time.perf_counter()
        st = be.run_loop()
        dt = time.perf_counter() - t0
    finally:
        be.close()
    n = int(st.rx_packets)
    nb = n / tr.n
    return {"mpkts": n / dt / 1e6, "gbps": nb * algo_bytes(tr) / dt / 1e9, "frames": n, "seconds": round(dt, 3),
            "method": "mosrx_rx_loop over gpu_module_func (pipelined), in-memory source replaying the trace"}


def main():
    global STREAMS
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--warmup", type=int, default=100)
    ap.add_argument("--workloads",
                    default="M1500,S64,S64_hdr,S64_queue,M1500_queue,IMIX,M1500_fh,M1500_tx,IMIX_bpf,IMIX_cls_bpf")
    ap.add_argument("--streams", type=int, default=STREAMS,
                    help="rx batches in flight (1 = strictly serial launches, as for rocprof summaries)")
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg")
    ap.add_argument("--no-e2e", action="store_true", help="skip the end-to-end (PCIe) leg")
    args = ap.parse_args()
    STREAMS = args.streams

    ws, rank, local = dist_env()
    if ws != args.gpus:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE {ws}", file=sys.stderr)
    dist = Dist(ws, rank)
    # MOSRX_BENCH_DEVICE pins every rank to one device: a rehearsal of the
    # multi-rank path on a one-GPU box (scripts/gpu_r1_dist.sh), never a result
    device = int(os.environ.get("MOSRX_BENCH_DEVICE", local))
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
    if not args.no_e2e and "M1500" in traces:
        e2e = {k: measure_e2e(ctx, traces[k], {"M1500": 60, "S64": 800}[k]) for k in ("M1500", "S64") if k in traces}
        # the gpu_module_func backend itself (host thread = this rank)
        e2e["backend"] = {k: measure_backend(traces[k], k, {"S64": 16_000_000, "M1500": 2_000_000}.get(k, 4_000_000), device)
                          for k in ("M1500", "S64", "IMIX") if k in traces}
    cpu = None
    if rank == 0 and ws == 1 and not args.no_cpu:
        head = "M1500" if "M1500" in traces else keys[0]
        cpu = cpu_baseline(traces[head], head, min_s=10.0)
        ref = cpu_reference(traces[head], head, 10.0)
        if ref:
            cpu["reference"] = ref
        for k in keys:
            if k != head:
                results[k]["cpu_baseline"] = cpu_baseline(traces[k], k, min_s=2.0)
                if k in ("S64", "IMIX"):
                    ref = cpu_reference(traces[k], k, 2.0)
                    if ref:
                        results[k]["cpu_baseline"]["reference"] = ref
    ctx.close()
    dist.close()
    if rank != 0:
        return
    head = "M1500" if "M1500" in results else keys[0]
    h = results[head]
    line = {
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
        "data": "synthetic (seeded splitmix64 traces, BASELINE.md §3)",
        "config": {"workload": h["workload"], "batch": h["batch"],
                   "algo_bytes_per_batch": h["algo_bytes_per_batch"],
                   "parallelism": f"replicas x{ws}: batches round-robin per GPU, no collectives",
                   "streams_per_gpu": STREAMS,
                   "resident_copies": h["resident_copies"]},
        "roofline": h["roofline"],
        "cpu_baseline": cpu,
        "secondary": {k: {kk: (round(vv, 4) if isinstance(vv, float) else vv) for kk, vv in r.items()}
                      for k, r in results.items() if k != head},
        "e2e": e2e,
    }
    print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
