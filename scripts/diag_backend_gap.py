"""Why does the drop-in backend run the classify kernel slower than the
device-resident rows?  One phase per process, so each
runs alone under `rocprofv3 --kernel-trace` and its trace holds only its own
dispatches.  Every phase prints the dispatch-stamped median of its timed
launches; the kernel traces give the same launches' real durations.

  res_b2b    device-resident, back-to-back launches (the bench rows)
  res_gapN   device-resident, N ms of host sleep + sync before each launch
             (the backend's duty cycle: the GPU idles while the host walks)
  res_fresh  device-resident, the batch's frames re-copied over PCIe
             (pinned, synchronous) right before each launch
  be_g1 / be_auto   the backend itself (gpu_module_func + mosrx_rx_loop)

Usage: python3 scripts/diag_backend_gap.py {M1500|S64} PHASE"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "mos-networking-stack_amd"))
import numpy as np  # noqa: E402
import bench  # noqa: E402
import mosrx  # noqa: E402

key, phase = sys.argv[1], sys.argv[2]
# M1500c8: the 1500 B batch with 8-byte records (the backend's compact form)
compact = key != "M1500"
key = key.replace("c8", "")
kind, batch = {"M1500": (mosrx.TRACE_M1500, 65_536), "S64": (mosrx.TRACE_S64, 32_768)}[key]
# the backend's launch shape: M1500 one batch per launch (group 1); S64 its auto
# group (~238 batches of frames packed back to back, 8-byte records)
group = 1 if key == "M1500" else 238
akey = "c8" if compact else ""


def report(name, us):
    us = np.asarray(us, dtype=np.float64)
    tr = mosrx.Trace(kind, batch)
    ab = bench.algo_bytes(tr, akey) * group
    med = float(np.median(us))
    print(f"{key} {name}: n={len(us)} median {med:.2f} us (p10 {np.percentile(us, 10):.2f}, p90 "
          f"{np.percentile(us, 90):.2f}) per launch of {group} batch(es); frac {ab / (med * 1e-6) / 1e9 / 8000:.3f}",
          flush=True)


if phase.startswith("be_"):
    tr = mosrx.Trace(kind, batch)
    kw = dict(frames_target=2_000_000, group=1) if key == "M1500" else dict(frames_target=64_000_000, group=0)
    r = bench.measure_backend(tr, key, cpu=0, **kw)
    print(f"{key} {phase}: {r['kernel_launches']} launches, {r['batches_per_launch']} batches/launch, device "
          f"{r['device_us_per_batch']:.3f} us/batch, frac {r['device_roofline_frac']}, {r['mpkts']:.1f} Mpkt/s",
          flush=True)
    sys.exit(0)

ctx = mosrx.Context(0)
if key == "M1500":
    trs = [mosrx.Trace(kind, batch, seed=bench.job_seed(kind, b)) for b in range(12)]   # 1.2 GB distinct
    dbs = [ctx.upload(t.frames, t.off, t.len, frames_bytes=t.frames_bytes, max_len=t.max_len) for t in trs]
    qs = [ctx.queue_ex(dbs[i:i + 1], compact=compact) for i in range(len(dbs))]
else:
    trs = [bench.pack_uniform(mosrx.Trace(kind, batch, seed=bench.job_seed(kind, b))) for b in range(8)]
    dbs = [ctx.upload(t.frames, t.off, t.len, frames_bytes=t.frames_bytes, max_len=t.max_len)
           for t in (trs[i % 8] for i in range(2 * group))]
    qs = [ctx.queue_ex(dbs[i:i + group], compact=True) for i in range(0, 2 * group, group)]
bench.prewarm(lambda: qs[0].time(8, qs[1:], kernels=False), 0.5)
watch = None
if os.environ.get("MOSRX_DPM_WATCH"):   # sample the DPM clock levels through the phase (read-only sysfs)
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import dpm_watch  # noqa: E402
    watch = dpm_watch.Watch().start()
    watch.label = "prewarmed"
    time.sleep(0.05)
    watch.label = phase
us = []
if phase == "res_b2b":
    for _ in range(5):
        us.append(1e3 * qs[0].time_dispatch(100, qs[1:]))
elif phase.startswith("res_gap"):
    gap = float(phase[len("res_gap"):]) * 1e-3
    for i in range(60):
        time.sleep(gap)
        us.append(1e3 * qs[i % len(qs)].time_dispatch(1))
elif phase.startswith("res_fresh"):
    # res_fresh: the batch's frames copied in again over PCIe (pinned source) right
    # before every launch; res_fresh_other: the same copies into a spare buffer the
    # launch does not read (DMA activity, not the data it wrote); res_fresh_sleep10:
    # into the batch, 10 ms before the launch
    pins = []
    for t in trs:
        p, a = ctx.host_alloc(len(t.frames))
        a[:] = t.frames
        pins.append((p, a))
    spare = [mosrx.DevBuffer(ctx, len(t.frames)) for t in trs] if phase == "res_fresh_other" else None
    copy_s = 0.0
    for i in range(60 if key == "M1500" else 20):
        j = i % len(qs)
        t_c = time.perf_counter()
        for b in range(group):
            k = (j * group + b) % len(pins)
            dst = spare[k] if spare else dbs[j * group + b].d_frames
            if phase.endswith("_pull"):      # copied by the CUs (mosrx_memcpy_h2d_pull), not the SDMA engine
                mosrx._chk(mosrx.lib().mosrx_memcpy_h2d_pull(ctx.handle, dst.ptr, pins[k][0], len(pins[k][1])), "pull")
            else:
                dst.upload(pins[k][1])
        copy_s += time.perf_counter() - t_c
        if phase == "res_fresh_sleep10":
            time.sleep(0.01)
        us.append(1e3 * qs[j].time_dispatch(1))
    nb = sum(len(pins[(jj * group + b) % len(pins)][1]) for jj in range(60 if key == "M1500" else 20)
             for b in range(group))
    print(f"{key} {phase}: copies {nb / copy_s / 1e9:.1f} GB/s (host-timed, synchronous)", flush=True)
    for p, _ in pins:
        ctx.host_free(p)
    for d in spare or []:
        d.free()
elif phase in ("res_dma_hostpages", "res_dma_devpages"):
    # which side's pages: 100 MB of distinct pinned host pages copied into one 1 MB
    # device buffer (hostpages), or one 1 MB host buffer copied into 100 MB of distinct
    # device pages (devpages), before every launch
    L = mosrx.lib()
    mb, nmb = 1 << 20, 100
    p, a = ctx.host_alloc(mb * nmb)
    a[:] = 1
    dev = mosrx.DevBuffer(ctx, mb * (nmb if phase == "res_dma_devpages" else 1))
    for i in range(60 if key == "M1500" else 20):
        j = i % len(qs)
        for c in range(nmb):
            if phase == "res_dma_hostpages":
                mosrx._chk(L.mosrx_memcpy_h2d(ctx.handle, dev.ptr, p + c * mb, mb), "h2d")
            else:
                mosrx._chk(L.mosrx_memcpy_h2d(ctx.handle, dev.ptr + c * mb, p, mb), "h2d")
        us.append(1e3 * qs[j].time_dispatch(1))
    dev.free()
    ctx.host_free(p)
else:
    raise SystemExit(f"unknown phase {phase}")
report(phase, us)
if watch is not None:
    watch.label = "after"
    time.sleep(0.05)
    watch.stop()
    import json  # noqa: E402
    print(f"{key} {phase} dpm: {json.dumps(watch.report())}", flush=True)
for q in qs:
    q.destroy()
for d in dbs:
    d.free()
ctx.close()
