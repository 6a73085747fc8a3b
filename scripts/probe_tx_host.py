"""The host TX pass (mosrx_tx_csum_host) with the checks coming back as 8-byte
records (default) against round 3's pass that copies the rewritten frames
back (MOSRX_TX_HOST_INPLACE=1): milliseconds per batch (diagnostic).

    python3 scripts/probe_tx_host.py
"""
import os, subprocess, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mos-networking-stack_amd"))
import mosrx

if len(sys.argv) > 1:   # child: one mode
    ctx = mosrx.Context(0)
    for kind, n, name in ((mosrx.TRACE_M1500, 65536, "1500 B x 64K"), (mosrx.TRACE_IMIX, 262144, "IMIX x 256K"),
                          (mosrx.TRACE_S64, 32768, "64 B x 32K")):
        t = mosrx.Trace(kind, n)
        # the frames in pinned memory, as gpu_module_func's TX buffer is (cfg.tx_csum)
        ptr, arr = ctx.host_alloc(t.frames_bytes + 64)
        arr[:t.frames_bytes] = t.frames[:t.frames_bytes]
        off = np.ascontiguousarray(t.off, np.uint32)
        ln = np.ascontiguousarray(t.len, np.uint16)
        b = mosrx.Batch(ptr, t.frames_bytes, off.ctypes.data, ln.ctypes.data, n, 0)
        run = lambda: mosrx.lib().mosrx_tx_csum_host(ctx.handle, mosrx.C.byref(b), mosrx.TX_IP_CSUM | mosrx.TX_TCP_CSUM)  # noqa: E731
        for _ in range(5):
            assert run() == 0
        ts = []
        for _ in range(30):
            t0 = time.perf_counter()
            run()
            ts.append(time.perf_counter() - t0)
        print(f"{sys.argv[1]:8s} {name:14s} {1e3 * np.median(ts):7.3f} ms per batch "
              f"({t.frames_bytes / np.median(ts) / 1e9:5.1f} GB/s of frames)", flush=True)
    sys.exit(0)
for mode, env in (("records", {}), ("inplace", {"MOSRX_TX_HOST_INPLACE": "1"})):
    subprocess.run([sys.executable, os.path.abspath(__file__), mode], env=dict(os.environ, **env), check=True)
