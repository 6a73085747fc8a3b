"""The real-clock consumer scenario (round 3's soak seed 7, setup 3), run N times
with the filter set installed asynchronously (the backend's default) and N
times with the old synchronous install (MOSRX_BPF_SYNC=1: the mTCP thread
waits for hipRTC), each with comgr's compile cache on and off, printing per run whether the frames sent agree with
ProcessPacket's run, the ARP requests each sent, and the longest filter
install (diagnostic, not a test).

    python3 scripts/repro_real_clock.py [gpu|emul] [runs=3]
"""
import os, sys, tempfile, pathlib
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for d in ("tests", "mos-networking-stack_amd"):
    sys.path.insert(0, os.path.join(ROOT, d))
import pktlib, test_mos_consumer as T
exe = T.APP if len(sys.argv) < 2 or sys.argv[1] == "gpu" else T.APP_EMUL
runs = int(sys.argv[2]) if len(sys.argv) > 2 else 3
sc = T.SCENARIOS["real_clock_seed7_setup3"]
fr = pktlib.conversation_frames(sc["nflows"], seed=sc["seed"], listen_port=sc["listen"])
# AMD_COMGR_CACHE=0: every hipRTC compile cold, as on a fresh box (comgr caches compiled
# code objects under ~/.cache/comgr; a cold fused compile takes seconds)
for mode, extra in (("async", {}), ("sync", {"MOSRX_BPF_SYNC": "1"}),
                    ("async, cold compile", {"AMD_COMGR_CACHE": "0"}),
                    ("sync, cold compile", {"MOSRX_BPF_SYNC": "1", "AMD_COMGR_CACHE": "0"})):
    for r in range(runs):
        with tempfile.TemporaryDirectory() as td:
            tmp = pathlib.Path(td)
            pp = T.run_app(exe, "pp", tmp, "r", sc, fr)
            gpu = T.run_app(exe, "gpu", tmp, "r", sc, fr, extra)
            st = gpu["stats"]
            print(f"{mode} run {r}: tx {'equal' if gpu['tx'] == pp['tx'] else 'DIFFER'} "
                  f"({len(gpu['tx'])} vs {len(pp['tx'])} frames), ARP requests gpu {st['arp_sent']} "
                  f"pp {pp['stats']['arp_sent']}, first difference {T.first_diff(gpu['tx'], pp['tx'])}, "
                  f"returns {'equal' if gpu['returns'] == pp['returns'] else 'DIFFER'}, "
                  f"longest filter install {st['max_filter_sync_ns'] / 1e6:.2f} ms, "
                  f"installs {st['filter_installs']}", flush=True)
