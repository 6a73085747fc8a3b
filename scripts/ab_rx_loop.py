"""A/B of two builds of the mOS harness (oracle/_ref/mos_app*) on bench.py's
rx-loop CPU legs (diagnostic): per-frame CPU time of RunMainLoop's rx section
with ProcessPacket and with the consumer on the GPU records, alternating the
builds `rounds` times.  Usage: python3 scripts/ab_rx_loop.py A_exe B_exe [rounds]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "mos-networking-stack_amd"))
import bench  # noqa: E402
import mosrx  # noqa: E402

exes = [os.path.abspath(a) for a in sys.argv[1:3]]
rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 3
legs = {"M1500": (bench.orphan_segments(8192), 16, 0), "FW64": (mosrx.Trace(mosrx.TRACE_FW64, 10_000), 20, 1)}
for r in range(rounds):
    for exe in exes:
        out = {"exe": os.path.basename(exe)}
        for k, (tr, loops, fwd) in legs.items():
            leg = bench.cpu_rx_loop_leg(tr, loops, fwd, reps=2, exe=exe)
            out[k] = None if leg is None else {"pp": leg["processpacket_ns_per_frame"],
                                               "gpu": leg["gpu_records_ns_per_frame"]}
        print(json.dumps(out), flush=True)
