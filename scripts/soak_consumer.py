"""Soak of the mOS verdict consumer (diagnostic, not a test).

    python3 scripts/soak_consumer.py [seconds=300] [seed=1] [emul|gpu|asan]

Random setups of tests/test_mos_consumer.py's harness (oracle/_ref/mos_app:
mOS itself, mtcp_init + RunMainLoop over gpu_module_func) until the time is
up: conversation traces of random size and seed (with or without flows to a
local listener; some with the reference's golden fixture frames mixed in),
forward 0/1, 0-2 stream monitors, raw / SYN / orphan BPF filters, a listener, a monitor or raw filter appearing mid-trace, frames per
batch and batches per launch, resolving ARP with mOS's own TX checksums taken
by the GPU (cfg.tx_csum, clock frozen), the flow lookup on the GPU hash or on
mOS's.  Each setup runs mOS twice -- ProcessPacket, then the consumer on the
GPU records -- and every per-frame return, NETSTAT, callback, the flow table
and every frame sent must agree.  "emul" (default) runs the CPU stand-in for
the GPU (oracle/_ref/mos_app_emul), "gpu" the real kernels, "asan" the
stand-in with the host code under AddressSanitizer + UBSan.  A mismatch
prints the setup and exits 1.
"""
import os
import random
import sys
import tempfile
import time
import pathlib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mos-networking-stack_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import pktlib  # noqa: E402
import test_mos_consumer as T  # noqa: E402


def setup(rnd):
    env = {}
    listen = 0
    if rnd.random() < 0.3:
        listen = rnd.choice([80, 8080])
        env["MOSAPP_LISTEN"] = str(listen)
    env["MOSAPP_MONITORS"] = str(rnd.choice([0, 1, 1, 1, 2]))
    if rnd.random() < 0.3:
        env["MOSAPP_RAW"] = rnd.choice(["tcp port 80", "tcp[tcpflags] & tcp-syn != 0", "tcp and ip[8] > 32"])
    elif rnd.random() < 0.2:
        env["MOSAPP_RAW_NOFILTER"] = "1"
    if rnd.random() < 0.25 and env["MOSAPP_MONITORS"] != "0":
        env["MOSAPP_SYN"] = rnd.choice(["tcp port 80 or tcp port 443", "tcp port 8080"])
        env["MOSAPP_ORPHAN"] = rnd.choice(["net 10.9.0.0/16", "src net 10.0.0.0/8"])
    if rnd.random() < 0.15 and "MOSAPP_RAW" in env:
        env["MOSAPP_LATE_RAW_AT"] = str(rnd.randint(1, 300))
    if rnd.random() < 0.15 and env["MOSAPP_MONITORS"] == "0":
        env["MOSAPP_LATE_MON_AT"] = str(rnd.randint(1, 300))
    env["MOSAPP_BATCH"] = str(rnd.choice([17, 61, 97, 512, 4096]))
    env["MOSAPP_GROUP"] = str(rnd.choice([0, 1, 2, 3]))
    if rnd.random() < 0.2:
        env["MOSAPP_FLOWHASH"] = "0"
    sc = dict(forward=rnd.randint(0, 1), env=env, listen=listen, nflows=rnd.choice([8, 64, 200]),
              seed=rnd.randint(1, 1 << 30))
    if rnd.random() < 0.3:
        sc["arp_all"] = True
        env["MOSAPP_FROZEN_CLOCK"] = "1"
        if rnd.random() < 0.7:
            sc["gpu_env"] = {"MOSAPP_TX_CSUM": "1"}
    return sc


def describe(pp, gpu):
    """What differs, for the record: per-frame returns, the frames sent (count, ARP
    requests, ethertypes of the first differing pair), the longest filter install."""
    rp, rg = pp["returns"], gpu["returns"]
    bad = [i for i, (a, b) in enumerate(zip(rp, rg)) if a != b]
    print(f"  returns: {len(bad)} frames differ, first {bad[:8]}", flush=True)
    tp, tg = pp["tx"], gpu["tx"]
    arp = lambda fs: sum(1 for f in fs if f[12:14] == b"\x08\x06")  # noqa: E731
    print(f"  sent: {len(tg)} (gpu) vs {len(tp)} (pp) frames; ARP requests {arp(tg)} vs {arp(tp)}; "
          f"first difference (index, ethertypes) {T.first_diff(tg, tp)}", flush=True)
    for k in ("max_filter_sync_ns", "filter_installs", "reclassified", "gpu_errors", "arp_sent"):
        print(f"  {k}: gpu {gpu['stats'].get(k)} pp {pp['stats'].get(k)}", flush=True)


def main():
    budget = float(sys.argv[1]) if len(sys.argv) > 1 else 300.0
    seed = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    mode = sys.argv[3] if len(sys.argv) > 3 else "emul"
    exe = {"gpu": T.APP, "asan": T.ASAN_APP}.get(mode, T.APP_EMUL)
    if mode == "asan":      # the host-side sanitizer build (make -C oracle asan)
        os.environ["ASAN_OPTIONS"] = "detect_leaks=0:verify_asan_link_order=0:halt_on_error=1"
        os.environ["UBSAN_OPTIONS"] = "print_stacktrace=1:halt_on_error=1"
    rnd = random.Random(seed)
    fixtures = {fix: T.fixture_frames(fix) for fix in ("edge", "rand_small", "rand_mid")}
    t0 = last = time.time()
    count = frames = 0
    while time.time() - t0 < budget:
        sc = setup(rnd)
        name = f"s{count}"
        T.SCENARIOS[name] = sc
        fr = pktlib.conversation_frames(sc["nflows"], seed=sc["seed"], listen_port=sc["listen"])
        if rnd.random() < 0.3:     # the reference's golden fixture frames mixed in at random places
            extra = [f for fix in ("edge", "rand_small", "rand_mid") for f in fixtures[fix]]
            for f in rnd.sample(extra, k=rnd.randint(1, 60)):
                fr.insert(rnd.randint(0, len(fr)), f)
        with tempfile.TemporaryDirectory() as td:
            tmp = pathlib.Path(td)
            try:
                pp = T.run_app(exe, "pp", tmp, name, sc, fr)
                gpu = T.run_app(exe, "gpu", tmp, name, sc, fr, sc.get("gpu_env"))
                assert gpu["returns"] == pp["returns"], "per-frame return values"
                assert gpu["state"] == pp["state"], "flow table / NETSTAT"
                assert gpu["callbacks"] == pp["callbacks"], "callbacks"
                assert gpu["tx"] == pp["tx"], "frames sent"
                assert gpu["stats"]["consumer_frames"] == len(fr)
            except AssertionError as e:
                print(f"FAIL setup {count}: {sc}: {str(e)[:2000]}", flush=True)
                describe(pp, gpu)
                sys.exit(1)
        del T.SCENARIOS[name]
        count += 1
        frames += len(fr)
        if time.time() - last > 10:
            last = time.time()
            print(f"[soak] {count} setups, {frames} frames, {last - t0:.0f} s", flush=True)
    print(f"[soak] OK: {count} setups, {frames} frames in {time.time() - t0:.0f} s "
          f"(seed {seed}, {os.path.basename(exe)})", flush=True)


if __name__ == "__main__":
    main()
