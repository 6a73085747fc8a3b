"""mOS running with the GPU verdicts: csrc/mos_rx.c against mOS's own ProcessPacket.

oracle/_ref/mos_app is mOS itself -- mtcp_init from a mos.conf, an mTCP thread
in RunMainLoop, monitor sockets with callbacks and BPF filters, an end-host
listener -- with gpu_module_func as its I/O module and everything it sends
going out through the backend's TX into a pcap dump.  RunMainLoop's per-frame
call (core.c:906) goes either to mOS's ProcessPacket ("pp": every check on
the CPU) or to mosrx_mos_process_packet ("gpu": the checks' outcome from the
GPU records, eth_in.c / ip_in.c / tcp.c side effects reproduced, then the
stream step of tcp.c:445-514).  Both runs of a scenario must agree on
everything mOS does: each frame's return value, NETSTAT, every callback with
the packet it saw, the flow table after the last frame, and every frame sent
(forwards, RSTs, ICMP replies).

The CPU leg runs oracle/_ref/mos_app_emul, the same program over a stand-in
for the GPU (oracle/gpu_emul.c: the oracle makes the records); the GPU leg
runs the real kernels.  Scenarios cover forward 0/1 (simple_firewall runs
with 1), stream monitors with and without SYN / orphan filters, raw monitors
with and without a filter (filters evaluated on the GPU from the match
masks), an end-host listener (RSTs for orphans), no socket at all (nothing
verified, everything forwarded), a filter bound and a monitor created in the
middle of a batch (the batch classified again), and batches of 1..N per
launch -- over conversation traces, and over the frames of the reference's
golden fixtures.
"""
import os
import struct
import subprocess

import pytest

import pktlib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = os.path.join(ROOT, "oracle", "_ref")
APP = os.path.join(REF, "mos_app")
APP_EMUL = os.path.join(REF, "mos_app_emul")
# the builds and record forms every scenario runs in: the consumer restating
# tcp.c's static stream functions, with 8-byte records (the module's default in
# an mOS build) and with 16-byte ones; and the consumer calling mOS's own
# functions under the upstream patch of INTEGRATION.md §2b (mos_app_x)
FORMS = {"c8": ("", {}), "rec16": ("", {"MOSAPP_COMPACT": "0"}), "tcp_exports": ("_x", {})}

CONF = """mos {{
	forward = {forward}
	netdev {{
		lo 0x0001
	}}
	mos_log = {log}/
	arp_table {{
{arp}
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

# mOS's GetDestinationHWaddr (arp.c:89-119) never picks a /0 entry (it wants a prefix
# longer than 0) and reads prefix 1 as an exact address, so the default table
# resolves nothing: frames mOS builds itself wait for ARP and only forwarded ones
# leave.  Four /2 entries resolve every address, so mOS sends its own RSTs / ACKs.
ARP_NONE = "\t\t0.0.0.0/0 02:00:00:00:00:aa"
ARP_ALL = "\n".join(f"\t\t{a}.0.0.0/2 02:00:00:00:00:aa" for a in (0, 64, 128, 192))

SCENARIOS = {
    # simple_firewall's stack: one stream monitor, forward = 1 (setup.sh:135)
    "monitor_fwd": dict(forward=1, env={}),
    "monitor_nofwd": dict(forward=0, env={}),
    "filters": dict(forward=1, env={"MOSAPP_RAW": "tcp port 80", "MOSAPP_SYN": "tcp port 80 or tcp port 443",
                                    "MOSAPP_ORPHAN": "net 10.9.0.0/16"}),
    "two_monitors_raw": dict(forward=1, env={"MOSAPP_MONITORS": "2", "MOSAPP_RAW_NOFILTER": "1"}),
    "listener": dict(forward=1, env={"MOSAPP_LISTEN": "8080"}, listen=8080),
    # mOS's TX checksums taken by the backend as a NIC offload (dev_ioctl PKT_TX_*_CSUM,
    # dpdk_module.c:556-566) and filled on the GPU at send_pkts, in the GPU run only: the
    # frames sent must equal those of the ProcessPacket run, whose checksums mOS computed
    "listener_tx_csum": dict(forward=1, env={"MOSAPP_LISTEN": "8080", "MOSAPP_FROZEN_CLOCK": "1"}, listen=8080,
                             arp_all=True,
                             gpu_env={"MOSAPP_TX_CSUM": "1"}),
    "listener_arp": dict(forward=1, env={"MOSAPP_LISTEN": "8080", "MOSAPP_FROZEN_CLOCK": "1"}, listen=8080,
                         arp_all=True),
    "no_socket": dict(forward=1, env={"MOSAPP_MONITORS": "0"}),
    "late_filter": dict(forward=1, env={"MOSAPP_RAW": "tcp[tcpflags] & tcp-syn != 0", "MOSAPP_LATE_RAW_AT": "150"}),
    "late_monitor": dict(forward=1, env={"MOSAPP_MONITORS": "0", "MOSAPP_LATE_MON_AT": "200"}),
    "batch_1_per_launch": dict(forward=1, env={"MOSAPP_GROUP": "1", "MOSAPP_BATCH": "97"}),
    "groups_of_3": dict(forward=1, env={"MOSAPP_GROUP": "3", "MOSAPP_BATCH": "61"}),
    # FindStream through HTSearch's own hash instead of the GPU's bucket (the default)
    "cpu_flow_hash": dict(forward=1, env={"MOSAPP_FLOWHASH": "0"}),
    # 600 conversations (~6K frames) in batches of 512, automatic groups of several batches
    "many_flows": dict(forward=1, env={"MOSAPP_BATCH": "512", "MOSAPP_RAW": "tcp and ip[8] > 32"}, nflows=600),
    # the reference fixtures' frames (tests/golden/make_golden.py: the ihl 0..4 quirk, IP / TCP
    # options up to 15 words, ICMP, mutation-fuzzed frames at odd and even alignments)
    "golden_edge_fwd": dict(forward=1, env={"MOSAPP_RAW_NOFILTER": "1"}, fixture="edge"),
    "golden_edge_nofwd": dict(forward=0, env={}, fixture="edge"),
    "golden_edge_listener": dict(forward=1, env={"MOSAPP_LISTEN": "80"}, fixture="edge"),
    "golden_edge_listener_tx_csum": dict(forward=1, env={"MOSAPP_LISTEN": "80", "MOSAPP_FROZEN_CLOCK": "1"},
                                         fixture="edge", arp_all=True,
                                         gpu_env={"MOSAPP_TX_CSUM": "1"}),
    "golden_rand_small_fwd": dict(forward=1, env={"MOSAPP_ORPHAN": "src net 10.0.0.0/8"}, fixture="rand_small"),
    "golden_rand_mid_fwd": dict(forward=1, env={"MOSAPP_BATCH": "37", "MOSAPP_GROUP": "2"}, fixture="rand_mid"),
    "golden_rand_large_nofwd": dict(forward=0, env={}, fixture="rand_large"),
    # round 3's consumer soak, seed 7, setup 3 (scripts/soak_consumer.py), with mOS's wall clock
    # running: forward 0, a listener (RSTs need ARP, unresolved: mOS sends ARP requests, and
    # ARPTimer, arp.c:313-327, retires a request after 1 s), a raw monitor, SYN and orphan filters
    # (bound before the first frame: the first filter evaluation installs them on the GPU).  The
    # ARP requests mOS sends depend on how long the run takes, so the filter install must not
    # stall the mTCP thread (the set is in effect at once, its hipRTC compile runs behind)
    "real_clock_seed7_setup3": dict(forward=0, env={"MOSAPP_LISTEN": "80", "MOSAPP_MONITORS": "1",
                                                    "MOSAPP_RAW_NOFILTER": "1", "MOSAPP_SYN": "tcp port 8080",
                                                    "MOSAPP_ORPHAN": "net 10.9.0.0/16", "MOSAPP_BATCH": "4096",
                                                    "MOSAPP_GROUP": "2"},
                                    listen=80, nflows=64, seed=1000704748, real_clock=True),
    # a raw monitor's program freed mid-trace (as FreeMonListener does, socket.c:33-36) and a
    # filter of the same length bound in its place, usually at the same address: the GPU's set
    # must follow the programs, not their addresses
    "reopen_filter": dict(forward=1, env={"MOSAPP_RAW": "tcp port 80", "MOSAPP_RAW2": "tcp port 443",
                                          "MOSAPP_REOPEN_RAW_AT": "333", "MOSAPP_BATCH": "97"}),
}


def fixture_frames(fix):
    """The fixture's frames, less those mOS's harness skipped in any state (headers
    claiming bytes past the capture: ProcessPacket reads past its buffer there)
    and those longer than 1514 B: a monitor's callback reading the packet
    (mtcp_getlastpkt) copies it into a 1514 B buffer (mos_api.c:422-430, the
    length assert compiled out), so mOS overruns it in either mode."""
    import numpy as np
    z = np.load(os.path.join(ROOT, "tests", "golden", f"{fix}.npz"))
    skip = np.zeros(len(z["off"]), bool)
    for k in z.files:
        if k.endswith("__have"):
            skip |= (z[k] & 8) != 0
    fr = z["frames"]
    skip |= z["len"] > 1514
    return [bytes(fr[int(o):int(o) + int(n)]) for o, n, s in zip(z["off"], z["len"], skip) if not s]


def pcap_frames(path):
    """The frames of a classic pcap file (record timestamps are wall time: left out)."""
    raw = open(path, "rb").read()
    out, pos = [], 24
    while pos + 16 <= len(raw):
        _, _, incl, _ = struct.unpack("<IIII", raw[pos:pos + 16])
        out.append(raw[pos + 16:pos + 16 + incl])
        pos += 16 + incl
    return out


def run_app(exe, mode, tmp, name, sc, frames, extra_env=None):
    d = tmp / f"{name}_{mode}"
    d.mkdir()
    log = tmp / f"{name}_{mode}_log"
    log.mkdir()
    conf = tmp / f"{name}_{mode}.conf"
    conf.write_text(CONF.format(forward=sc["forward"], log=log, arp=ARP_ALL if sc.get("arp_all") else ARP_NONE))
    trace = tmp / f"{name}.mrxt"
    if not trace.exists():
        buf, off, ln = pktlib.pack_frames(frames)
        pktlib.write_ref_trace(str(trace), buf, off, ln, forward=sc["forward"])
    # mOS's clock frozen in both runs unless the scenario asks for the real one: ARPTimer
    # (arp.c:313-327) drops a pending request after 1 s of wall time and the next frame to
    # that address asks again, so a run slower than 1 s (a fresh GPU's first launches)
    # would send more ARP requests than the other; the TCP timestamps and ISNs mOS puts
    # in the frames it builds would differ too
    env = dict(os.environ, **({} if sc.get("real_clock") else {"MOSAPP_FROZEN_CLOCK": "1"}))
    env.update(sc["env"], **(extra_env or {}))
    r = subprocess.run([exe, mode, str(conf), str(trace), str(d)], capture_output=True, text=True, timeout=120,
                       env=env)
    assert r.returncode == 0, f"{mode}: rc {r.returncode}\n{r.stdout[-2000:]}\n{r.stderr[-2000:]}"
    import json
    stats = json.loads(r.stdout.strip().splitlines()[-1])
    return dict(returns=(d / "returns.bin").read_bytes(), state=(d / "state.txt").read_text(),
                callbacks=(d / "callbacks.txt").read_text(), tx=pcap_frames(d / "tx.pcap"), stats=stats)


def compare_modes(exe, tmp, name, form="c8"):
    suffix, form_env = FORMS[form]
    exe += suffix
    sc = dict(SCENARIOS[name])
    sc["env"] = dict(sc["env"], **form_env)
    if "fixture" in sc:
        frames = fixture_frames(sc["fixture"])
    else:
        frames = pktlib.conversation_frames(sc.get("nflows", 64), seed=sc.get("seed", 11),
                                            listen_port=sc.get("listen", 0))
    pp = run_app(exe, "pp", tmp, name, sc, frames)
    gpu = run_app(exe, "gpu", tmp, name, sc, frames, sc.get("gpu_env"))
    assert len(pp["returns"]) == len(frames)
    assert gpu["returns"] == pp["returns"], "per-frame return values"
    assert gpu["state"] == pp["state"], "flow table / NETSTAT"
    assert gpu["callbacks"] == pp["callbacks"], "callbacks"
    assert gpu["tx"] == pp["tx"], (f"frames sent: {len(gpu['tx'])} vs {len(pp['tx'])}, ARP requests "
                                    f"{gpu['stats']['arp_sent']} vs {pp['stats']['arp_sent']}, first difference at "
                                    f"{first_diff(gpu['tx'], pp['tx'])}")
    assert gpu["stats"]["consumer_frames"] == len(frames)
    assert gpu["stats"]["gpu_errors"] == 0 and gpu["stats"]["gpu_dropped"] == 0
    return pp, gpu


def first_diff(a, b):
    """Index and ethertypes of the first frame sent that differs between two runs."""
    for i, (x, y) in enumerate(zip(a, b)):
        if x != y:
            return i, x[12:14].hex(), y[12:14].hex()
    return min(len(a), len(b)), None, None


def _have(exe):
    return os.access(exe, os.X_OK)


@pytest.mark.skipif(not _have(APP_EMUL) or not _have(APP_EMUL + "_x"),
                    reason="needs oracle/_ref/mos_app_emul{,_x} (make -C oracle ref)")
@pytest.mark.parametrize("form", sorted(FORMS))
@pytest.mark.parametrize("name", sorted(SCENARIOS))
def test_consumer_matches_processpacket_emulated(tmp_path, name, form):
    pp, gpu = compare_modes(APP_EMUL, tmp_path, name, form)
    _check_scenario(name, pp, gpu, form)


# on the GPU every scenario runs in the module's mOS form (8-byte records); the
# 16-byte form and the patched build over a spread of them (all of them run in
# both on the CPU stand-in above)
GPU_FORM_CASES = [(n, "c8") for n in sorted(SCENARIOS)] + [
    (n, f) for f in ("rec16", "tcp_exports")
    for n in ("filters", "golden_edge_listener", "late_filter", "listener_tx_csum", "many_flows", "monitor_fwd",
              "reopen_filter")]


@pytest.mark.gpu
@pytest.mark.skipif(not _have(APP) or not _have(APP + "_x"),
                    reason="needs oracle/_ref/mos_app{,_x} (built by make -C oracle ref)")
@pytest.mark.parametrize("name,form", GPU_FORM_CASES)
def test_consumer_matches_processpacket_on_gpu(tmp_path, name, form):
    pp, gpu = compare_modes(APP, tmp_path, name, form)
    _check_scenario(name, pp, gpu, form)


ASAN_APP = os.path.join(REF, "asan", "mos_app_emul")


@pytest.mark.skipif(not _have(ASAN_APP), reason="needs oracle/_ref/asan/mos_app_emul (make -C oracle asan)")
@pytest.mark.parametrize("name", sorted(SCENARIOS))
def test_consumer_under_sanitizers(tmp_path, monkeypatch, name):
    """Host code only: the backend (gpu_module.c), the consumer (mos_rx.c) and the
    frame sources (loopback.c) built with AddressSanitizer + UBSan into the
    emulated program; every scenario gives the suite's results and the
    sanitizers report nothing (a report ends the run with a non-zero status)."""
    monkeypatch.setenv("ASAN_OPTIONS", "detect_leaks=0:verify_asan_link_order=0:halt_on_error=1")
    monkeypatch.setenv("UBSAN_OPTIONS", "print_stacktrace=1:halt_on_error=1")
    pp, gpu = compare_modes(ASAN_APP, tmp_path, name, "c8")
    _check_scenario(name, pp, gpu, "c8")


@pytest.mark.skipif(not os.path.exists(os.path.join(REF, "mos_rx_mos_x.o")),
                    reason="needs oracle/_ref (make -C oracle ref)")
def test_patched_build_calls_mos_own_stream_functions():
    """Under the upstream patch the consumer compiles none of its tcp.c
    restatement and calls mOS's CreateStream / HandleSockStream /
    HandleMonitorStream, which the patched tcp.c object defines."""
    def syms(obj, *flags):
        out = subprocess.run(["nm", *flags, os.path.join(REF, obj)], capture_output=True, text=True,
                             check=True).stdout
        return {ln.split()[-1] for ln in out.splitlines() if ln.strip()}
    # (the restated functions are static and inlined: what they call tells them apart --
    # CreateServerStream's ParseTCPOptions, CreateStream's CreateClientTCPStream,
    # HandleMonitorStream's UpdateMonitor)
    restated = {"ParseTCPOptions", "CreateClientTCPStream", "UpdateMonitor"}
    assert restated <= syms("mos_rx_mos.o", "-u") and not (restated & syms("mos_rx_mos_x.o", "-u"))
    want = {"CreateStream", "HandleSockStream", "HandleMonitorStream"}
    assert want <= syms("mos_rx_mos_x.o", "-u") and not (want & syms("mos_rx_mos.o", "-u"))
    assert want | {"DetectStreamType"} <= syms("tcp_x.o", "-g", "--defined-only")


def _check_scenario(name, pp, gpu, form="c8"):
    """What each scenario must have exercised (so a scenario cannot pass vacuously)."""
    st, cb = gpu["stats"], pp["callbacks"]
    # the record form the consumer read: 8-byte records in the compact forms (with
    # filters too: the fused kernels' 8-byte forms), none in the 16-byte one
    assert (st["batches_c8"] == 0) if form == "rec16" else (st["batches_c8"] > 0)
    nstat = pp["state"].splitlines()[-1].split()
    assert int(nstat[6]) > 0                                   # rx_errors: bad checksums etc. were seen
    if name in ("monitor_fwd", "filters", "two_monitors_raw", "listener", "late_filter", "batch_1_per_launch",
                "groups_of_3", "cpu_flow_hash", "many_flows"):
        assert " ev 4 " in cb and " ev 1 " in cb               # MOS_ON_CONN_START, MOS_ON_PKT_IN
        assert st["stream_step"] > 0
    if name == "cpu_flow_hash":
        assert st["gpu_flow_hash"] == 0
    elif st["stream_step"]:
        # every lookup on the GPU's bucket, filters or not (the fused classify + BPF pass makes them too)
        assert st["gpu_flow_hash"] == st["stream_step"]
    # a filter install never stalls the mTCP thread on a compile (the set runs on the interpreter
    # kernel until its hipRTC kernels are in): the longest install + reclassification
    assert st["max_filter_sync_ns"] < (10e6 if name.startswith("real_clock") else 50e6), st["max_filter_sync_ns"]
    if name == "monitor_nofwd":
        assert all(f[12:14] == b"\x08\x06" for f in pp["tx"])  # forward = 0: only mOS's own ARP requests leave
    if name in ("monitor_fwd", "no_socket"):
        assert len(pp["tx"]) > 0
    if name == "filters":
        assert st["filters_gpu"] == 3 and st["filter_installs"] >= 1
        assert " ev 100 " in cb                                # MOS_ON_ORPHAN through the orphan filter
    if name.startswith("listener"):
        assert any(f[47] & 0x04 for f in pp["tx"] if len(f) > 47 and f[23] == 6)   # RSTs to orphans
    if name.endswith("_tx_csum"):
        # the GPU filled the checks of every TCP frame mOS built (SYN-ACKs, ACKs, RSTs);
        # forwarded frames keep theirs and ask for nothing
        # (at least the RSTs SendTCPPacketStandalone builds for orphans, tcp.c:503-506: IP id 0,
        # TCP window 0); the frames themselves were compared above, checks included
        built = sum(1 for f in gpu["tx"] if len(f) > 47 and f[12:14] == b"\x08\x00" and f[23] == 6
                    and f[18:20] == b"\x00\x00" and f[48:50] == b"\x00\x00")
        assert built > 0
        assert gpu["stats"]["tx_csum_offloaded"] >= built and gpu["stats"]["tx_errors"] == 0
        assert pp["stats"]["tx_csum_offloaded"] == 0
    if name == "late_filter":
        assert st["filter_installs"] >= 1 and st["reclassified"] >= 1
    if name == "reopen_filter":
        assert st["filter_installs"] >= 2 and st["filters_gpu"] == 1   # the freed program's entry went
        assert st["reopen_same_addr"] == 1 and pp["stats"]["reopen_same_addr"] == 1
    if name.startswith("real_clock"):
        assert st["filter_installs"] >= 1 and st["filters_gpu"] == 2
        assert pp["stats"]["arp_sent"] > 0 and gpu["stats"]["arp_sent"] == pp["stats"]["arp_sent"]
    if name == "late_monitor":
        assert st["reclassified"] >= 1
    if name.startswith("golden_"):
        assert st["stream_step"] > 0
        assert len(set(pp["returns"])) == 3                     # -1, 0 and 1 all reached


def _gpu_error_run(exe, tmp_path):
    """late_monitor with the consumer's first reclassification failing (a GPU error in the
    middle of a batch, injected by the harness): the rest of that batch is dropped and
    counted, mOS carries on, and everything else equals ProcessPacket's run."""
    sc = dict(SCENARIOS["late_monitor"])
    sc["env"] = dict(sc["env"], MOSAPP_BATCH="97", MOSAPP_GROUP="1")
    frames = pktlib.conversation_frames(64, seed=11)
    pp = run_app(exe, "pp", tmp_path, "gpu_error", sc, frames)
    gpu = run_app(exe, "gpu", tmp_path, "gpu_error", sc, frames, {"MOSAPP_FAIL_RECLASSIFY": "1"})
    st = gpu["stats"]
    assert st["consumer_frames"] == len(frames) and st["gpu_errors"] == 1
    at = int(SCENARIOS["late_monitor"]["env"]["MOSAPP_LATE_MON_AT"]) - 1   # the frame the monitor appears at
    end = min((at // 97 + 1) * 97, len(frames))                           # the end of its batch
    # the reclassification comes at the first IPv4 frame from `at` on (the checksum gate, ip_in.c:67)
    first = end - st["gpu_dropped"]
    assert at <= first < end
    r_pp, r_gpu = pp["returns"], gpu["returns"]
    assert r_gpu[:first] == r_pp[:first] and r_gpu[end:] == r_pp[end:]   # the frames around them: unchanged
    assert set(r_gpu[first:end]) == {0xFF}                                # dropped: -1
    n_pp, n_gpu = (x["state"].splitlines()[-1].split() for x in (pp, gpu))
    assert n_gpu[2] == n_pp[2]                                            # rx_packets: every frame seen
    neg = sum(1 for x in r_gpu if x == 0xFF)
    assert int(n_gpu[6]) == neg                                           # rx_errors: the -1 returns, dropped ones in


@pytest.mark.skipif(not _have(APP_EMUL), reason="needs oracle/_ref/mos_app_emul (make -C oracle ref)")
def test_consumer_survives_gpu_error_emulated(tmp_path):
    _gpu_error_run(APP_EMUL, tmp_path)


@pytest.mark.gpu
@pytest.mark.skipif(not _have(APP), reason="needs oracle/_ref/mos_app (built by make -C oracle ref)")
def test_consumer_survives_gpu_error_on_gpu(tmp_path):
    _gpu_error_run(APP, tmp_path)
