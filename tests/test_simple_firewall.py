"""BASELINE config #1 through the reference's own application (VERDICT r5 next
#3): mOS's samples/simple_firewall/simple_firewall.c compiled unmodified
(oracle/Makefile _ref/simple_firewall*) over the ENABLE_GPU build of
INTEGRATION.md §2, gpu_module_func replaying a pcap file of config #1's
10 000 x 60 B one-flow trace plus handshakes of flows the firewall's rules
match (simple_firewall.c:307-330: DROP -> MOS_DROP, ACCEPT -> MOS_STOP_MON).

The sample runs twice on the same frames: RunMainLoop's per-frame call
(core.c:906) to mOS's own ProcessPacket ("pp"), and to the consumer of the GPU
records, mosrx_mos_process_packet ("gpu").  Both runs must agree on every
frame's return, NETSTAT, the sample's own rule table (flows per rule, printed by
DumpFWRuleTable, simple_firewall.c:78-126) and every frame forwarded.  The CPU
suite runs the binary over the CPU stand-in for the GPU (simple_firewall_emul);
the GPU suite runs it on the GPU."""
import os
import re
import struct
import subprocess

import numpy as np
import pytest

import mosrx
import oracle_py as O
import pktlib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = os.path.join(ROOT, "oracle", "_ref")

CONF = """mos {{
	forward = 1
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

# the sample's rule syntax (simple_firewall.c:217-289); first match wins, no match accepts
RULES = """# act   src           dst           ports
DROP    10.5.0.0/24   10.5.0.0/24   dport:80
ACCEPT  10.5.1.7      10.5.1.9      sport:1024
ACCEPT  10.5.2.7      10.5.2.9
DROP    10.5.3.0/24   10.5.4.0/24
"""


def handshake(cli, srv, cp, sp, isn=1000, data=3):
    """SYN, SYN-ACK, ACK and `data` segments each way of one flow."""
    f = [pktlib.tcp_frame(cli, srv, cp, sp, flags=0x02, seq=isn, ack=0),
         pktlib.tcp_frame(srv, cli, sp, cp, flags=0x12, seq=9000, ack=isn + 1),
         pktlib.tcp_frame(cli, srv, cp, sp, flags=0x10, seq=isn + 1, ack=9001)]
    cs, ss = isn + 1, 9001
    for i in range(data):
        pl = bytes([i + 1]) * (40 + 13 * i)
        f.append(pktlib.tcp_frame(cli, srv, cp, sp, pl, flags=0x18, seq=cs, ack=ss))
        cs += len(pl)
        f.append(pktlib.tcp_frame(srv, cli, sp, cp, b"", flags=0x10, seq=ss, ack=cs))
    return f


def firewall_frames():
    """Config #1's one flow (TRACE_FW64: 10 000 x 60 B, SYN first) with rule-matching
    flows interleaved, and a bad-checksum segment of an accepted flow."""
    t = mosrx.Trace(mosrx.TRACE_FW64, 10_000)
    base = [bytes(t.frames[int(o):int(o) + int(n)]) for o, n in zip(t.off, t.len)]
    flows = [handshake("10.5.0.5", "10.5.0.9", 40000, 80, 100),        # rule 1: DROP
             handshake("10.5.1.7", "10.5.1.9", 1024, 443, 200),        # rule 2: ACCEPT, stop monitoring
             handshake("10.5.2.7", "10.5.2.9", 5555, 8080, 300),       # rule 3: ACCEPT
             handshake("10.5.3.3", "10.5.4.4", 6000, 22, 400),         # rule 4: DROP
             handshake("192.168.8.1", "192.168.9.1", 7000, 80, 500)]   # no rule: ACCEPT
    bad = pktlib.tcp_frame("10.5.2.7", "10.5.2.9", 5555, 8080, b"zz", flags=0x18, seq=301, ack=9001, tcp_csum=0x1)
    out, k = [], 0
    for i, fr in enumerate(base):
        out.append(fr)
        if i % 400 == 399 and k < max(len(f) for f in flows):   # a frame of every rule flow, now and then
            out += [f[k] for f in flows if k < len(f)]
            k += 1
    out += [f[j] for j in range(k, max(len(f) for f in flows)) for f in flows if j < len(f)]
    out.append(bad)
    return out


def write_pcap(path, frames):
    with open(path, "wb") as fh:
        fh.write(struct.pack("<IHHiIII", 0xA1B2C3D4, 2, 4, 0, 0, 65535, 1))
        for i, fr in enumerate(frames):
            fh.write(struct.pack("<IIII", i, 0, len(fr), len(fr)) + fr)


def pcap_frames(path):
    raw = open(path, "rb").read()
    out, pos = [], 24
    while pos + 16 <= len(raw):
        incl = struct.unpack("<IIII", raw[pos:pos + 16])[2]
        out.append(raw[pos + 16:pos + 16 + incl])
        pos += 16 + incl
    return out


def rule_table(stdout):
    """The last table DumpFWRuleTable printed: [(idx, flows, target)] ([]: none printed)."""
    tables = stdout.split("Firewall rule table")
    if len(tables) < 2:
        return []
    rows = re.findall(r"^(\d+)\s+(\d+)\s+(ACCEPT|DROP)\s", tables[-1], re.M)
    return [(int(a), int(b), c) for a, b, c in rows]


def run_sample(exe, mode, tmp, frames, loops=1, linger_ms=1300):
    d = tmp / mode
    (d / "log").mkdir(parents=True)
    conf, rules, pcap = d / "mos.conf", d / "fw.conf", tmp / "trace.pcap"
    conf.write_text(CONF.format(log=d / "log"))
    rules.write_text(RULES)
    if not pcap.exists():
        write_pcap(pcap, frames)
    env = dict(os.environ, MOSRX_PCAP_lo=str(pcap), MOSRX_PCAP_LOOPS=str(loops), MOSRX_TX_PCAP_lo=str(d / "tx.pcap"),
               SFGLUE_MODE=mode, SFGLUE_FRAMES=str(len(frames) * loops), SFGLUE_OUT=str(d),
               SFGLUE_LINGER_MS=str(linger_ms))
    r = subprocess.run([exe, "-c", str(conf), "-f", str(rules), "-n", "1"], capture_output=True, text=True,
                       timeout=180, env=env, cwd=d)
    assert r.returncode == 0, f"{mode}: rc {r.returncode}\n{r.stdout[-2000:]}\n{r.stderr[-2000:]}"
    import json
    return dict(returns=(d / "returns.bin").read_bytes(), state=(d / "state.txt").read_text(),
                table=rule_table(r.stdout), tx=pcap_frames(d / "tx.pcap"),
                result=json.loads((d / "result.json").read_text()))


def is_arp(fr):
    return fr[12:14] == b"\x08\x06"


def check_modes(exe, tmp):
    frames = firewall_frames()
    pp = run_sample(exe, "pp", tmp, frames)
    gpu = run_sample(exe, "gpu", tmp, frames)
    n = len(frames)
    assert pp["result"]["done"] == gpu["result"]["done"] == n
    assert len(pp["returns"]) == n
    assert gpu["returns"] == pp["returns"], "per-frame returns"
    assert gpu["state"] == pp["state"], "NETSTAT / flow count"
    assert pp["table"] and gpu["table"] == pp["table"], "the sample's rule table"
    fwd_pp = [f for f in pp["tx"] if not is_arp(f)]
    fwd_gpu = [f for f in gpu["tx"] if not is_arp(f)]
    assert fwd_gpu == fwd_pp, f"forwarded frames: {len(fwd_gpu)} vs {len(fwd_pp)}"
    # the firewall did what its rules say: each rule flow looked up once, at its SYN
    # (the sample's CatchInitSYN event); mOS's own verdicts are the checks' (the
    # trace's corrupted frames and the one bad TCP checksum, per the oracle)
    assert pp["table"] == [(1, 1, "DROP"), (2, 1, "ACCEPT"), (3, 1, "ACCEPT"), (4, 1, "DROP")]
    buf, off, ln = pktlib.pack_frames(frames)
    ora = O.classify(buf, off, ln, O.params())
    rets = np.frombuffer(pp["returns"], np.int8)
    assert ((rets < 0) == (ora["verdict"] < 0)).all()
    assert f"rx_errors {int((ora['verdict'] < 0).sum())} " in pp["state"]
    assert gpu["result"]["consumer_frames"] == n and gpu["result"]["gpu_errors"] == 0
    return pp, gpu


def test_simple_firewall_unmodified_over_gpu_module_cpu_standin(tmp_path):
    exe = os.path.join(REF, "simple_firewall_emul")
    if not os.access(exe, os.X_OK):
        pytest.skip("oracle/_ref/simple_firewall_emul not built (make -C oracle ref; needs /root/reference)")
    check_modes(exe, tmp_path)


@pytest.mark.gpu
def test_simple_firewall_unmodified_over_gpu_module(tmp_path):
    exe = os.path.join(REF, "simple_firewall")
    if not os.access(exe, os.X_OK):
        pytest.skip("oracle/_ref/simple_firewall did not travel with the tree")
    check_modes(exe, tmp_path)
