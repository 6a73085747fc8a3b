"""Pin the oracle (C restatement) against mOS's own outputs.

The fixtures in tests/golden/ were produced by mOS's compiled core/src rx path
(oracle/_ref/mosref, see tests/golden/make_golden.py); the MSDN Toeplitz KAT
comes from util/rss.c:177-193.  When oracle/_ref/mosref exists (this build
container) the oracle is also fuzzed against the reference directly.
"""
import os
import random

import numpy as np
import pytest

import oracle_py as O
from pktlib import NREASON, R, REF_FIELDS, icmp_frame, pack_frames, tcp_frame

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
FIXTURES = ["edge", "rand_small", "rand_mid", "rand_large"]
LOCAL = ("10.0.0.2", "192.168.1.1", "172.16.9.77")   # tests/golden/make_golden.py
STATES = {  # name -> (num_msp, num_esp, num_queues, queue_mode, netdev addresses)
    "msp1": (1, 0, 1, 1, ()), "noverify": (0, 0, 1, 1, ()), "esp1": (0, 1, 1, 1, ()),
    "q2_i40e": (1, 0, 2, 1, ()), "q4_i40e": (1, 0, 4, 1, ()), "q8_i40e": (1, 0, 8, 1, ()),
    "q3_ixgbe": (1, 0, 3, 0, ()), "q8_ixgbe": (1, 0, 8, 0, ()),
    "msp1_local": (1, 0, 1, 1, LOCAL), "esp1_local": (0, 1, 4, 1, LOCAL), "noverify_local": (0, 0, 1, 1, LOCAL),
}


def state_params(state, **kw):
    msp, esp, nq, qm, loc = STATES[state]
    return O.params(num_msp=msp, num_esp=esp, forward=0, num_queues=nq, queue_mode=qm, local=loc, **kw)


def compare_with_ref(res, ref, p, fh=None, ti=None):
    """Field-by-field agreement of records with the reference harness output:
    every one of the 16 record bytes that the reference defines for the frame.

    `fh` (optional) is the per-frame flow hash; its low 17 bits must equal the
    reference's HashFlow() bucket wherever the reference computed one.  `ti`
    (optional) is the mosrx_tcpinfo side array: seq / ack_seq / window / ip_len
    as mOS's own FillPacketContextTCPInfo left them in pkt_info."""
    trunc = res["reason"] == R["TRUNCATED"]
    skipped = (ref["have"] & 8) != 0
    np.testing.assert_array_equal(trunc, skipped, err_msg="TRUNCATED set differs from reference skips")
    live = ~trunc
    np.testing.assert_array_equal(res["verdict"][live], ref["verdict"][live], err_msg="verdict")
    # header fields are defined once the version check passed
    fields = live & ~np.isin(res["reason"], [R["ARP"], R["NON_IPV4"], R["IP_SHORT"], R["IP_BADVER"]])
    np.testing.assert_array_equal(res["rss"][fields], ref["rss"][fields], err_msg="rss")
    np.testing.assert_array_equal(res["queue"][fields], ref["queue"][fields].astype(np.uint8), err_msg="queue")
    if p.num_msp or p.num_esp:
        np.testing.assert_array_equal(res["ip_csum"][fields], ref["ip_csum"][fields], err_msg="ip_csum")
    tcp = live & np.isin(res["reason"], [R["TCP_OK"], R["TCP_BADCSUM"]])
    assert np.all(ref["have"][tcp] & 2)
    np.testing.assert_array_equal(res["tcp_csum"][tcp], ref["tcp_csum"][tcp], err_msg="tcp_csum")
    np.testing.assert_array_equal(res["tcp_csum"][tcp] == 0, res["verdict"][tcp] == 1)
    # pkt_info TCP fields (FillPacketContextTCPInfo, tcp.c:258-270), run by mOS itself on every
    # in-bounds TCP frame; the record defines them once the header fields are (payload_off != 0)
    tcpf = live & (res["payload_off"] != 0)
    assert np.all(ref["have"][tcpf] & 32), "pkt_info fields defined where the reference has none"
    for f in ("payloadlen", "payload_off", "tcp_flags", "ihl_doff"):
        np.testing.assert_array_equal(res[f][tcpf], ref[f][tcpf].astype(res[f].dtype), err_msg=f)
    # ... and zero on every other frame (no TCP header: nothing for the flow engine)
    notcp = ~tcpf
    assert np.all(res["payloadlen"][notcp] == 0) and np.all(res["tcp_flags"][notcp] == 0)
    assert np.all(res["ihl_doff"][notcp] & 0xF == 0)
    if ti is not None:
        for f in ("seq", "ack_seq", "window", "ip_len"):
            np.testing.assert_array_equal(ti[f][tcpf], ref[f][tcpf], err_msg=f)
            assert np.all(ti[f][notcp] == 0), f
    if fh is not None:
        hashed = live & (res["payload_off"] != 0)
        # the harness hashes every in-bounds TCP frame; the path defines it where FindStream runs
        assert np.all(ref["have"][hashed] & 16), "flow hash defined where the reference has none"
        np.testing.assert_array_equal(fh[hashed] & 0x1FFFF, ref["fbucket"][hashed], err_msg="fbucket")


@pytest.mark.parametrize("fix", FIXTURES)
@pytest.mark.parametrize("state", list(STATES))
def test_oracle_matches_reference_fixture(fix, state):
    z = np.load(os.path.join(GOLDEN, f"{fix}.npz"))
    p = state_params(state)
    res, fh, ti = O.classify_ex(z["frames"], z["off"], z["len"], p)
    ref = {k: z[f"{state}__{k}"] for k in REF_FIELDS}
    compare_with_ref(res, ref, p, fh, ti)
    # NETSTAT view (eth_in.c:42-45, 80-84) over the frames the reference processed
    live = res["reason"] != R["TRUNCATED"]
    st = z[f"{state}__stats"]
    assert st[0] == live.sum()
    assert st[1] == (z["len"][live].astype(np.uint64) + 24).sum()
    assert st[2] == (res["verdict"][live] < 0).sum()


def test_fixtures_cover_every_reason():
    seen = set()
    for fix in FIXTURES:
        z = np.load(os.path.join(GOLDEN, f"{fix}.npz"))
        for state in STATES:
            seen |= set(np.unique(O.classify(z["frames"], z["off"], z["len"], state_params(state))["reason"]).tolist())
    missing = {k for k, v in R.items() if v not in seen} - {"TCP_LEN_OK"}
    assert not missing, missing


def test_msdn_rss_kat():
    z = np.load(os.path.join(GOLDEN, "rss_msdn_kat.npz"))
    key = bytes(z["key"])
    for v in z["kat"]:
        assert O.rss_hash(key, int(v["sip"]), int(v["dip"]), int(v["sp"]), int(v["dp"])) == int(v["hash"])


def test_default_key_survey_values():
    # 10.0.0.1:1234 -> 10.0.0.2:80 hashes to 0x27272727 with the 0x05 key;
    # num_queues=8 gives queue 4 with the i40e map and 7 with ixgbe.
    cache_key = b"\x05" * 40
    h = O.rss_hash(cache_key, 0x0A000001, 0x0A000002, 1234, 80)
    assert h == 0x27272727
    assert O.lib().mo_rss_queue(h, 1, 8) == 4
    assert O.lib().mo_rss_queue(h, 0, 8) == 7
    # symmetric key: swapping the endpoints keeps the hash
    assert O.rss_hash(cache_key, 0x0A000002, 0x0A000001, 80, 1234) == h


def test_ip_fast_csum_quirk():
    f = tcp_frame(ihl=4, pad_to=60)
    for ihl in range(5):
        assert O.lib().mo_ip_fast_csum(f[14:], ihl) == (f[14] | (f[15] << 8))


def test_forward_nonip_verdicts():
    # eth_in.c:62-77: forward && num_msp makes every non-IPv4 frame 1 (with mOS's own
    # ProcessPacket on the fixtures under forward = 1: tests/test_forwarding.py)
    frames = [tcp_frame(ethertype=0x86DD, pad_to=60), tcp_frame(ethertype=0x0806, pad_to=60)]
    buf, off, ln = pack_frames(frames)
    a = O.classify(buf, off, ln, O.params(num_msp=1, forward=1))
    assert list(a["verdict"]) == [1, 1]
    b = O.classify(buf, off, ln, O.params(num_msp=0, num_esp=1, forward=1))
    assert list(b["verdict"]) == [-1, 1]


@pytest.mark.skipif(not O.have_ref(), reason="oracle/_ref/mosref not built (needs /root/reference)")
@pytest.mark.parametrize("seed", [1, 2, 3])
def test_oracle_fuzz_vs_reference(seed):
    from golden.make_golden import random_frames
    rng = random.Random(seed)
    frames = random_frames(rng, 300, seed % 3)
    buf, off, ln = pack_frames(frames, phase=rng.choice([2, 3, 6, 9]))
    for msp, esp, nq, qm, loc in [(1, 0, 1, 1, ()), (0, 1, 5, 0, ()), (1, 1, 7, 1, ("10.0.0.2",))]:
        p = O.params(num_msp=msp, num_esp=esp, forward=0, num_queues=nq, queue_mode=qm, local=loc)
        rec, _ = O.run_ref(buf, off, ln, num_msp=msp, num_esp=esp, num_queues=nq, queue_mode=qm, local=loc)
        res, fh, ti = O.classify_ex(buf, off, ln, p)
        compare_with_ref(res, rec, p, fh, ti)


@pytest.mark.skipif(not O.have_ref(), reason="oracle/_ref/mosref not built (needs /root/reference)")
def test_oracle_vs_reference_on_seeded_trace():
    import mosrx
    t = mosrx.Trace(mosrx.TRACE_IMIX, 6000, nflows=1000)
    p = O.params(forward=0)
    rec, _ = O.run_ref(t.frames, t.off, t.len)
    res, fh, ti = O.classify_ex(t.frames, t.off, t.len, p)
    compare_with_ref(res, rec, p, fh, ti)
    # corruption schedule of the generator: 1/1024 IP, 1/1024 TCP
    idx = np.arange(t.n)
    assert np.all(res["reason"][idx % 1024 == 511] == R["IP_BADCSUM"])
    assert np.all(res["reason"][idx % 1024 == 1023] == R["TCP_BADCSUM"])
    ok = (idx % 1024 != 511) & (idx % 1024 != 1023)
    assert np.all(res["reason"][ok] == R["TCP_OK"])


@pytest.mark.skipif(not O.have_ref(), reason="oracle/_ref/mosref not built (needs /root/reference)")
def test_icmp_local_fuzz_vs_reference():
    """ICMP frames to and past the netdev addresses (icmp.c:193-200), random types
    and mutations, against mOS's own ProcessICMPPacket verdicts."""
    rng = random.Random(77)
    local = ("10.0.0.2", "192.168.1.1")
    dsts = list(local) + ["10.0.0.3", "192.168.1.2", "2.0.0.10"]
    frames = []
    for _ in range(200):
        f = bytearray(icmp_frame(dst=rng.choice(dsts), icmp_type=rng.choice([0, 3, 5, 8, 11, 13, 200]),
                                 payload=bytes(rng.getrandbits(8) for _ in range(rng.randint(0, 40))),
                                 ihl=rng.choice([5, 5, 6, 15])))
        if rng.random() < 0.2:
            f[rng.randint(14, len(f) - 1)] ^= 1 << rng.randint(0, 7)
        frames.append(bytes(f))
    buf, off, ln = pack_frames(frames, phase=rng.choice([2, 5]))
    for msp, esp in [(1, 0), (0, 1), (0, 0)]:
        p = O.params(num_msp=msp, num_esp=esp, forward=0, local=local)
        rec, _ = O.run_ref(buf, off, ln, num_msp=msp, num_esp=esp, local=local)
        res, fh, ti = O.classify_ex(buf, off, ln, p)
        compare_with_ref(res, rec, p, fh, ti)
        if msp or esp:
            assert (res["reason"] == R["ICMP_LOCAL"]).sum() > 20
