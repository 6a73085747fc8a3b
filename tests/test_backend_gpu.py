"""GPU tests of gpu_module_func as a faithful peer of pcap_module_func
(pcap_module.c:34-89, :124-160), driven through the C ABI: records against the
oracle for every way a batch reaches the GPU (per-frame, runs, zero-copy,
groups of batches in one launch, a pcap file), pkt_info fields through
dev_ioctl, stack-state updates, and TX (get_wptr / send_pkts) reaching the
source."""
import ctypes as C
import os
import socket
import struct

import numpy as np
import pytest

import mosrx
import oracle_py as O
from pktlib import NREASON, icmp_frame, pack_frames, tcp_frame
from test_parity_gpu import assert_records_equal

pytestmark = pytest.mark.gpu


def write_pcap(path, frames, off, ln):
    with open(path, "wb") as fh:
        fh.write(struct.pack("<IHHiIII", 0xA1B2C3D4, 2, 4, 0, 0, 65535, 1))
        for i, (o, n) in enumerate(zip(off.tolist(), ln.tolist())):
            fh.write(struct.pack("<IIII", i, 0, n, n) + bytes(frames[o:o + n]))


# the frames mOS forwards for a record under (forward, num_msp, listener): eth_in.c:60-77
# (every non-IPv4 frame, ARP too), ip_in.c:66-70 (no monitor / stream socket),
# ip_in.c:86-91 (other protocols), tcp.c:438-442 (bad TCP checksum), and, for accepted
# segments of flows without a stream, the monitor stream / orphan path unless an
# end-host socket listens (tcp.c:453-510); pinned to mOS itself by
# test_backend_inside_mos_checked_by_processpacket and tests/golden/forward.npz
def mos_forwarded(rec, forward=1, num_msp=1, listener=0):
    r = rec["reason"]
    R = mosrx.R
    if not forward:
        return np.zeros(len(rec), bool)
    msp_only = (r == R["NON_IPV4"]) | (r == R["ARP"]) | (r == R["NOT_TCP"]) | (r == R["TCP_BADCSUM"])
    ok = (r == R["TCP_OK"]) | (r == R["TCP_LEN_OK"])
    return (msp_only & (num_msp != 0)) | (r == R["NOVERIFY_PASS"]) | (ok & (num_msp != 0) & (not listener))


def drain(be, n_expect=None):
    """recv_pkts until idle: (records, frames) in arrival order."""
    recs, frames = [], []
    while True:
        n = be.recv_pkts(0)
        assert n >= 0
        if n == 0:
            break
        recs.append(be.results(0, n))
        frames += [be.get_rptr(0, i) for i in range(n)]
    return (np.concatenate(recs) if recs else np.zeros(0, mosrx.RESULT_DTYPE)), frames


@pytest.mark.parametrize("group", [1, 3, 8])
@pytest.mark.parametrize("mode", [mosrx.SRC_BEST, mosrx.SRC_FILL, mosrx.SRC_PER_FRAME])
def test_groups_of_batches_one_launch(group, mode):
    """cfg.group batches per kernel launch (the batch queue from host memory):
    records equal the oracle over three replays of the trace, every batch a
    separate recv_pkts, get_rptr frames intact, one timed launch per group."""
    t = mosrx.Trace(mosrx.TRACE_IMIX, 7000, nflows=300)
    src = mosrx.mem_source(t.frames, t.off, t.len, loops=3, mode=mode)
    be = mosrx.GpuBackend([src], batch=1024, pipeline=True, cpu=5, group=group, timing=True)
    try:
        seen, sizes = 0, []
        ora = O.classify(t.frames, t.off, t.len, O.params())
        while True:
            n = be.recv_pkts(0)
            assert n >= 0
            if n == 0:
                break
            sizes.append(n)
            idx = (seen + np.arange(n)) % t.n
            assert_records_equal(be.results(0, n), ora[idx], f"group {group} batch@{seen}")
            for i in (0, n - 1):
                j = int(idx[i])
                assert be.get_rptr(0, i) == bytes(t.frames[t.off[j]:t.off[j] + t.len[j]])
            seen += n
        assert seen == 3 * t.n
        st = be.stats()
        assert st.rx_frames == seen and st.rx_batches == len(sizes)
        # a group ends early where the source runs dry (the replay's end), never later
        assert -(-len(sizes) // group) <= st.kernel_launches <= len(sizes) and st.kernel_ms > 0
        if group == 1:
            assert st.kernel_launches == len(sizes)
    finally:
        be.close()


@pytest.mark.parametrize("group", [1, 4])
def test_tcpinfo_through_the_backend(group):
    t = mosrx.Trace(mosrx.TRACE_IMIX, 9000, nflows=700)
    src = mosrx.mem_source(t.frames, t.off, t.len, loops=1)
    be = mosrx.GpuBackend([src], batch=2048, cpu=6, group=group, tcpinfo=True)
    try:
        ora, _, oti = O.classify_ex(t.frames, t.off, t.len, O.params())
        seen = 0
        while (n := be.recv_pkts(0)) > 0:
            assert_records_equal(be.results(0, n), ora[seen:seen + n], "records")
            np.testing.assert_array_equal(be.tcpinfo(0, n), oti[seen:seen + n])
            seen += n
        assert seen == t.n
    finally:
        be.close()


@pytest.mark.parametrize("group,tcpinfo", [(1, False), (4, True), (0, False)])
def test_flow_hash_through_the_backend(group, tcpinfo):
    """cfg.flowhash: every batch carries FindStream's flow-table hash per frame
    (dev_ioctl(MOSRX_PKT_RX_FHASH)), equal to the oracle's HashFlow restatement
    (pinned to mOS's own in test_flow_hash_golden), whatever the batches per
    launch (1, 4, auto) and with the pkt_info fields beside it."""
    t = mosrx.Trace(mosrx.TRACE_IMIX, 9000, nflows=700)
    src = mosrx.mem_source(t.frames, t.off, t.len, loops=1)
    be = mosrx.GpuBackend([src], batch=1500, cpu=6, group=group, tcpinfo=tcpinfo, flowhash=True)
    try:
        ora, ofh = O.classify_fh(t.frames, t.off, t.len, O.params())
        seen = 0
        while (n := be.recv_pkts(0)) > 0:
            assert_records_equal(be.results(0, n), ora[seen:seen + n], "records")
            np.testing.assert_array_equal(be.fhashes(0, n), ofh[seen:seen + n])
            seen += n
        assert seen == t.n
    finally:
        be.close()


def test_backend_fed_from_a_pcap_file(tmp_path):
    """mosrx_source_pcap (the libpcap-free pcap_next, pcap_module.c:41) behind the
    backend: the trace written to a pcap file classifies exactly as the oracle
    says, through the RunMainLoop-shaped loop and batch by batch."""
    t = mosrx.Trace(mosrx.TRACE_IMIX, 12000, nflows=900)
    path = str(tmp_path / "trace.pcap")
    write_pcap(path, t.frames, t.off, t.len)
    ora = O.classify(t.frames, t.off, t.len, O.params())
    src = mosrx.lib().mosrx_source_pcap(path.encode(), 1)
    assert src
    be = mosrx.GpuBackend([src], batch=4096, cpu=7)
    try:
        recs, frames = drain(be)
        assert_records_equal(recs, ora, "pcap source")
        assert frames[::997] == [bytes(t.frames[o:o + n]) for o, n in zip(t.off[::997], t.len[::997])]
    finally:
        be.close()
    src = mosrx.lib().mosrx_source_pcap(path.encode(), 2)
    be = mosrx.GpuBackend([src], batch=4096, cpu=8, group=2)
    try:
        st = be.run_loop()
        assert st.rx_packets == 2 * t.n
        assert list(st.by_reason) == (2 * np.bincount(ora["reason"], minlength=NREASON)).tolist()
    finally:
        be.close()


def test_small_frames_through_the_backend():
    """64 B frames (BASELINE config #2) through the backend: the batch's real max
    caplen goes with it (not cfg.max_frame), so the SMALL tile classifies it;
    records equal the oracle and every 32K batch is one timed launch."""
    t = mosrx.Trace(mosrx.TRACE_S64, 32768)
    src = mosrx.mem_source(t.frames, t.off, t.len, loops=4)
    be = mosrx.GpuBackend([src], batch=32768, cpu=9, timing=True)
    try:
        recs, _ = drain(be)
        st = be.stats()
    finally:
        be.close()
    ora = O.classify(t.frames, t.off, t.len, O.params())
    assert_records_equal(recs, np.concatenate([ora] * 4), "S64 via backend")
    assert st.kernel_launches == 4 and st.kernel_ms > 0


def test_set_params_ioctl_changes_the_stack_state():
    """dev_ioctl(MOSRX_PKT_SET_PARAMS): a monitor socket appears (num_msp 0 -> 1,
    socket.c:77-78), so checksums are verified from the next submitted batch."""
    frames = [tcp_frame(ip_csum=0x1111), icmp_frame(dst="10.0.0.2")] * 600
    buf, off, ln = pack_frames(frames)
    src = mosrx.mem_source(buf, off, ln, loops=4)
    p0 = mosrx.default_params(num_msp=0, num_esp=0)
    be = mosrx.GpuBackend([src], batch=1200, cpu=10, params=p0, pipeline=False)
    try:
        n = be.recv_pkts(0)
        r = be.results(0, n)
        assert set(r["reason"].tolist()) == {mosrx.R["NOVERIFY_PASS"]}
        p1 = mosrx.default_params(num_msp=1, local=["10.0.0.2"])
        assert be.set_params(0, p1) == 0
        n = be.recv_pkts(0)
        r = be.results(0, n)
        assert set(r["reason"][0::2].tolist()) == {mosrx.R["IP_BADCSUM"]}
        assert set(r["reason"][1::2].tolist()) == {mosrx.R["ICMP_LOCAL"]}
        assert set(r["verdict"][1::2].tolist()) == {1}
    finally:
        be.close()


def test_tx_reaches_the_source(tmp_path):
    """get_wptr + send_pkts (pcap_module.c:67-89): frames written by the
    application leave through the source -- here its pcap dump -- in order; a
    full TX buffer is flushed by get_wptr itself (dpdk_get_wptr).  Then the
    RunMainLoop-shaped loop with the ForwardEthernetFrame consumer
    (eth_out.c:105-129) sends back every frame the checks accepted."""
    t = mosrx.Trace(mosrx.TRACE_IMIX, 5000, nflows=300)
    src = mosrx.mem_source(t.frames, t.off, t.len, loops=1)
    path = str(tmp_path / "tx.pcap")
    mosrx.source_tx_pcap(src, path)
    be = mosrx.GpuBackend([src], batch=1024, cpu=11, tx_batch=16)
    ora = O.classify(t.frames, t.off, t.len, O.params())
    try:
        mine = [tcp_frame(payload=bytes([i]) * (i * 11), seq=i) for i in range(40)]
        for f in mine[:16]:
            be.send(0, f)
        assert be.send_pkts(0) == 16
        for f in mine[16:]:               # 24 frames: the 17th get_wptr flushes the first 16
            be.send(0, f)
        assert be.stats().tx_packets == 32
        assert be.send_pkts(0) == 8
        fwd = be.forwarder([0])
        st = be.run_loop(forward=fwd)
        assert st.rx_packets == t.n
        assert fwd.forwarded == int(mos_forwarded(ora).sum()) and fwd.dropped == t.n - fwd.forwarded
        assert be.stats().tx_packets == 40 + fwd.forwarded
    finally:
        be.close()
    sent = mosrx.read_pcap(path)
    keep = np.nonzero(mos_forwarded(ora))[0]
    assert sent[:40] == mine
    assert sent[40:] == [bytes(t.frames[t.off[i]:t.off[i] + t.len[i]]) for i in keep]


def _zero_checks(f: bytes) -> bytes:
    """mOS builds its frames with iph->check = 0 (ip_out.c:167) and leaves the TCP
    check to the offload; zero both as it does."""
    b = bytearray(f)
    b[24:26] = b"\0\0"
    ihl = (b[14] & 15) * 4
    if b[23] == 6 and len(b) >= 14 + ihl + 18:
        b[14 + ihl + 16:14 + ihl + 18] = b"\0\0"
    return bytes(b)


def test_tx_checksum_offload(tmp_path):
    """cfg.tx_csum: dev_ioctl(PKT_TX_IP_CSUM / PKT_TX_TCP_CSUM) on the frame get_wptr
    returned last is taken as a NIC offload (dpdk_dev_ioctl, dpdk_module.c:556-566) and
    send_pkts fills those checks on the GPU before the frames leave: each frame as
    the oracle's TX rewrite (= mOS's ip_fast_csum / TCPCalcChecksum, test_tx_csum.py)
    makes it for the checks it asked for; frames that asked for nothing leave as
    written.  Without cfg.tx_csum, or for a pointer that is not the last frame's IP
    header, the ioctl returns -1 (mOS computes the checksum itself)."""
    t = mosrx.Trace(mosrx.TRACE_IMIX, 300, nflows=40)
    frames = [_zero_checks(bytes(t.frames[t.off[i]:t.off[i] + t.len[i]])) for i in range(t.n)]
    frames += [_zero_checks(tcp_frame(payload=bytes(range(256)) * 5 + b"x" * i, seq=i)) for i in range(7)]
    asks = [(i % 4 != 3, i % 4 in (0, 2)) for i in range(len(frames))]   # (IP, TCP): both, IP, both, none
    src = mosrx.mem_source(t.frames, t.off, t.len, loops=1)
    path = str(tmp_path / "tx.pcap")
    mosrx.source_tx_pcap(src, path)
    be = mosrx.GpuBackend([src], batch=1024, cpu=3, tx_batch=64, tx_csum=True)
    try:
        for f, (ip, tcp) in zip(frames, asks):
            assert be.send_offloaded(0, f, ip, tcp) == ((0 if ip else None), (0 if tcp else None))
        # not the last frame's IP header: refused, mOS would compute it
        assert be.ioctl_raw(0, mosrx.PKT_TX_IP_CSUM, C.c_void_p(0x1000)) == -1
        be.send_pkts(0)
        st = be.stats()
        assert st.tx_packets == len(frames) and st.tx_errors == 0
        assert st.tx_csum_offloaded == sum(1 for a in asks if any(a))
    finally:
        be.close()
    want = []
    for f, (ip, tcp) in zip(frames, asks):
        fl = (mosrx.TX_IP_CSUM if ip else 0) | (mosrx.TX_TCP_CSUM if tcp else 0)
        buf = np.frombuffer(f, np.uint8)
        want.append(bytes(O.tx_csum(buf, [0], [len(f)], fl)) if fl else f)
    assert mosrx.read_pcap(path) == want

    src = mosrx.mem_source(t.frames, t.off, t.len, loops=1)
    be = mosrx.GpuBackend([src], batch=1024, cpu=3, tx_csum=False)
    try:
        assert be.send_offloaded(0, frames[0], True, True) == (-1, -1)
    finally:
        be.close()


def _have_raw():
    try:
        socket.socket(socket.AF_PACKET, socket.SOCK_RAW, socket.htons(3)).close()
        return True
    except (PermissionError, OSError, AttributeError):
        return False


@pytest.mark.skipif(not _have_raw(), reason="needs CAP_NET_RAW for AF_PACKET")
def test_afpacket_ring_lent_zero_copy_to_the_backend():
    """The TPACKET_V3 ring registered with the HIP runtime: batches are runs of the
    ring itself (no host copy), given back to the kernel when recycled."""
    t = mosrx.Trace(mosrx.TRACE_IMIX, 6000, nflows=100)
    src = mosrx.afpacket_source("lo", ring_blocks=4)
    info = mosrx.afpacket_info(src)
    peer = socket.socket(socket.AF_PACKET, socket.SOCK_RAW, socket.htons(3))
    peer.bind(("lo", 0))
    be = mosrx.GpuBackend([src], batch=1024, cpu=12)
    got = []
    try:
        import time
        for k in range(0, t.n, 200):
            for i in range(k, min(k + 200, t.n)):
                peer.send(bytes(t.frames[t.off[i]:t.off[i] + t.len[i]]))
            time.sleep(0.003)
        t0 = time.time()
        while len(got) < t.n and time.time() - t0 < 10:
            n = be.recv_pkts(0)
            if n <= 0:
                time.sleep(0.002)
                continue
            r = be.results(0, n)
            got += [(be.get_rptr(0, i), r[i]) for i in range(n)]
    finally:
        be.close()
        peer.close()
    mine = [(f, r) for f, r in got if f[0:6] == bytes(t.frames[t.off[0]:t.off[0] + 6])]
    assert len(mine) == t.n
    assert [f for f, _ in mine] == [bytes(t.frames[o:o + n]) for o, n in zip(t.off, t.len)]
    ora = O.classify(t.frames, t.off, t.len, O.params())
    assert_records_equal(np.array([r for _, r in mine], mosrx.RESULT_DTYPE), ora, "afpacket")
    assert info.zero_copy == 1


def test_config1_simple_firewall_end_to_end(tmp_path):
    """BASELINE config #1 through the drop-in boundary: 10 000 x 60 B frames of
    one flow in a pcap file, read by the libpcap-free pcap source (pcap_next,
    pcap_module.c:41), classified by gpu_module_func in simple_firewall's state
    (num_msp 1, forward 1, num_queues 1, i40e map), consumed by RunMainLoop's rx
    loop (core.c:897-909) with the ForwardEthernetFrame consumer (eth_out.c:105-129)
    -- the frames mOS forwards in that state (mosrx_mos_forwards) -- whose frames leave
    through the source's TX (pcap_inject's place, here a pcap dump).  NETSTAT,
    the reason census and the forwarded frames equal what the oracle says mOS
    does; nothing is dropped or reordered."""
    t = mosrx.Trace(mosrx.TRACE_FW64, 10_000)
    path, out = str(tmp_path / "fw.pcap"), str(tmp_path / "out.pcap")
    write_pcap(path, t.frames, t.off, t.len)
    src = mosrx.lib().mosrx_source_pcap(path.encode(), 1)
    assert src
    mosrx.source_tx_pcap(src, out)
    be = mosrx.GpuBackend([src], params=mosrx.default_params(), batch=4096, cpu=13, timing=True)
    try:
        fwd = be.forwarder([0])
        st = be.run_loop(forward=fwd)
        ms = be.stats()
    finally:
        be.close()
    ora = O.classify(t.frames, t.off, t.len, O.params())
    assert st.rx_packets == t.n and st.batches == 3
    assert st.rx_bytes == int(t.len.astype(np.int64).sum()) + 24 * t.n     # + ETHER_OVR per frame
    assert st.rx_errors == int((ora["verdict"] < 0).sum())
    assert list(st.by_reason) == np.bincount(ora["reason"], minlength=NREASON).tolist()
    keep = np.nonzero(mos_forwarded(ora))[0]
    assert fwd.forwarded == len(keep) and fwd.dropped == t.n - len(keep)
    assert ms.tx_packets == len(keep) and ms.kernel_launches == 3
    sent = mosrx.read_pcap(out)
    assert sent == [bytes(t.frames[t.off[i]:t.off[i] + t.len[i]]) for i in keep]


def test_two_netdevs_forwarding_between_them(tmp_path):
    """Two netdevs behind one context (RunMainLoop walks every rx_inf, core.c:897),
    each with its own source and TX, frames forwarded across (the NIC forwarding
    table, eth_out.c:105-129: 0 -> 1, 1 -> 0): every netdev's census equals the
    oracle on its own trace, and each TX carries exactly the other netdev's
    accepted frames, in order."""
    ta = mosrx.Trace(mosrx.TRACE_IMIX, 7000, nflows=500, seed=21)
    tb = mosrx.Trace(mosrx.TRACE_M1500, 3000, nflows=500, seed=22)
    sa = mosrx.mem_source(ta.frames, ta.off, ta.len, loops=1, mode=mosrx.SRC_FILL)
    sb = mosrx.mem_source(tb.frames, tb.off, tb.len, loops=1)
    outa, outb = str(tmp_path / "a.pcap"), str(tmp_path / "b.pcap")
    mosrx.source_tx_pcap(sa, outa)
    mosrx.source_tx_pcap(sb, outb)
    be = mosrx.GpuBackend([sa, sb], batch=2048, cpu=14, group=2)
    by_if = {0: [], 1: []}
    try:
        while True:
            any_rx = False
            for i in (0, 1):
                n = be.recv_pkts(i)
                assert n >= 0
                if n:
                    any_rx = True
                    by_if[i].append(be.results(i, n))
            if not any_rx:
                break
    finally:
        be.close()
    ra, rb = np.concatenate(by_if[0]), np.concatenate(by_if[1])
    assert_records_equal(ra, O.classify(ta.frames, ta.off, ta.len, O.params()), "netdev 0")
    assert_records_equal(rb, O.classify(tb.frames, tb.off, tb.len, O.params()), "netdev 1")

    # the same two netdevs through the rx loop with the forwarding consumer
    sa = mosrx.mem_source(ta.frames, ta.off, ta.len, loops=1)
    sb = mosrx.mem_source(tb.frames, tb.off, tb.len, loops=1, mode=mosrx.SRC_PER_FRAME)
    mosrx.source_tx_pcap(sa, outa)
    mosrx.source_tx_pcap(sb, outb)
    be = mosrx.GpuBackend([sa, sb], batch=2048, cpu=15, tx_batch=32)
    try:
        fwd = be.forwarder([1, 0])
        st = be.run_loop(forward=fwd)
    finally:
        be.close()
    oa = O.classify(ta.frames, ta.off, ta.len, O.params())
    ob = O.classify(tb.frames, tb.off, tb.len, O.params())
    assert st.rx_packets == ta.n + tb.n
    ka, kb = np.nonzero(mos_forwarded(oa))[0], np.nonzero(mos_forwarded(ob))[0]
    assert fwd.forwarded == len(ka) + len(kb)
    assert mosrx.read_pcap(outb) == [bytes(ta.frames[ta.off[i]:ta.off[i] + ta.len[i]]) for i in ka]
    assert mosrx.read_pcap(outa) == [bytes(tb.frames[tb.off[i]:tb.off[i] + tb.len[i]]) for i in kb]


def test_two_mtcp_threads_run_concurrently():
    """One context per mTCP thread (core.c:1282-1349), each thread with its own
    source for the same netdev (mosrx_gpu_module_bind_source, as one
    PACKET_FANOUT socket per thread would be) and its own GPU context, both
    rx loops running at the same time on their own host threads: each thread's
    census equals the oracle on its own frames."""
    import ctypes as C
    import threading
    traces = [mosrx.Trace(mosrx.TRACE_IMIX, 20000, nflows=800, seed=31),
              mosrx.Trace(mosrx.TRACE_M1500, 6000, nflows=800, seed=32)]
    srcs = [mosrx.mem_source(t.frames, t.off, t.len, loops=3) for t in traces]
    L = mosrx.lib()
    cfg = mosrx.ModuleCfg()
    L.mosrx_gpu_module_cfg_default(C.byref(cfg))
    cfg.num_ifs, cfg.src[0], cfg.batch, cfg.ngpu, cfg.group = 1, srcs[0], 4096, 1, 2
    assert L.mosrx_gpu_module_configure(C.byref(cfg)) == 0
    m = mosrx.gpu_module()
    mosrx._VOIDFN(m.load_module_upper_half)()
    cpus = (40, 41)
    ctx_objs = [C.c_uint64(0xBEEF0000 + c) for c in cpus]
    ctxs = [C.addressof(o) for o in ctx_objs]
    for c, x, s in zip(cpus, ctxs, srcs):
        assert L.mosrx_gpu_module_bind(x, c) == 0
        assert L.mosrx_gpu_module_bind_source(c, 0, s) == 0
    for x in ctxs:
        mosrx._CTXFN(m.init_handle)(x)
    stats = [mosrx.RxStats(), mosrx.RxStats()]
    rcs = [None, None]
    opts = mosrx.RxLoopOpts(0, 1, 0, 0)

    def run(i):
        rcs[i] = L.mosrx_rx_loop_ex(C.addressof(m), ctxs[i], 1, C.byref(opts), None, None, C.byref(stats[i]))

    th = [threading.Thread(target=run, args=(i,)) for i in (0, 1)]
    try:
        for t in th:
            t.start()
        for t in th:
            t.join(60)
    finally:
        for x in ctxs:
            mosrx._CTXFN(m.destroy_handle)(x)
        for s in srcs:
            L.mosrx_source_close(s)
    assert rcs == [0, 0]
    for t, st in zip(traces, stats):
        ora = O.classify(t.frames, t.off, t.len, O.params())
        assert st.rx_packets == 3 * t.n
        assert list(st.by_reason) == (3 * np.bincount(ora["reason"], minlength=NREASON)).tolist()


# ---------------------------------------------------------------- inside mOS
MOS_LOOP = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle", "_ref",
                        "mos_gpu_loop")


def _raw_ip(s):
    return struct.unpack("<I", socket.inet_aton(s))[0]


@pytest.mark.skipif(not os.path.exists(MOS_LOOP),
                    reason="needs oracle/_ref/mos_gpu_loop (make -C oracle ref, built where /root/reference is)")
@pytest.mark.parametrize("fix,state,batch,period,forward", [
    ("edge", "msp1", 256, 0, 0), ("edge", "esp1_local", 100, 0, 0), ("edge", "noverify_local", 4096, 0, 0),
    ("rand_small", "q3_ixgbe", 128, 0, 0), ("rand_mid", "msp1_local", 64, 0, 0), ("rand_large", "q8_i40e", 50, 0, 0),
    ("imix_full", "msp1", 32768, 0, 0), ("m1500_full", "q4_i40e", 65536, 0, 0),
    # the stack state changes under the backend: num_msp toggles every `period` batches
    ("edge", "msp1_local", 64, 1, 0), ("rand_mid", "msp1", 50, 2, 0), ("imix_full", "msp1", 8192, 3, 0),
    # forward = 1 (simple_firewall): which frames mOS forwards, against mosrx_mos_forwards
    ("edge", "msp1", 128, 0, 1), ("edge", "noverify_local", 128, 0, 1), ("rand_small", "msp1_local", 64, 0, 1),
    ("rand_mid", "q4_i40e", 100, 2, 1), ("imix_full", "msp1", 32768, 0, 1),
    # several batches per launch (cfg.group), the stack state changing between groups
    ("rand_mid", "msp1", 32, (0, 8), 1), ("imix_full", "msp1_local", 4096, (16, 4), 0),
    # ... and inside a group (period not a multiple of group: the rest of the group
    # is classified again before its next batch is handed out); group 0 = auto
    ("edge", "msp1_local", 32, (1, 8), 0), ("rand_mid", "msp1", 16, (3, 8), 1),
    ("imix_full", "msp1", 4096, (5, 0), 1), ("edge", "q3_ixgbe", 16, (0, 0), 0)])
def test_backend_inside_mos_checked_by_processpacket(tmp_path, fix, state, batch, period, forward):
    """gpu_module_func compiled inside mOS's tree (its own io_module.h /
    config.h) and registered as core.c:1725-1736 does, fed from a trace, with
    mOS's own RunMainLoop rx section + ProcessPacket run on every frame get_rptr
    hands out (oracle/mos_gpu_loop.c, linked from mOS's compiled objects): every
    GPU verdict equals ProcessPacket's return value, every PKT_RX_RSS hash
    (mOS's RssInfo) equals GetRSSHash, load_module_upper_half set mOS's
    num_queues, and mOS's NETSTAT equals the GPU census.  With a period, mOS's
    num_msp changes every `period` batches (a monitor socket created / closed)
    and the backend follows it through the thread context with no call from
    the core, re-classifying the batch it had in flight.  With forward = 1
    mOS's ForwardIPPacket / ForwardEthernetFrame are recorded instead of
    transmitting, and the frames ProcessPacket forwards must be those
    mosrx_mos_forwards() picks from the GPU records (the rx loop's forwarding
    consumer)."""
    _inside_mos(tmp_path, fix, state, batch, period, forward)


@pytest.mark.skipif(not os.path.exists(MOS_LOOP),
                    reason="needs oracle/_ref/mos_gpu_loop (make -C oracle ref, built where /root/reference is)")
@pytest.mark.parametrize("fix,msp,esp,listen", [
    ("rand_mid", 1, 1, False), ("rand_mid", 1, 1, True), ("rand_small", 0, 1, True),
    ("imix_full", 1, 2, False), ("imix_full", 1, 2, True)])
def test_backend_inside_mos_forwarding_with_end_host_sockets(tmp_path, fix, msp, esp, listen):
    """forward = 1 with end-host sockets: a client socket leaves the forwarding of
    segments without a stream as it is (CreateStream's monitor stream / the orphan
    path, tcp.c:453-510); an end-host socket listening (mtcp->listener, on a port
    the trace does not use) turns the orphans into RSTs, not forwarded.  The GPU
    records + mosrx_mos_forwards(listener) against mOS's own ProcessPacket."""
    _inside_mos(tmp_path, fix, (msp, esp, 1, 1, ()), 256, 0, 1, listen=listen)


def _unused_tcp_port(frames, off, ln):
    """A port no TCP frame of the trace is sent to (the listener's SYNs would start end-host streams)."""
    frames, off, ln = np.asarray(frames), np.asarray(off, np.int64), np.asarray(ln, np.int64)
    ok = ln >= 38
    o = off[ok]
    tcp = (frames[o + 12] == 8) & (frames[o + 13] == 0) & (frames[o + 23] == 6)
    o = o[tcp]
    p = o + 14 + (frames[o + 14] & 0xF).astype(np.int64) * 4 + 2
    p = p[p + 2 <= len(frames)]
    used = set(((frames[p].astype(np.int64) << 8) | frames[p + 1]).tolist())
    return next(x for x in range(1, 65536) if x not in used)


def _inside_mos(tmp_path, fix, state, batch, period, forward, listen=False):
    import json
    import subprocess
    from pktlib import write_ref_trace
    from test_oracle_golden import GOLDEN, STATES
    msp, esp, nq, qm, loc = STATES[state] if isinstance(state, str) else state
    period, group = period if isinstance(period, tuple) else (period, 1)
    if fix == "imix_full":
        t = mosrx.Trace(mosrx.TRACE_IMIX, 262_144)
        frames, off, ln = t.frames, t.off, t.len
    elif fix == "m1500_full":
        t = mosrx.Trace(mosrx.TRACE_M1500, 65_536)
        frames, off, ln = t.frames, t.off, t.len
    else:
        z = np.load(os.path.join(GOLDEN, f"{fix}.npz"))
        frames, off, ln = z["frames"], z["off"], z["len"]
    path = str(tmp_path / "trace.in")
    write_ref_trace(path, frames, off, ln, num_msp=msp, num_esp=esp, forward=forward, num_queues=nq, queue_mode=qm,
                    local=[_raw_ip(a) for a in loc])
    env = dict(os.environ)
    env.pop("MOSREF_LISTENER", None)
    if listen:
        env["MOSREF_LISTENER"] = str(_unused_tcp_port(frames, off, ln))
    r = subprocess.run([MOS_LOOP, path, str(batch), str(period), str(group)], capture_output=True,
                       text=True, timeout=120, env=env)
    assert r.stdout.strip(), r.stderr
    d = json.loads(r.stdout.strip().splitlines()[-1])
    assert r.returncode == 0, (d, r.stderr[-2000:])
    assert d["frames"] == len(off) and d["verdict_diff"] == 0 and d["rss_diff"] == 0
    assert d["num_queues"] == nq and d["nstat_ok"] == 1
    assert d["compared"] + d["skipped"] == len(off) and d["compared"] > 0.5 * len(off)
    assert d["batches"] == -(-len(off) // batch)
    if period and group and period % group == 0:  # every change caught a group in flight (changes fall on
        # group boundaries: a group is classified under one state)
        assert d["reclassified"] == (d["batches"] - 1) // period * group
    elif period:                                  # changes inside groups: the rest of the group again
        assert d["reclassified"] >= (d["batches"] - 1) // period
    assert d["forward_diff"] == 0
    # with forwarding on, mOS forwards something unless only end-host sockets exist (msp 0, esp > 0)
    assert (d["forwarded_by_mos"] > 0) == bool(forward and (msp or not esp))
