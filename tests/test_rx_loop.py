"""CPU tests of mosrx_rx_loop_ex (csrc/rx_loop.c), the receive half of
RunMainLoop (core.c:897-909, :999-1007), over a scripted io_module_func whose
members are Python callbacks -- no GPU: the verdict records are made up.

Checked: NETSTAT accounting (eth_in.c:42-45, 80-84: rx_packets, rx_bytes +=
len + ETHER_OVR, rx_errors for negative verdicts), the per-reason census, the
consumer called once per frame in order, send_pkts once per netdev per round,
a recv_pkts < 0 skipped as RunMainLoop's loop skips it (counted), and the stop
conditions (max_pkts, idle rounds)."""
import ctypes as C

import numpy as np

import mosrx

ETHER_OVR = 24


class FakeBackend:
    """io_module_func whose recv_pkts plays a script: per round and netdev a
    batch size (int), -1 for a failed receive, 0 for idle."""

    def __init__(self, script, nif):
        self.script = list(script)
        self.nif = nif
        self.sent = [0] * nif
        self.cur = {}
        self.m = mosrx.IoModuleFunc()
        self._keep = []
        self._set("recv_pkts", mosrx._RECVFN(self.recv))
        self._set("get_rptr", mosrx._RPTRFN(self.rptr))
        self._set("dev_ioctl", mosrx._IOCTLFN(self.ioctl))
        self._set("send_pkts", mosrx._SENDFN(self.send))

    def _set(self, name, fn):
        self._keep.append(fn)
        setattr(self.m, name, C.cast(fn, C.c_void_p).value)

    def recv(self, ctx, ifidx):
        n = self.script.pop(0) if self.script else 0
        if n > 0:
            rng = np.random.default_rng(len(self.script) * 7 + ifidx)
            lens = rng.integers(60, 1515, n).astype(np.uint16)
            bufs = [C.create_string_buffer(rng.integers(0, 256, int(x), dtype=np.uint8).tobytes(), int(x))
                    for x in lens]
            rec = np.zeros(n, mosrx.RESULT_DTYPE)
            rec["verdict"] = rng.choice([-1, 0, 1], n)
            rec["reason"] = rng.integers(0, mosrx.NREASON, n)
            self.cur[ifidx] = (bufs, lens, np.ascontiguousarray(rec))
        return n

    def rptr(self, ctx, ifidx, i, plen):
        bufs, lens, _ = self.cur[ifidx]
        plen[0] = int(lens[i])
        return C.addressof(bufs[i])

    def ioctl(self, ctx, ifidx, cmd, argp):
        if cmd != mosrx.PKT_RX_RESULTS:
            return -1
        C.cast(argp, C.POINTER(C.c_void_p))[0] = self.cur[ifidx][2].ctypes.data
        return 0

    def send(self, ctx, ifidx):
        self.sent[ifidx] += 1
        return 0


def run(fb, max_pkts=0, idle_rounds=1, consumer=None):
    st = mosrx.RxStats()
    o = mosrx.RxLoopOpts(max_pkts, idle_rounds, 0, 0)
    fn = mosrx._PKTFN(consumer) if consumer else None
    rc = mosrx.lib().mosrx_rx_loop_ex(C.addressof(fb.m), None, fb.nif, C.byref(o),
                                      C.cast(fn, C.c_void_p) if fn else None, None, C.byref(st))
    return rc, st


def test_netstat_and_census_over_two_netdevs():
    seen = []

    def consumer(arg, ifidx, i, pkt, ln, res):
        seen.append((ifidx, i, ln, res.contents.verdict))

    # two netdevs, three busy rounds, then one idle round ends the loop
    fb = FakeBackend([5, 3, 0, 7, 4, 2, 0, 0], nif=2)
    recs = []
    orig = fb.recv

    def recv(ctx, ifidx):
        n = orig(ctx, ifidx)
        if n > 0:
            recs.append((ifidx, fb.cur[ifidx][1].copy(), fb.cur[ifidx][2].copy()))
        return n

    fb._set("recv_pkts", mosrx._RECVFN(recv))
    rc, st = run(fb, consumer=consumer)
    assert rc == 0
    lens = np.concatenate([r[1] for r in recs]).astype(np.int64)
    res = np.concatenate([r[2] for r in recs])
    assert st.rx_packets == len(lens) == 21
    assert st.rx_bytes == int(lens.sum()) + ETHER_OVR * len(lens)
    assert st.rx_errors == int((res["verdict"] < 0).sum())
    assert list(st.by_reason) == np.bincount(res["reason"], minlength=mosrx.NREASON).tolist()
    assert st.batches == 5 and st.rounds == 4
    assert fb.sent == [4, 4]                       # send_pkts once per netdev per round
    exp = [(ifx, i, int(ln[i]), int(r["verdict"][i])) for ifx, ln, r in recs for i in range(len(ln))]
    assert seen == exp                             # every frame once, in batch order


def test_failed_receive_is_skipped_like_runmainloop():
    # a round whose receives all failed counts as idle (a backend that keeps
    # failing cannot spin the loop forever): with 2 idle rounds allowed the
    # batch after the failure is still received
    fb = FakeBackend([4, -1, 6, 0, 0], nif=1)
    rc, st = run(fb, idle_rounds=2)
    assert rc == 0
    assert st.rx_packets == 10 and st.recv_errors == 1 and st.batches == 2
    fb = FakeBackend([4, -1, 6], nif=1)
    rc, st = run(fb, idle_rounds=1)
    assert rc == 0 and st.rx_packets == 4 and st.recv_errors == 1


def test_stop_conditions():
    fb = FakeBackend([8] * 10, nif=1)
    rc, st = run(fb, max_pkts=20)
    assert rc == 0 and st.rx_packets == 24       # stops after the round that crossed 20
    fb = FakeBackend([3, 0, 0, 3, 0, 0, 0], nif=1)
    rc, st = run(fb, idle_rounds=3)
    assert rc == 0 and st.rx_packets == 6        # two idle rounds in a row did not end it


def test_backend_without_results_is_refused():
    fb = FakeBackend([4], nif=1)
    fb._set("dev_ioctl", mosrx._IOCTLFN(lambda ctx, i, cmd, argp: -1))
    rc, _ = run(fb)
    assert rc == -95                              # -ENOTSUP: not a classifying backend


def test_forwarder_consumer_sends_what_mos_forwards():
    """mosrx_forward_frame as the rx loop's consumer (ForwardEthernetFrame,
    eth_out.c:105-129): frames the rule picks (mosrx_mos_forwards) are copied into
    get_wptr buffers of out_if[in_if] and leave with the round's send_pkts; netdev 1
    maps to -1 (no output netdev): its forwardable frames count as dropped."""
    fb = FakeBackend([6, 5, 9, 4, 0, 0], nif=2)
    recs, tx, sent_rounds = [], [], []
    orig = fb.recv

    def recv(ctx, ifidx):
        n = orig(ctx, ifidx)
        if n > 0:
            recs.append((ifidx, [bytes(C.string_at(C.addressof(b), len(b))) for b in fb.cur[ifidx][0]],
                         fb.cur[ifidx][2].copy()))
        return n

    bufs = []

    def wptr(ctx, ifidx, ln):
        b = C.create_string_buffer(ln)
        bufs.append(b)
        tx.append((ifidx, b))
        return C.addressof(b)

    def send(ctx, ifidx):
        sent_rounds.append((ifidx, len(tx)))
        return 0

    fb._set("recv_pkts", mosrx._RECVFN(recv))
    fb._set("get_wptr", mosrx._WPTRFN(wptr))
    fb._set("send_pkts", mosrx._SENDFN(send))
    fw = mosrx.Forwarder()
    fw.iom, fw.ctx = C.addressof(fb.m), None
    for i in range(16):
        fw.out_if[i] = -1
    fw.out_if[0] = 1
    fw.forward, fw.num_msp, fw.listener = 1, 1, 0
    st = mosrx.RxStats()
    o = mosrx.RxLoopOpts(0, 1, 0, 0)
    rc = mosrx.lib().mosrx_rx_loop_ex(C.addressof(fb.m), None, 2, C.byref(o),
                                      C.cast(mosrx.lib().mosrx_forward_frame, C.c_void_p), C.byref(fw), C.byref(st))
    assert rc == 0
    rule = mosrx.lib().mosrx_mos_forwards
    exp, drop = [], 0
    for ifidx, frames, rec in recs:
        for i, f in enumerate(frames):
            r = np.ascontiguousarray(rec[i:i + 1])
            if rule(C.c_void_p(r.ctypes.data), 1, 1, 0):
                if ifidx == 0:
                    exp.append(f)
                else:
                    drop += 1
            else:
                drop += 1
    assert fw.forwarded == len(exp) == len(tx) and fw.dropped == drop
    assert all(ifx == 1 for ifx, _ in tx)                      # out_if[0] = 1
    assert [b.raw for _, b in tx] == exp                       # copied byte for byte, in order
    assert len(sent_rounds) == 2 * st.rounds                   # send_pkts per netdev per round
