"""mos.conf `forward = 1` against mOS's own ProcessPacket (CPU, no GPU).

tests/golden/forward.npz (tests/golden/make_golden_forward.py) holds, for the
frames of the edge / rand_* fixtures and six stack states, ProcessPacket's
verdicts with forwarding on and whether it forwarded each frame (the harness
wraps ForwardIPPacket / ForwardEthernetFrame and records the call).  Pinned
here:
  * the oracle's verdicts with forward = 1 (the GPU path's are pinned to the
    oracle bit-exactly, and to the same fixture in test_parity_gpu.py);
  * mosrx_mos_forwards (csrc/rx_loop.c), the rule the rx loop's forwarding
    consumer applies to the records, frame by frame;
and, where oracle/_ref/mosref is built, both on fresh random frames too."""
import ctypes as C
import os
import random

import numpy as np
import pytest

import mosrx
import oracle_py as O
from pktlib import R, pack_frames
from test_oracle_golden import FIXTURES, GOLDEN

FWD = np.load(os.path.join(GOLDEN, "forward.npz"))
LOCAL = ("10.0.0.2", "192.168.1.1", "172.16.9.77")
FSTATES = {  # name -> (num_msp, num_esp, netdev addresses, end-host listener); make_golden_forward.py
    "msp1": (1, 0, (), False), "noverify": (0, 0, (), False), "esp1": (0, 1, (), False),
    "msp1_esp1": (1, 1, (), False), "msp1_esp1_listen": (1, 1, (), True), "msp1_local": (1, 0, LOCAL, False),
}


def rule(rec, forward, msp, listener):
    """mosrx_mos_forwards over every record, through the C ABI."""
    L = mosrx.lib()
    rec = np.ascontiguousarray(rec)
    base, step = rec.ctypes.data, rec.dtype.itemsize
    return np.array([L.mosrx_mos_forwards(C.c_void_p(base + step * i), forward, msp, int(listener))
                     for i in range(len(rec))], np.uint8)


def check(rec_oracle, verdict, fwd, have, msp, listener):
    skipped = (have & 8) != 0
    np.testing.assert_array_equal(rec_oracle["reason"] == R["TRUNCATED"], skipped)
    live = ~skipped
    np.testing.assert_array_equal(rec_oracle["verdict"][live], verdict[live], err_msg="verdict, forward=1")
    mine = rule(rec_oracle, 1, msp, listener)
    bad = np.nonzero(live & (mine != fwd))[0]
    assert not len(bad), [(int(i), int(rec_oracle["reason"][i]), int(fwd[i]), int(mine[i])) for i in bad[:8]]
    assert not mine[skipped].any()                 # frames mOS never processes are not forwarded


@pytest.mark.parametrize("fix", FIXTURES)
@pytest.mark.parametrize("state", list(FSTATES))
def test_forwarding_matches_processpacket(fix, state):
    z = np.load(os.path.join(GOLDEN, f"{fix}.npz"))
    msp, esp, loc, listen = FSTATES[state]
    ora = O.classify(z["frames"], z["off"], z["len"], O.params(num_msp=msp, num_esp=esp, forward=1, local=loc))
    k = f"{fix}__{state}__"
    check(ora, FWD[k + "verdict"], FWD[k + "fwd"], FWD[k + "have"], msp, listen)


def test_fixture_covers_every_forwarding_path():
    """Each rule row is exercised: frames forwarded and frames kept, per state."""
    n = {s: sum(int(FWD[f"{fx}__{s}__fwd"].sum()) for fx in FIXTURES) for s in FSTATES}
    assert n["esp1"] == 0                          # no monitor socket: only NOVERIFY forwards, none here
    assert n["noverify"] > n["msp1"] > n["msp1_esp1_listen"] > 0
    assert n["msp1_esp1"] == n["msp1"]             # client sockets do not change it, a listener does


def test_forward_off_forwards_nothing():
    rec = np.zeros(mosrx.NREASON, mosrx.RESULT_DTYPE)
    rec["reason"] = np.arange(mosrx.NREASON)
    for msp in (0, 1):
        for listen in (0, 1):
            assert not rule(rec, 0, msp, listen).any()


@pytest.mark.skipif(not O.have_ref(), reason="oracle/_ref/mosref not built (needs /root/reference)")
@pytest.mark.parametrize("seed", [11, 12])
def test_forwarding_fuzz_vs_reference(seed):
    from golden.make_golden import random_frames
    rng = random.Random(seed)
    frames = random_frames(rng, 300, seed % 3)
    buf, off, ln = pack_frames(frames, phase=rng.choice([2, 3, 6]))
    port = int(FWD["listen_port"][0])
    for msp, esp, listen in [(1, 0, False), (1, 1, True), (0, 0, False), (2, 3, False)]:
        rec, _ = O.run_ref(buf, off, ln, num_msp=msp, num_esp=esp, forward=1,
                           listen_port=port if listen else None)
        ora = O.classify(buf, off, ln, O.params(num_msp=msp, num_esp=esp, forward=1))
        check(ora, rec["verdict"], rec["fwd"].astype(np.uint8), rec["have"], msp, listen)
    rec, _ = O.run_ref(buf, off, ln, num_msp=1, forward=0)      # forwarding off: mOS forwards nothing
    assert not rec["fwd"].any()
