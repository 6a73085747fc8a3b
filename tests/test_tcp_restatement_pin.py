"""The consumer's unpatched build restates four static functions of mOS's
tcp.c (csrc/mos_rx.c:370-472: DetectStreamType + CreateServerStream,
CreateStream, HandleSockStream's call, HandleMonitorStream).  Nothing else
would notice if tcp.c changed under that restatement, so its text is pinned
here: a digest of each restated range, taken from the reference this build was
checked against.  Skipped when the reference tree is absent (the GPU box).

When this fails, tcp.c changed: re-read the range, bring mos_rx.c's
restatement (or the line citations) up to date, run test_mos_consumer.py in
both builds (mos_app and the patched mos_app_x of INTEGRATION.md §2b, which
calls mOS's own functions and is the recommended build), then re-pin."""
import hashlib
import os

import pytest

TCP_C = "/root/reference/core/src/tcp.c"

# (first line, last line) of tcp.c -> sha256 of the lines, trailing blanks stripped
PINNED = {
    (25, 109): "5fe7f6392c8c2ddc3a122308bb843ad3f68e90670ae1f0ade451476c4d83ed39",    # DetectStreamType, CreateServerStream
    (195, 256): "2f78038ad3e7560cae1f81e75bc233f3ee92ddb3510b29565ac8e337056d2d7e",   # CreateStream
    (275, 281): "87f1e0f1253f8029a1fb240b6220db257125d6957f1af3cd0865556274542044",   # HandleSockStream
    (377, 406): "5b08eb2a992822209691e0777b4202cb683b4bbaccaa44a758fa59a62e1f867f",   # HandleMonitorStream
}


def _digest(lines, a, b):
    return hashlib.sha256("\n".join(x.rstrip() for x in lines[a - 1:b]).encode()).hexdigest()


@pytest.mark.skipif(not os.path.exists(TCP_C), reason="reference tree absent")
@pytest.mark.parametrize("span", sorted(PINNED))
def test_restated_tcp_c_range_unchanged(span):
    with open(TCP_C) as fh:
        lines = fh.read().split("\n")
    a, b = span
    assert _digest(lines, a, b) == PINNED[span], (
        f"tcp.c:{a}-{b} changed since the consumer's restatement was written: update "
        f"mos-networking-stack_amd/csrc/mos_rx.c:370-472 (or build with the INTEGRATION.md §2b patch, "
        f"-DMOSRX_MOS_TCP_EXPORTS) and re-pin")


def test_restatement_cites_the_pinned_ranges():
    """mos_rx.c's restatement names the ranges this file pins (no reference needed)."""
    src = open(os.path.join(os.path.dirname(__file__), "..", "mos-networking-stack_amd", "csrc", "mos_rx.c")).read()
    for cite in ("tcp.c:25-85", "tcp.c:87-109", "tcp.c:195-256", "tcp.c:275-281", "tcp.c:377-406"):
        assert cite in src, cite
