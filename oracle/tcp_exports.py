#!/usr/bin/env python3
"""TEST INFRASTRUCTURE ONLY -- the upstream patch of INTEGRATION.md §2b, applied
on the fly: mOS's core/src/tcp.c with `static` dropped from the definitions
of DetectStreamType (tcp.c:25), CreateStream (:195), HandleSockStream (:275)
and HandleMonitorStream (:377), written to stdout for the compiler (the
Makefile pipes it into gcc; no copy of the source is kept).  Under
-fgnu89-inline a plain `inline` definition is an external one, as mOS's own
FillPacketContextTCPInfo (tcp.c:258) already is.  Exits non-zero if the four
definitions are not found exactly once each (the upstream file changed)."""
import re
import sys

NAMES = ("DetectStreamType", "CreateStream", "HandleSockStream", "HandleMonitorStream")


def main(path):
    src = open(path).read()
    for name in NAMES:
        src, n = re.subn(r"^static ((?:inline )?[^\n(]*)\n(%s\()" % name, r"\1\n\2", src, flags=re.M)
        if n != 1:
            sys.exit(f"tcp_exports: {name}: {n} definitions found, 1 expected")
    sys.stdout.write(src)


if __name__ == "__main__":
    main(sys.argv[1])
