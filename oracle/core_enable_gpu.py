#!/usr/bin/env python3
"""TEST INFRASTRUCTURE ONLY -- the core.c half of INTEGRATION.md §2 (the
ENABLE_GPU build), applied on the fly: mOS's core/src/core.c with one more
branch in mtcp_init's compile-time backend choice (core.c:1725-1733),

    #elif defined(ENABLE_GPU)
        current_iomodule_func = &gpu_module_func;

written to stdout for the compiler (the Makefile pipes it into gcc with
-DENABLE_GPU; no copy of the source is kept).  The declaration
io_module.h:100-111 would carry is made at block scope in the branch itself.
Exits non-zero if the netmap branch it follows is not found exactly once."""
import re
import sys


def main(path):
    src = open(path).read()
    src, n = re.subn(r"(#elif defined\(ENABLE_NETMAP\)\n\s*current_iomodule_func = &netmap_module_func;\n)",
                     r"\1#elif defined(ENABLE_GPU)\n"
                     r"\t{ extern io_module_func gpu_module_func; current_iomodule_func = &gpu_module_func; }\n",
                     src)
    if n != 1:
        sys.exit(f"core_enable_gpu: the netmap branch of mtcp_init: {n} found, 1 expected")
    sys.stdout.write(src)


if __name__ == "__main__":
    main(sys.argv[1])
