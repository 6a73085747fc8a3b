#!/bin/bash
# A/B/C of library builds under scripts/ab/*/libmosrx.so (scripts/ab_lib.py), then
# the -m gpu parity file on the in-tree library.  Log under gpurun_out/.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 600 python -u scripts/ab_lib.py --rounds ${ROUNDS:-3} ${LIBS:-scripts/ab/A/libmosrx.so scripts/ab/B/libmosrx.so scripts/ab/C/libmosrx.so} 2>&1 | tee gpurun_out/ab_lib.log || exit $?
[ -n "$NOTEST" ] && exit 0
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_parity_gpu.py} -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_ab.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_ab.log
exit $rc
