#!/bin/bash
# 64 B ring attribution probe: one 8M-frame SMALL launch
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/r3_small
timeout -k 10 180 scripts/probe_small > gpurun_out/r3_small/s64.log 2>&1 || exit $?
cat gpurun_out/r3_small/s64.log
