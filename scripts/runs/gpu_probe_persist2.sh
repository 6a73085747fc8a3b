#!/bin/bash
# round 4: persistent grid with per-XCD counters, XCD remap, heaviest-first order
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/r4_persist
timeout -k 10 180 scripts/probe_persist2 3 262144 > gpurun_out/r4_persist/imix.log 2>&1 || exit $?
timeout -k 10 120 scripts/probe_persist2 2 65536 > gpurun_out/r4_persist/m1500.log 2>&1 || exit $?
cat gpurun_out/r4_persist/*.log
