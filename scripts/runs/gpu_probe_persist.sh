#!/bin/bash
# persistent-grid probe: 1500 B 64K and IMIX 256K single launches
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/r3_persist
timeout -k 10 120 scripts/probe_persist 2 65536 > gpurun_out/r3_persist/m1500.log 2>&1 || exit $?
timeout -k 10 180 scripts/probe_persist 3 262144 > gpurun_out/r3_persist/imix.log 2>&1 || exit $?
cat gpurun_out/r3_persist/*.log
