#!/bin/bash
# finer tail tiles probe: IMIX 256K and 1500 B 64K single launches
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/r3_tail
timeout -k 10 180 scripts/probe_tail 3 262144 > gpurun_out/r3_tail/imix.log 2>&1 || exit $?
timeout -k 10 120 scripts/probe_tail 2 65536 > gpurun_out/r3_tail/m1500.log 2>&1 || exit $?
cat gpurun_out/r3_tail/*.log
