#!/bin/bash
# finer tail tiles, sweep 1: 1500 B 64K and IMIX 256K single launches
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/r3_tail2
timeout -k 10 120 scripts/probe_tail 2 65536 1 > gpurun_out/r3_tail2/m1500.log 2>&1 || exit $?
timeout -k 10 180 scripts/probe_tail 3 262144 1 > gpurun_out/r3_tail2/imix.log 2>&1 || exit $?
cat gpurun_out/r3_tail2/*.log
