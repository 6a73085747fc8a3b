#!/bin/bash
# Toeplitz-form probe: 1500 B 64K and IMIX 256K single launches
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/r3_rss
timeout -k 10 120 scripts/probe_rss 2 65536 > gpurun_out/r3_rss/m1500.log 2>&1 || exit $?
timeout -k 10 180 scripts/probe_rss 3 262144 > gpurun_out/r3_rss/imix.log 2>&1 || exit $?
cat gpurun_out/r3_rss/*.log
