#!/bin/bash
# round 4: the fused 64 B ring's cost per filter (8 copies of each bench filter)
cd "${GRAFT_REPO_ROOT:-.}"
out=gpurun_out/r4k
mkdir -p $out
timeout -k 10 400 python -u scripts/probe_fused_cost.py S64 0,1,2,3,4,5,6,7,8,9,10 > $out/fused_each.log 2>&1 || exit $?
cat $out/fused_each.log
