#!/bin/bash
# round 4: dynamic instruction counts of the fused 64 B ring (plain / 8 x ret / 8 filters), branchy vs predicated
cd "${GRAFT_REPO_ROOT:-.}"
out=gpurun_out/r4i
mkdir -p $out
export PROBE_SHORT=1
for m in 0 1; do
  for k in 0 1 2; do
    MOSRX_BPF_PRED=$m timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_INSTS_BRANCH \
      --kernel-trace -d $out/p${m}_s$k -o run --output-format csv -- python3 scripts/probe_fused_cost.py S64 $k > $out/p${m}_s$k.log 2>&1 || exit $?
  done
done
ls -R $out | head -40
