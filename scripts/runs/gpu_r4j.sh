#!/bin/bash
# round 4: if-converted BPF with liveness-driven selects: parity, fused-cost timing (branchy vs predicated), PMC counts
cd "${GRAFT_REPO_ROOT:-.}"
out=gpurun_out/r4j
mkdir -p $out
timeout -k 10 400 python -u -m pytest -v --maxfail=5 --timeout 120 --timeout-method thread -m gpu \
    tests/test_bpf.py tests/test_bpf_groups.py > $out/pytest_bpf.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $out/pytest_bpf.log
if [ $rc -ne 0 ]; then exit $rc; fi
for w in S64 IMIX; do
  for m in 0 1; do
    MOSRX_BPF_PRED=$m timeout -k 10 300 python -u scripts/probe_fused_cost.py $w > $out/fused_${w}_pred$m.log 2>&1 || exit $?
  done
done
tail -n 3 $out/fused_*.log
PROBE_SHORT=1 MOSRX_BPF_PRED=1 timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_INSTS_BRANCH \
  --kernel-trace -d $out/p1_s2 -o run --output-format csv -- python3 scripts/probe_fused_cost.py S64 2 > $out/p1_s2.log 2>&1 || exit $?
