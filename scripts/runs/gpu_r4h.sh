#!/bin/bash
# round 4: BPF parity with the if-converted (predicated) programs, then the fused-cost probe branchy vs predicated
cd "${GRAFT_REPO_ROOT:-.}"
out=gpurun_out/r4h
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
tail -n 12 $out/fused_*.log
