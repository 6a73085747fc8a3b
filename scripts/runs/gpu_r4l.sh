#!/bin/bash
# round 4: LDS window copy for indexed loads at X other than 4 * ihl: parity, then the fused-cost probe per filter
cd "${GRAFT_REPO_ROOT:-.}"
out=gpurun_out/r4l
mkdir -p $out
timeout -k 10 400 python -u -m pytest -v --maxfail=5 --timeout 120 --timeout-method thread -m gpu \
    tests/test_bpf.py tests/test_bpf_groups.py > $out/pytest_bpf.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $out/pytest_bpf.log
if [ $rc -ne 0 ]; then exit $rc; fi
for m in 1 0; do
  MOSRX_BPF_PRED=$m timeout -k 10 400 python -u scripts/probe_fused_cost.py S64 0,1,2,9 > $out/fused_S64_pred$m.log 2>&1 || exit $?
  MOSRX_BPF_PRED=$m timeout -k 10 300 python -u scripts/probe_fused_cost.py IMIX 0,1,2 > $out/fused_IMIX_pred$m.log 2>&1 || exit $?
done
tail -n 4 $out/fused_*.log
