#!/bin/bash
# round 4: BPF parity with the fast (check-free) program copies, then the fused-cost probe
cd "${GRAFT_REPO_ROOT:-.}"
out=gpurun_out/r4g
mkdir -p $out
timeout -k 10 400 python -u -m pytest -v --maxfail=5 --timeout 120 --timeout-method thread -m gpu \
    tests/test_bpf.py tests/test_bpf_groups.py > $out/pytest_bpf.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $out/pytest_bpf.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u scripts/probe_fused_cost.py S64 > $out/fused_s64.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/probe_fused_cost.py IMIX > $out/fused_imix.log 2>&1 || exit $?
cat $out/fused_*.log
