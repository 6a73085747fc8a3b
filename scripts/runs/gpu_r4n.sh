#!/bin/bash
# round 4: the hook's LDS window sized by header lanes (stream tile 64): parity, fused-cost timing
cd "${GRAFT_REPO_ROOT:-.}"
out=gpurun_out/r4n
mkdir -p $out
timeout -k 10 400 python -u -m pytest -v --maxfail=5 --timeout 120 --timeout-method thread -m gpu \
    tests/test_bpf.py tests/test_bpf_groups.py > $out/pytest_bpf.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $out/pytest_bpf.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 400 python -u scripts/probe_fused_cost.py S64 0,1,2 > $out/fused_S64.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/probe_fused_cost.py IMIX 0,1,2,9 > $out/fused_IMIX.log 2>&1 || exit $?
cat $out/fused_*.log
