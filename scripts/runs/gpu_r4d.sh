#!/bin/bash
# round 4: BPF parity after the fused hook's speculative indexed loads, then the
# new bench rows and the persistent-grid probe.  A failure ends the script.
cd "${GRAFT_REPO_ROOT:-.}"
out=gpurun_out/r4d
mkdir -p $out
timeout -k 10 400 python -u -m pytest -v --maxfail=5 --timeout 120 --timeout-method thread -m gpu \
    tests/test_bpf.py tests/test_bpf_groups.py > $out/pytest_bpf.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $out/pytest_bpf.log
if [ $rc -ne 0 ]; then exit $rc; fi
bash scripts/runs/gpu_r4c.sh || exit $?
bash scripts/runs/gpu_probe_persist2.sh
