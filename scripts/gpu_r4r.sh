#!/bin/bash
# round 4: the standalone BPF kernel's stage sized to the set vs 96 bytes (A/B), parity first
cd "${GRAFT_REPO_ROOT:-.}"
out=gpurun_out/r4r
mkdir -p $out
timeout -k 10 400 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu tests/test_bpf.py tests/test_bpf_groups.py > $out/pytest_bpf.log 2>&1 || { tail -5 $out/pytest_bpf.log; exit 1; }
tail -1 $out/pytest_bpf.log
for rep in 1 2; do
  timeout -k 10 200 python -u bench.py --workloads IMIX_bpf --no-cpu --no-e2e 2>&1 | grep "^\[bench\]" | sed "s/^/sized  /"
  MOSRX_BPF_STAGE96=1 timeout -k 10 200 python -u bench.py --workloads IMIX_bpf --no-cpu --no-e2e 2>&1 | grep "^\[bench\]" | sed "s/^/96B    /"
done
