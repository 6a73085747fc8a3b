#!/bin/bash
# the bench's dispatch-stamped launch_us against rocprofv3's kernel-trace
# average of the same command (headline ring and the single-launch rows)
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r3e
for W in M1500 M1500_1 IMIX_1 IMIX S64; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r3e/kt_$W -o kt --output-format csv -- \
      python3 bench.py --workloads $W --streams 1 --no-cpu --no-e2e --detail gpurun_out/r3e/detail_$W.json \
      > gpurun_out/r3e/kt_$W.log 2>&1; rc=$?
  echo "kt $W rc=$rc"; grep "^\[bench\]" gpurun_out/r3e/kt_$W.log
  [ $rc -ne 0 ] && exit $rc
done
exit 0
