#!/bin/bash
# one box: the bench's launch timings without a profiler, then the same command
# under rocprofv3 --kernel-trace (which kernel duration agrees with the trace)
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r3f
W=M1500,M1500_1,IMIX_1,S64_1
timeout -k 10 300 python3 bench.py --workloads $W --streams 1 --no-cpu --no-e2e --detail gpurun_out/r3f/plain.json \
    > gpurun_out/r3f/plain.out 2> gpurun_out/r3f/plain.err; rc=$?
echo "plain rc=$rc"; grep "^\[bench\]" gpurun_out/r3f/plain.err; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r3f/kt -o kt --output-format csv -- \
    python3 bench.py --workloads $W --streams 1 --no-cpu --no-e2e --detail gpurun_out/r3f/prof.json \
    > gpurun_out/r3f/prof.log 2>&1; rc=$?
echo "prof rc=$rc"; grep "^\[bench\]" gpurun_out/r3f/prof.log
exit $rc
