#!/bin/bash
# round 4: the driver's bench command with the LDS indexed loads (full record in the detail file)
cd "${GRAFT_REPO_ROOT:-.}"
out=gpurun_out/r4m
mkdir -p $out
timeout -k 10 900 python -u bench.py --gpus 1 --steps 20 --warmup 5 --detail $out/bench_detail.json > $out/bench.out 2> $out/bench.err || exit $?
cat $out/bench.out
