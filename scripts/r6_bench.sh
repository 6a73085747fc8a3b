# round 6: the driver's bench command
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6bench
timeout -k 10 1000 python -u bench.py --gpus 1 --steps 20 --warmup 5 --detail gpurun_out/r6bench/bench_detail.json \
  > gpurun_out/r6bench/bench.out 2> gpurun_out/r6bench/bench.err; rc=$?
grep "^\[bench" gpurun_out/r6bench/bench.err | tail -70
tail -c 3000 gpurun_out/r6bench/bench.out
exit $rc
