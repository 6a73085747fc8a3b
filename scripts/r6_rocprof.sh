# round 6: rocprofv3 kernel-trace summary of the driver's bench command
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6prof
timeout -k 10 1100 rocprofv3 --kernel-trace --stats -d /tmp/r6prof -o kt --output-format csv -- \
  python3 bench.py --gpus 1 --steps 20 --warmup 5 --detail gpurun_out/r6prof/bench_detail.json \
  > gpurun_out/r6prof/bench.out 2> gpurun_out/r6prof/bench.err; rc=$?
find /tmp/r6prof -name "*stats.csv" -exec cp {} gpurun_out/r6prof/ \;
ls -la gpurun_out/r6prof
grep "^\[bench" gpurun_out/r6prof/bench.err | tail -5
head -c 600 gpurun_out/r6prof/bench.out
exit $rc
