# round 5: rocprofv3 kernel-trace summary of the driver's exact bench command (the
# contract's cross-check of the line's launch duration)
set -o pipefail
mkdir -p gpurun_out/r5p
export TMPDIR=/tmp
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d gpurun_out/r5p/kt -o kt --output-format csv -- \
  python3 bench.py --gpus 1 --steps 20 --warmup 5 --detail gpurun_out/r5p/bench_detail.json \
  > gpurun_out/r5p/bench.out 2> gpurun_out/r5p/bench.err; rc=$?
echo "rc=$rc"; grep "^\[bench\]" gpurun_out/r5p/bench.err | head -3
f=$(find gpurun_out/r5p/kt -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && cp "$f" gpurun_out/r5p/kt_kernel_stats.csv; du -sh gpurun_out/r5p/kt
rm -rf gpurun_out/r5p/kt   # (the full trace is far past the 64 MiB copy-back limit)
exit $rc
