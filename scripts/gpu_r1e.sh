# bench (device legs) + one rocprofv3 kernel-trace pass per workload (1 stream,
# so the trace average is the isolated per-launch duration bench's roofline uses)
set -o pipefail
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --no-cpu --no-e2e > gpurun_out/bench_dev.log 2>&1; rc=$?
echo "bench rc=$rc"; grep "^\[bench\]" gpurun_out/bench_dev.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python bench.py --workloads M1500,IMIX,S64 --streams 1 --no-cpu --no-e2e > gpurun_out/bench_1s.log 2>&1; rc=$?
echo "bench 1-stream rc=$rc"; grep "^\[bench\]" gpurun_out/bench_1s.log
[ $rc -ne 0 ] && exit $rc
for W in M1500 IMIX S64 M1500_tx IMIX_bpf M1500_fh; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/kt_$W -o kt --output-format csv -- python3 bench.py --workloads $W --streams 1 --no-cpu --no-e2e > gpurun_out/prof/kt_$W.log 2>&1; rc=$?
  echo "kt $W rc=$rc"; grep "^\[bench\]" gpurun_out/prof/kt_$W.log
  [ $rc -ne 0 ] && exit $rc
done
exit 0
