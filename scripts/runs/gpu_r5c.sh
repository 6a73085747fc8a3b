# round 5: rocprof A/B of the layout hint on config #2's single launch (same box,
# alternating), the default bench (driver's N=1 command), the 2-rank rehearsal
set -o pipefail
mkdir -p gpurun_out/r5c
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_layout_hint.py -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/r5c/pytest.log 2>&1; rc=$?
tail -1 gpurun_out/r5c/pytest.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
  for h in "" "--no-hint"; do
    d=gpurun_out/r5c/kt_S64_1_${r}${h}
    timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $d -o kt --output-format csv -- \
      python3 bench.py --workloads S64_1 --streams 1 --no-cpu --no-e2e $h > $d.log 2>&1; rc=$?
    echo "kt S64_1 $r ${h:-hint} rc=$rc"; [ $rc -ne 0 ] && exit $rc
    grep classify $(find $d -name "*kernel_stats.csv") | cut -c1-60,190-260
  done
done
timeout -k 10 900 python -u bench.py --steps 20 --warmup 5 --detail gpurun_out/r5c/bench_detail.json \
  > gpurun_out/r5c/bench.out 2> gpurun_out/r5c/bench.err; rc=$?
echo "bench rc=$rc"; grep "^\[bench\]" gpurun_out/r5c/bench.err; [ $rc -ne 0 ] && exit $rc
MOSRX_BENCH_DEVICE=0 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 10 --warmup 3 \
  --workloads M1500,S64,IMIX --detail gpurun_out/r5c/dist2_detail.json \
  > gpurun_out/r5c/bench_dist2.out 2> gpurun_out/r5c/bench_dist2.err; rc=$?
echo "dist2 rc=$rc"
exit $rc
