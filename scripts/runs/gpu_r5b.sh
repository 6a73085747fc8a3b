# round 5: the layout hint A/B (same box, interleaved), the compact full-verdict ring,
# the backend tests, and the 2-rank torchrun rehearsal of the N>1 line on the one card
set -o pipefail
mkdir -p gpurun_out/r5b
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_backend_gpu.py tests/test_layout_hint.py tests/test_bpf_streams.py -m gpu -x -q \
  --timeout 120 --timeout-method thread > gpurun_out/r5b/pytest.log 2>&1; rc=$?
tail -2 gpurun_out/r5b/pytest.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
  for h in "" "--no-hint"; do
    timeout -k 10 200 python -u bench.py --workloads S64_1,S64,S64_c8,S64_hdr --no-cpu --no-e2e $h \
      --detail gpurun_out/r5b/ab_${r}${h}.json > gpurun_out/r5b/ab_${r}${h}.out 2> gpurun_out/r5b/ab_${r}${h}.err; rc=$?
    echo "ab round $r ${h:-hint} rc=$rc"; grep "^\[bench\]" gpurun_out/r5b/ab_${r}${h}.err
    [ $rc -ne 0 ] && exit $rc
  done
done
MOSRX_BENCH_DEVICE=0 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 10 --warmup 3 \
  --workloads M1500,S64,IMIX --detail gpurun_out/r5b/dist2_detail.json \
  > gpurun_out/r5b/bench_dist2.out 2> gpurun_out/r5b/bench_dist2.err; rc=$?
echo "dist2 rc=$rc"; tail -c 3000 gpurun_out/r5b/bench_dist2.out
exit $rc
