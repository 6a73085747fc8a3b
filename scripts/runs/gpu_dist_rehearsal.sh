# rehearsal of the multi-rank bench path (torchrun, gloo barrier/max) with two
# ranks sharing the box's one GPU, every default workload + the e2e leg; the
# numbers are not results (two ranks share one GPU)
set -o pipefail
mkdir -p gpurun_out
MOSRX_BENCH_DEVICE=0 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 5 \
  > gpurun_out/bench_dist2.log 2>&1; rc=$?
echo "torchrun rc=$rc"; grep "^\[bench\]" gpurun_out/bench_dist2.log; grep "^{" gpurun_out/bench_dist2.log | cut -c1-600
exit $rc
