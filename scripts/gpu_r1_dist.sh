# rehearsal of the multi-rank bench path (torchrun, gloo barrier/max) with two
# ranks sharing the box's one GPU; the numbers are not results
set -o pipefail
mkdir -p gpurun_out
MOSRX_BENCH_DEVICE=0 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 200 --warmup 20 \
  --workloads M1500,S64_queue > gpurun_out/bench_dist2.log 2>&1; rc=$?
echo "torchrun rc=$rc"; grep "^\[bench\]" gpurun_out/bench_dist2.log; grep "^{" gpurun_out/bench_dist2.log | cut -c1-400
exit $rc
