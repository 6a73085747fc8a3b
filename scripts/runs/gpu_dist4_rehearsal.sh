# four torchrun ranks sharing the box's one GPU through the multi-rank bench path
# (shard_plan over 4 ranks, gloo barrier/max); a rehearsal, not a result
set -o pipefail
mkdir -p gpurun_out
MOSRX_BENCH_DEVICE=0 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 \
  --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 4 --steps 10 --warmup 2 \
  --workloads M1500,IMIX,S64_1 > gpurun_out/bench_dist4.log 2>&1; rc=$?
echo "torchrun rc=$rc"; grep "^\[bench\]" gpurun_out/bench_dist4.log; grep "^{" gpurun_out/bench_dist4.log | cut -c1-300
exit $rc
