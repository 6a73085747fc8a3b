# round 5: eight torchrun ranks on the box's one GPU through the N>1 bench path (the
# shape of the driver's 8-GPU SCALE run: gloo barriers / gathers over 8 ranks, every
# leg on every rank, rank-0 CPU legs after the last GPU barrier); a rehearsal, not a result
set -o pipefail
mkdir -p gpurun_out/r5m
MOSRX_BENCH_DEVICE=0 timeout -k 10 1000 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \
  --master-addr 127.0.0.1 --master-port 29547 bench.py --gpus 8 --steps 10 --warmup 3 \
  --workloads M1500,S64_c8,S64_1 --detail gpurun_out/r5m/dist8_detail.json \
  > gpurun_out/r5m/bench_dist8.out 2> gpurun_out/r5m/bench_dist8.err; rc=$?
echo "torchrun rc=$rc"; grep "^\[bench\]" gpurun_out/r5m/bench_dist8.err | head; tail -c 1200 gpurun_out/r5m/bench_dist8.out
exit $rc
