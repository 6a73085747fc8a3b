# round 5: four torchrun ranks on the box's one GPU through the whole N>1 bench path
# (every leg on every rank between barriers, rank-0 CPU legs after the last GPU
# barrier, job_share of 4 x 16 threads); a rehearsal of the driver's SCALE runs, not a result
set -o pipefail
mkdir -p gpurun_out/r5k
MOSRX_BENCH_DEVICE=0 timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 \
  --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 4 --steps 10 --warmup 3 \
  --workloads M1500,S64,S64_c8,IMIX,S64_1 --detail gpurun_out/r5k/dist4_detail.json \
  > gpurun_out/r5k/bench_dist4.out 2> gpurun_out/r5k/bench_dist4.err; rc=$?
echo "torchrun rc=$rc"; grep "^\[bench\]" gpurun_out/r5k/bench_dist4.err | head -20; tail -c 2500 gpurun_out/r5k/bench_dist4.out
exit $rc
