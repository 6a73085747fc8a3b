# two torchrun ranks sharing the box's one GPU through the driver's N=2 bench
# command (default workloads; shard_plan over 2 ranks, gloo barrier/max, each
# rank bound to its GPU's NUMA node before its first GPU call); a rehearsal of
# the code path, not a result
set -o pipefail
mkdir -p gpurun_out/dist2
MOSRX_BENCH_DEVICE=0 timeout -k 10 700 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29582 bench.py --gpus 2 --steps ${STEPS:-5} --warmup 2 \
  > gpurun_out/dist2/bench_dist2.out 2> gpurun_out/dist2/bench_dist2.err; rc=$?
echo "torchrun rc=$rc"; grep "^\[bench\]" gpurun_out/dist2/bench_dist2.err | head -30; wc -c gpurun_out/dist2/bench_dist2.out
python3 -c "import json; d=json.loads(open('gpurun_out/dist2/bench_dist2.out').read().strip().splitlines()[-1]); print({k: d[k] for k in ('value','n_gpus','ms_per_step','scaling')})"
exit $rc
