# eight torchrun ranks sharing the box's one GPU through the driver's N=8 bench
# command (default workloads; shard_plan over 8 ranks, gloo barrier/max); a
# rehearsal of the code path, not a result
set -o pipefail
mkdir -p gpurun_out
MOSRX_BENCH_DEVICE=0 timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \
  --master-addr 127.0.0.1 --master-port 29581 bench.py --gpus 8 --steps ${STEPS:-5} --warmup 2 \
  > gpurun_out/bench_dist8.out 2> gpurun_out/bench_dist8.err; rc=$?
echo "torchrun rc=$rc"; grep "^\[bench\]" gpurun_out/bench_dist8.err; wc -c gpurun_out/bench_dist8.out
python3 -c "import json; d=json.loads(open('gpurun_out/bench_dist8.out').read().strip().splitlines()[-1]); print({k: d[k] for k in ('value','n_gpus','ms_per_step','scaling')})"
exit $rc
