# round-5 validation record of the last tree (one record per round), in two calls:
#   PART=tests: the whole -m gpu suite and smoke()
#   PART=bench: the driver's bench command (timed) and a 2-rank torchrun rehearsal on the one card
set -o pipefail
mkdir -p gpurun_out/final
export TMPDIR=/tmp
if [ "${PART:-tests}" = tests ]; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread \
    > gpurun_out/final/pytest.log 2>&1; rc=$?
  tail -3 gpurun_out/final/pytest.log; [ $rc -ne 0 ] && exit $rc
  timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final/smoke.log 2>&1; rc=$?
  tail -3 gpurun_out/final/smoke.log
  exit $rc
fi
t0=$(date +%s)
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 --detail gpurun_out/final/bench_detail.json \
  > gpurun_out/final/bench.out 2> gpurun_out/final/bench.err; rc=$?
echo "bench rc=$rc wall $(( $(date +%s) - t0 )) s" | tee gpurun_out/final/bench.wall
grep "^\[bench\]" gpurun_out/final/bench.err; [ $rc -ne 0 ] && exit $rc
MOSRX_BENCH_DEVICE=0 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29535 bench.py --gpus 2 --steps 10 --warmup 3 \
  --workloads M1500,S64,S64_c8,IMIX --detail gpurun_out/final/dist2_detail.json \
  > gpurun_out/final/bench_dist2.out 2> gpurun_out/final/bench_dist2.err; rc=$?
echo "dist2 rc=$rc"
exit $rc
