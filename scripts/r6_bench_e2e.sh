# round 6: the bench's end-to-end / backend / latency legs alone (timing of each leg)
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6e
timeout -k 10 1000 python -u bench.py --workloads M1500,S64,IMIX --steps 5 --warmup 2 --no-cpu \
  --detail gpurun_out/r6e/bench_detail.json > gpurun_out/r6e/bench.out 2> gpurun_out/r6e/bench.err; rc=$?
grep "^\[bench" gpurun_out/r6e/bench.err | tail -60
exit $rc
