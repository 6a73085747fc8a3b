# experiment: timing-stream hardware queues, IMIX shapes, LDS-staged BPF
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests -m gpu -q -x --timeout=120 -p no:cacheprovider -k "forced or bpf or tx" > gpurun_out/pytest_f.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_f.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python scripts/tune_streams.py > gpurun_out/streams_pool.log 2>&1; rc=$?
echo "streams rc=$rc"; cat gpurun_out/streams_pool.log
[ $rc -ne 0 ] && exit $rc
GPU_MAX_HW_QUEUES=8 timeout -k 10 200 python scripts/tune_streams.py > gpurun_out/streams_q8.log 2>&1; rc=$?
echo "streams q8 rc=$rc"; cat gpurun_out/streams_q8.log
[ $rc -ne 0 ] && exit $rc
TUNE_VARIANTS=2,14,18,22,26 TUNE_ROUNDS=3 TUNE_BW=0 TUNE_SCALE=0 timeout -k 10 300 python scripts/tune.py > gpurun_out/tune_shapes.log 2>&1; rc=$?
echo "tune rc=$rc"; cat gpurun_out/tune_shapes.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python bench.py --workloads M1500,IMIX_bpf,IMIX --no-cpu --no-e2e > gpurun_out/bench_f.log 2>&1; rc=$?
echo "bench rc=$rc"; grep "^\[bench\]" gpurun_out/bench_f.log
exit $rc
