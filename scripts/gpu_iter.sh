# quick iteration: GPU parity tests, then device-resident bench (no CPU / e2e legs)
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests -m gpu -q -x --timeout=120 -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 100 --warmup 10 --no-cpu --no-e2e ${BENCH_ARGS} > gpurun_out/bench.log 2>&1; rc=$?
echo "bench rc=$rc"; grep "^\[bench\]" gpurun_out/bench.log
exit $rc
