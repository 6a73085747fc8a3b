mkdir -p gpurun_out
timeout -k 10 480 python -m pytest tests -m gpu -q --timeout=120 -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -30 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -5 gpurun_out/smoke.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 50 --warmup 5 > gpurun_out/bench.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -8 gpurun_out/bench.log
exit $rc
