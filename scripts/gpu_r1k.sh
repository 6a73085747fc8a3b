# stream_scan as default (S13/S14): full parity, smoke, probe, default bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout=120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_k.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_k.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_k.log 2>&1; rc=$?
echo "smoke rc=$rc"; tail -2 gpurun_out/smoke_k.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 100 ./scripts/probe_classify 2 65536 > gpurun_out/probe_stream_scan.log 2>&1 && timeout -k 10 100 ./scripts/probe_classify 3 262144 >> gpurun_out/probe_stream_scan.log 2>&1; rc=$?
cat gpurun_out/probe_stream_scan.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u bench.py > gpurun_out/bench_k.log 2>&1; rc=$?
echo "bench rc=$rc"; grep "^\[bench\]" gpurun_out/bench_k.log; tail -c 1500 gpurun_out/bench_k.log
exit $rc
