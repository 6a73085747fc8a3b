# round-1 full pass: tests, smoke, bench (default), rocprof kernel-trace of the
# headline bench command (1 stream), PMC FETCH_SIZE / WRITE_SIZE passes.
set -o pipefail
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
timeout -k 10 480 python -m pytest tests -m gpu -q -x --timeout=120 -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?
echo "smoke rc=$rc"; tail -3 gpurun_out/smoke.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py > gpurun_out/bench.log 2>&1; rc=$?
echo "bench rc=$rc"; grep "^\[bench\]" gpurun_out/bench.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/kt -o kt --output-format csv -- python3 bench.py --workloads M1500,S64,IMIX,M1500_tx,IMIX_bpf --streams 1 --no-cpu --no-e2e > gpurun_out/prof/kt_bench.log 2>&1; rc=$?
echo "kt rc=$rc"; tail -2 gpurun_out/prof/kt_bench.log
[ $rc -ne 0 ] && exit $rc
for W in M1500 IMIX S64; do
  timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof/pmcf_$W -o pmc --output-format csv -- python3 scripts/pmc_run.py $W 40 > gpurun_out/prof/pmcf_$W.log 2>&1; rc=$?
  echo "pmc fetch $W rc=$rc"; [ $rc -ne 0 ] && exit $rc
  timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/prof/pmcw_$W -o pmc --output-format csv -- python3 scripts/pmc_run.py $W 40 > gpurun_out/prof/pmcw_$W.log 2>&1; rc=$?
  echo "pmc write $W rc=$rc"; [ $rc -ne 0 ] && exit $rc
  python3 scripts/pmc_parse.py $W gpurun_out/prof/pmcf_$W gpurun_out/prof/pmcw_$W mosrx_classify_kernel gpurun_out/pmc_traffic.json
done
find gpurun_out/prof -name "*stats*" | head -20
exit 0
