# round-1 re-measure after the stream-scan kernels: parity, bench, kernel-trace
# (1 stream) and PMC HBM traffic per workload
set -o pipefail
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout=120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_m.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_m.log
[ $rc -ne 0 ] && exit $rc
rm -f gpurun_out/pmc_traffic.json
for W in M1500 IMIX S64; do
  timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof/pmcf_$W -o pmc --output-format csv -- python3 scripts/pmc_run.py $W 40 > gpurun_out/prof/pmcf_$W.log 2>&1; rc=$?
  echo "pmc fetch $W rc=$rc"; [ $rc -ne 0 ] && exit $rc
  timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/prof/pmcw_$W -o pmc --output-format csv -- python3 scripts/pmc_run.py $W 40 > gpurun_out/prof/pmcw_$W.log 2>&1; rc=$?
  echo "pmc write $W rc=$rc"; [ $rc -ne 0 ] && exit $rc
  python3 scripts/pmc_parse.py $W gpurun_out/prof/pmcf_$W gpurun_out/prof/pmcw_$W mosrx_classify_kernel gpurun_out/pmc_traffic.json
done
cat gpurun_out/pmc_traffic.json
for W in M1500 IMIX S64; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/kt_$W -o kt --output-format csv -- python3 bench.py --workloads $W --streams 1 --no-cpu --no-e2e > gpurun_out/prof/kt_$W.log 2>&1; rc=$?
  echo "kt $W rc=$rc"; grep "^\[bench\]" gpurun_out/prof/kt_$W.log
  [ $rc -ne 0 ] && exit $rc
done
timeout -k 10 400 python -u bench.py > gpurun_out/bench_m.log 2>&1; rc=$?
echo "bench rc=$rc"; grep "^\[bench\]" gpurun_out/bench_m.log; tail -c 400 gpurun_out/bench_m.log
exit $rc
