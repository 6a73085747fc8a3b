# round-1 refresh of every judged artefact from the current tree: GPU parity
# tests, smoke, PMC HBM traffic (separate FETCH/WRITE passes), rocprofv3
# kernel-trace summaries (1 stream) per workload, then the default bench.
set -o pipefail
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?
cat gpurun_out/smoke.log; [ $rc -ne 0 ] && exit $rc
rm -f gpurun_out/pmc_traffic.json
for W in ${PMC_W:-M1500 IMIX S64}; do
  timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof/pmcf_$W -o pmc --output-format csv -- python3 scripts/pmc_run.py $W 40 > gpurun_out/prof/pmcf_$W.log 2>&1; rc=$?
  echo "pmc fetch $W rc=$rc"; [ $rc -ne 0 ] && exit $rc
  timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/prof/pmcw_$W -o pmc --output-format csv -- python3 scripts/pmc_run.py $W 40 > gpurun_out/prof/pmcw_$W.log 2>&1; rc=$?
  echo "pmc write $W rc=$rc"; [ $rc -ne 0 ] && exit $rc
  python3 scripts/pmc_parse.py $W gpurun_out/prof/pmcf_$W gpurun_out/prof/pmcw_$W mosrx_classify_kernel gpurun_out/pmc_traffic.json
done
[ -f gpurun_out/pmc_traffic.json ] && cp gpurun_out/pmc_traffic.json profiles/pmc_traffic.json
for W in ${KT_W:-M1500 IMIX S64 S64_queue M1500_queue M1500_fh M1500_tx IMIX_bpf IMIX_cls_bpf}; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/kt_$W -o kt --output-format csv -- python3 bench.py --workloads $W --streams 1 --no-cpu --no-e2e > gpurun_out/prof/kt_$W.log 2>&1; rc=$?
  echo "kt $W rc=$rc"; grep "^\[bench\]" gpurun_out/prof/kt_$W.log
  [ $rc -ne 0 ] && exit $rc
done
timeout -k 10 600 python -u bench.py > gpurun_out/bench_r.log 2>&1; rc=$?
echo "bench rc=$rc"; grep "^\[bench\]" gpurun_out/bench_r.log
exit $rc
