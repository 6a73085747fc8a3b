# round-1 evidence for the current kernels: PMC HBM traffic (separate FETCH/WRITE
# passes), rocprofv3 kernel-trace summaries (1 stream), then the default bench
set -o pipefail
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
rm -f gpurun_out/pmc_traffic.json
for W in M1500 IMIX S64; do
  timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof/pmcf_$W -o pmc --output-format csv -- python3 scripts/pmc_run.py $W 40 > gpurun_out/prof/pmcf_$W.log 2>&1; rc=$?
  echo "pmc fetch $W rc=$rc"; [ $rc -ne 0 ] && exit $rc
  timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/prof/pmcw_$W -o pmc --output-format csv -- python3 scripts/pmc_run.py $W 40 > gpurun_out/prof/pmcw_$W.log 2>&1; rc=$?
  echo "pmc write $W rc=$rc"; [ $rc -ne 0 ] && exit $rc
  python3 scripts/pmc_parse.py $W gpurun_out/prof/pmcf_$W gpurun_out/prof/pmcw_$W mosrx_classify_kernel gpurun_out/pmc_traffic.json
done
cp gpurun_out/pmc_traffic.json profiles/pmc_traffic.json
for W in M1500 IMIX S64 S64_queue M1500_queue M1500_fh M1500_tx IMIX_bpf; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/kt_$W -o kt --output-format csv -- python3 bench.py --workloads $W --streams 1 --no-cpu --no-e2e > gpurun_out/prof/kt_$W.log 2>&1; rc=$?
  echo "kt $W rc=$rc"; grep "^\[bench\]" gpurun_out/prof/kt_$W.log
  [ $rc -ne 0 ] && exit $rc
done
timeout -k 10 500 python -u bench.py > gpurun_out/bench_r.log 2>&1; rc=$?
echo "bench rc=$rc"; grep "^\[bench\]" gpurun_out/bench_r.log
exit $rc
