# round-5 evidence: PMC HBM traffic (separate FETCH_SIZE / WRITE_SIZE passes) and
# rocprofv3 kernel-trace summaries (1 stream) of the bench rows, under gpurun_out/prof5.
# PHASE=pmc or PHASE=kt (one gpurun call each).
set -o pipefail
mkdir -p gpurun_out/prof5
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-.}"
if [ "${PHASE:-pmc}" = pmc ]; then
  for W in ${PMC_W:-M1500 IMIX S64 S64_c8 S64_c8_packed S64_hdr S64_hdr_packed S64_cls_bpf_ring IMIX_cls_bpf_ring M1500_1 IMIX_1 S64_1}; do
    case $W in *_1) K=mosrx_classify_kernel ;; *_cls_bpf_ring) K=mosrx_classify_bpf_queue ;; *) K=mosrx_classify_queue_kernel ;; esac
    N=40; case $W in S64*) N=12 ;; M1500|IMIX|IMIX_cls_bpf_ring) N=16 ;; esac
    case $W in *_1) N=40 ;; esac
    timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof5/pmcf_$W -o pmc --output-format csv -- python3 scripts/pmc_run.py $W $N > gpurun_out/prof5/pmcf_$W.log 2>&1; rc=$?
    echo "pmc fetch $W rc=$rc"; [ $rc -ne 0 ] && exit $rc
    timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/prof5/pmcw_$W -o pmc --output-format csv -- python3 scripts/pmc_run.py $W $N > gpurun_out/prof5/pmcw_$W.log 2>&1; rc=$?
    echo "pmc write $W rc=$rc"; [ $rc -ne 0 ] && exit $rc
    python3 scripts/pmc_parse.py $W gpurun_out/prof5/pmcf_$W gpurun_out/prof5/pmcw_$W $K gpurun_out/prof5/pmc_traffic.json
  done
else
  for W in ${KT_W:-M1500 IMIX S64 S64_c8 S64_c8_packed S64_hdr S64_hdr_packed M1500_1 IMIX_1 S64_1 IMIX_bpf IMIX_cls_bpf IMIX_cls_bpf_ring S64_cls_bpf_ring}; do
    timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof5/kt_$W -o kt --output-format csv -- python3 bench.py --workloads $W --streams 1 --no-cpu --no-e2e > gpurun_out/prof5/kt_$W.log 2>&1; rc=$?
    echo "kt $W rc=$rc"; grep "^\[bench\]" gpurun_out/prof5/kt_$W.log
    [ $rc -ne 0 ] && exit $rc
  done
fi
exit 0
