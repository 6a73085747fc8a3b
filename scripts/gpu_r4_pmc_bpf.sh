# round 4: HBM traffic of the standalone BPF launch and the fused single launch (IMIX 256K)
set -o pipefail
mkdir -p gpurun_out/prof4b
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-.}"
rm -f gpurun_out/prof4b/pmc_traffic.json
for W in IMIX_bpf IMIX_cls_bpf; do
  case $W in IMIX_bpf) K=mosrx_bpf_jit ;; *) K=mosrx_classify_bpf_stream ;; esac
  timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof4b/pmcf_$W -o pmc --output-format csv -- python3 scripts/pmc_run.py $W 40 > gpurun_out/prof4b/pmcf_$W.log 2>&1; rc=$?
  echo "pmc fetch $W rc=$rc"; [ $rc -ne 0 ] && exit $rc
  timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/prof4b/pmcw_$W -o pmc --output-format csv -- python3 scripts/pmc_run.py $W 40 > gpurun_out/prof4b/pmcw_$W.log 2>&1; rc=$?
  echo "pmc write $W rc=$rc"; [ $rc -ne 0 ] && exit $rc
  python3 scripts/pmc_parse.py $W gpurun_out/prof4b/pmcf_$W gpurun_out/prof4b/pmcw_$W $K gpurun_out/prof4b/pmc_traffic.json
  grep "algo bytes" gpurun_out/prof4b/pmcf_$W.log
done
