# round-1 closing evidence: full GPU parity, smoke, PMC HBM traffic, kernel-trace
# summaries (1 stream) for every bench workload, then the default bench
set -o pipefail
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout=120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_final.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_final.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_final.log 2>&1; rc=$?
echo "smoke rc=$rc"; tail -1 gpurun_out/smoke_final.log
[ $rc -ne 0 ] && exit $rc
bash scripts/gpu_r1r.sh
