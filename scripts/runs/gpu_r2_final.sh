# round-2 final evidence on the current tree.  PART=1: GPU suite + smoke, the
# driver-style and default bench; PART=2: PMC traffic passes and kernel-trace
# summaries (scripts/runs/gpu_r2_profiles.sh), then the two-rank rehearsal
set -o pipefail
mkdir -p gpurun_out
if [ "${PART:-1}" = 1 ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
  tail -2 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
  timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?
  tail -1 gpurun_out/smoke.log; [ $rc -ne 0 ] && exit $rc
  bash scripts/gpu_bench.sh || exit $?
else
  bash scripts/runs/gpu_r2_profiles.sh > gpurun_out/profiles_run.log 2>&1; rc=$?
  tail -30 gpurun_out/profiles_run.log; [ $rc -ne 0 ] && exit $rc
  bash scripts/runs/gpu_dist_rehearsal.sh
fi
