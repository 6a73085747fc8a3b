# round-2 final evidence on the current tree: driver-style + default bench, then
# PMC traffic passes and kernel-trace summaries (scripts/gpu_r2_profiles.sh)
set -o pipefail
mkdir -p gpurun_out
bash scripts/gpu_bench.sh || exit $?
bash scripts/gpu_r2_profiles.sh > gpurun_out/profiles_run.log 2>&1; rc=$?
tail -30 gpurun_out/profiles_run.log
exit $rc
