# rocprofv3 kernel-trace summary of a short bench run (one workload per pass).
set -o pipefail
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
W=${1:-M1500}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/kt_$W -o kt --output-format csv -- python3 bench.py --steps 50 --warmup 5 --workloads $W --no-cpu --no-e2e > gpurun_out/prof/bench_$W.log 2>&1
rc=$?; echo "rocprof kt rc=$rc"
find gpurun_out/prof/kt_$W -name "*stats*" | head
exit $rc
