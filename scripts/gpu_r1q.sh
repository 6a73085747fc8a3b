# streams in flight per workload
set -o pipefail
mkdir -p gpurun_out
for S in 1 2 3 4; do
timeout -k 10 200 python -u bench.py --workloads M1500,S64,IMIX --streams $S --no-cpu --no-e2e > gpurun_out/bench_s$S.log 2>&1; rc=$?
echo "streams $S rc=$rc"; grep "^\[bench\]" gpurun_out/bench_s$S.log; [ $rc -ne 0 ] && exit $rc
done
exit 0
