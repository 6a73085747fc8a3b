# why bench's back-to-back kernel time differs from the probe's
set -o pipefail
mkdir -p gpurun_out
for S in 100 1000; do
timeout -k 10 200 python bench.py --workloads M1500,IMIX --steps $S --streams 1 --no-cpu --no-e2e > gpurun_out/bench_n$S.log 2>&1; rc=$?
echo "bench $S rc=$rc"; grep "^\[bench\]" gpurun_out/bench_n$S.log; [ $rc -ne 0 ] && exit $rc
done
timeout -k 10 100 ./scripts/probe_classify 2 65536 > gpurun_out/probe_n.log 2>&1; rc=$?
head -4 gpurun_out/probe_n.log
exit $rc
