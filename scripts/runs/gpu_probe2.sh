# probe_classify on ring-sized single batches (the queue kernel's work in one launch) and batch-sized ones
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/probe2.log
for args in ${PROBE_ARGS:-"1 8388608 x 3" "1 32768 x 6" "2 524288 x 3 q" "3 2097152 x 3 q" "2 65536 x 13" "3 262144 x 13"}; do
  echo "== probe $args" >> gpurun_out/probe2.log
  timeout -k 10 150 ./scripts/probe_classify $args >> gpurun_out/probe2.log 2>&1; rc=$?
  [ $rc -ne 0 ] && { cat gpurun_out/probe2.log; exit $rc; }
done
cat gpurun_out/probe2.log
