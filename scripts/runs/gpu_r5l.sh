# round 5: soaks of the round's new paths on the GPU -- random batches with layout
# hints (right, partly wrong, wrong, unpackable) in 16- and 8-byte records, random batch
# queues mixing them with 8-byte queues, and random mOS setups over the consumer
# (8-byte records, the module's default)
set -o pipefail
mkdir -p gpurun_out/r5l
timeout -k 10 330 python3 -u scripts/soak_classify.py 300 21 > gpurun_out/r5l/soak_classify_seed21.log 2>&1; rc=$?
tail -2 gpurun_out/r5l/soak_classify_seed21.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 270 python3 -u scripts/soak_classify.py 240 22 queue > gpurun_out/r5l/soak_queue_seed22.log 2>&1; rc=$?
tail -2 gpurun_out/r5l/soak_queue_seed22.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 330 python3 -u scripts/soak_consumer.py 300 23 gpu > gpurun_out/r5l/soak_consumer_gpu_seed23.log 2>&1; rc=$?
tail -2 gpurun_out/r5l/soak_consumer_gpu_seed23.log
exit $rc
