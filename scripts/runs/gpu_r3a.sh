#!/bin/bash
# round 3: consumer + backend GPU tests, then the driver-style bench line.
# A timeout / crash of the tests ends the script (no further GPU work).
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/r3a
timeout -k 10 420 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
    tests/test_mos_consumer.py tests/test_tpacket_ring.py tests/test_backend_gpu.py > gpurun_out/r3a/pytest.log 2>&1
rc=$?
echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r3a/bench.out 2> gpurun_out/r3a/bench.err
echo "bench rc=$?"
wc -c gpurun_out/r3a/bench.out
