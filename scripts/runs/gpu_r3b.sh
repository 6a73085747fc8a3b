#!/bin/bash
# round 3: flow-hash / consumer / backend GPU tests, then the rocprof evidence
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/r3b
timeout -k 10 420 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
    tests/test_mos_consumer.py tests/test_backend_gpu.py > gpurun_out/r3b/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/r3b/pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
bash scripts/runs/gpu_r3_profiles.sh
