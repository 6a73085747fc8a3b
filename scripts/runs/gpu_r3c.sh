#!/bin/bash
# round 3: the consumer's GPU leg (conversation + golden-fixture scenarios).
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/r3c
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
    tests/test_mos_consumer.py > gpurun_out/r3c/pytest.log 2>&1
rc=$?
echo "pytest rc=$rc"
tail -3 gpurun_out/r3c/pytest.log
exit $rc
