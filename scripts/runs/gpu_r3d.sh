#!/bin/bash
# dispatch-stamped kernel timing: its GPU test, then the bench rows (no CPU / e2e legs)
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/r3d
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
    tests/test_parity_gpu.py -k "dispatch_stamped or batch_queue" > gpurun_out/r3d/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r3d/pytest.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py --no-cpu --no-e2e --detail gpurun_out/r3d/bench_detail.json > gpurun_out/r3d/bench.out 2> gpurun_out/r3d/bench.err
rc=$?; echo "bench rc=$rc"; grep "^\[bench\]" gpurun_out/r3d/bench.err
exit $rc
