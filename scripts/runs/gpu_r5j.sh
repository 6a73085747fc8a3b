# round 5: the empty-kernel stamp floor of the one-launch rows, and the full-verdict
# compact row on the backend's packed layout
set -o pipefail
mkdir -p gpurun_out/r5j
timeout -k 10 200 python -u -m pytest tests/test_parity_gpu.py -k "stamped or hint" -m gpu -x -q \
  --timeout 120 --timeout-method thread > gpurun_out/r5j/pytest.log 2>&1; rc=$?
tail -2 gpurun_out/r5j/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --workloads S64_c8,S64_c8_packed,S64_1,M1500_1,IMIX_1,M1500_fh --no-cpu --no-e2e \
  --detail gpurun_out/r5j/rows.json > gpurun_out/r5j/rows.out 2> gpurun_out/r5j/rows.err; rc=$?
grep "^\[bench\]" gpurun_out/r5j/rows.err; tail -c 1500 gpurun_out/r5j/rows.out
exit $rc
