# round 5, first GPU pass: the layout-hint tests + the parity suite, then
# rocprof kernel traces of the 64 B single launch (config #2 literally) and ring
set -o pipefail
mkdir -p gpurun_out/r5a
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_layout_hint.py tests/test_parity_gpu.py tests/test_mos_consumer.py -m gpu -x -q \
  --timeout 120 --timeout-method thread > gpurun_out/r5a/pytest.log 2>&1; rc=$?
tail -3 gpurun_out/r5a/pytest.log; [ $rc -ne 0 ] && exit $rc
for W in S64_1 S64 S64_hdr; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r5a/kt_$W -o kt --output-format csv -- \
    python3 bench.py --workloads $W --streams 1 --no-cpu --no-e2e > gpurun_out/r5a/kt_$W.log 2>&1; rc=$?
  echo "kt $W rc=$rc"; grep "^\[bench\]" gpurun_out/r5a/kt_$W.log
  [ $rc -ne 0 ] && exit $rc
done
find gpurun_out/r5a -name "*kernel_stats.csv" | while read f; do echo "== $f"; head -4 "$f"; done
exit 0
