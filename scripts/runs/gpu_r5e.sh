# round 5: workgroup size of config #2's isolated hinted launch (probe_hint_tiles)
set -o pipefail
mkdir -p gpurun_out/r5e
export TMPDIR=/tmp
for r in 1 2; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r5e/kt_$r -o kt --output-format csv -- \
    scripts/probe_hint_tiles 3000 > gpurun_out/r5e/kt_$r.log 2>&1; rc=$?
  echo "probe $r rc=$rc"; cat gpurun_out/r5e/kt_$r.log | grep -v rocprofv3 | head -5; [ $rc -ne 0 ] && exit $rc
  grep k_hint $(find gpurun_out/r5e/kt_$r -name "*kernel_stats.csv") | cut -c1-40,60-140
done
exit 0
