# round 5: controlled A/B of the layout hint on the isolated 32K x 64 B launch
set -o pipefail
mkdir -p gpurun_out/r5d
export TMPDIR=/tmp
for r in 1 2 3; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r5d/kt_$r -o kt --output-format csv -- \
    python3 scripts/probe_hint.py 4000 > gpurun_out/r5d/kt_$r.log 2>&1; rc=$?
  echo "probe $r rc=$rc"; [ $rc -ne 0 ] && exit $rc
  grep classify $(find gpurun_out/r5d/kt_$r -name "*kernel_stats.csv") | cut -c1-60,190-260
done
exit 0
