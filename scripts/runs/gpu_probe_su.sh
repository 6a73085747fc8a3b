# streamers per tile x loads in flight (scripts/probe_timeline mode 5): IMIX and 1500 B, single batch and ring size
set -o pipefail
mkdir -p gpurun_out/probe
for a in "3 262144 13" "3 2097152 2" "2 65536 13" "2 524288 2"; do
  set -- $a
  timeout -k 10 200 scripts/probe_timeline $1 $2 $3 5 > gpurun_out/probe/su_$1_$2.log 2>&1; rc=$?
  echo "== kind $1 n $2 rc=$rc"; grep -E "median" gpurun_out/probe/su_$1_$2.log; [ $rc -ne 0 ] && exit $rc
done
exit 0
