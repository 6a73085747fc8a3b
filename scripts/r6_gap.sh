# the backend's device-time gap, phase by phase under rocprofv3 kernel traces
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/gap
for k in M1500 S64; do
  for p in res_b2b res_gap2 res_gap30 res_fresh be_g1; do
    [ $k = S64 ] && [ $p = be_g1 ] && p=be_auto
    timeout -k 10 150 rocprofv3 --kernel-trace --stats -d gpurun_out/gap/kt_${k}_$p -o kt -- \
      python3 -u scripts/diag_backend_gap.py $k $p >> gpurun_out/gap/diag.log 2>gpurun_out/gap/err_${k}_$p.log || exit $?
  done
done
