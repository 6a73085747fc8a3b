cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pull
for p in res_b2b res_fresh res_fresh_pull res_fresh_other res_fresh_other_pull; do
  timeout -k 10 150 rocprofv3 --kernel-trace --stats -d gpurun_out/pull/kt_$p -o kt -- \
    python3 -u scripts/diag_backend_gap.py M1500c8 $p >> gpurun_out/pull/diag.log 2>gpurun_out/pull/err_$p.log || exit 1
done
for p in res_fresh res_fresh_pull; do
  timeout -k 10 150 python3 -u scripts/diag_backend_gap.py S64 $p >> gpurun_out/pull/diag_nokt.log 2>&1 || exit 1
done
cat gpurun_out/pull/diag.log gpurun_out/pull/diag_nokt.log
