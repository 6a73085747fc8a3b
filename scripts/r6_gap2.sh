# VERDICT r5 next #1, second pass: what makes a launch over frames just copied in slower
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/gap2
run() {  # name, env, key, phase
  timeout -k 10 150 env $2 rocprofv3 --kernel-trace --stats -d gpurun_out/gap2/kt_$1 -o kt -- \
    python3 -u scripts/diag_backend_gap.py $3 $4 >> gpurun_out/gap2/diag.log 2>gpurun_out/gap2/err_$1.log || exit $?
}
run c8_b2b X=1 M1500c8 res_b2b
run c8_gap2 X=1 M1500c8 res_gap2
run c8_fresh X=1 M1500c8 res_fresh
run c8_fresh_other X=1 M1500c8 res_fresh_other
run c8_fresh_sleep10 X=1 M1500c8 res_fresh_sleep10
run c8_fresh_nosdma HSA_ENABLE_SDMA=0 M1500c8 res_fresh
run c8_be_g1 X=1 M1500c8 be_g1
run c8_be_g1_nosdma HSA_ENABLE_SDMA=0 M1500c8 be_g1
run s64_fresh_other X=1 S64 res_fresh_other
run s64_be_auto_nosdma HSA_ENABLE_SDMA=0 S64 be_auto
