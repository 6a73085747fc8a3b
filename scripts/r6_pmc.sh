# round 6: PMC passes (FETCH_SIZE, WRITE_SIZE, separate runs) over the backend-gap phases
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
R=gpurun_out/r6pmc
mkdir -p $R
for spec in "M1500c8 res_b2b" "M1500c8 res_fresh" "M1500c8 res_fresh_other" "M1500c8 be_g1" "S64 res_b2b" "S64 be_auto"; do
  set -- $spec
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 150 rocprofv3 --pmc $c --output-format csv -d $R/${1}_${2}_$c -o p -- python3 scripts/diag_backend_gap.py $1 $2 > $R/${1}_${2}_$c.log 2>&1 || { tail -5 $R/${1}_${2}_$c.log; exit 1; }
    grep -v "^\[\|^W2026\|^E2026" $R/${1}_${2}_$c.log | tail -2
  done
done
python3 scripts/r6_pmc_gap.py $R > $R/summary.json && cat $R/summary.json
find $R -name "*.csv" -size +20M -delete
