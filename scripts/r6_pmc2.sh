# round 6: memory-side read latency and DRAM credit stalls of the classify kernel per gap phase
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
R=gpurun_out/r6pmc2
mkdir -p $R
C="TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_EA0_RDREQ_DRAM_sum GRBM_GUI_ACTIVE"
for ph in res_b2b res_gap2 res_fresh res_fresh_other be_g1; do
  timeout -s KILL 150 rocprofv3 --pmc $C --output-format csv -d $R/$ph -o p -- python3 scripts/diag_backend_gap.py M1500c8 $ph > $R/$ph.log 2>&1 || { tail -5 $R/$ph.log; exit 1; }
  grep -v "^\[\|^W2026\|^E2026" $R/$ph.log | tail -1
done
python3 scripts/r6_pmc_lat.py $R > $R/summary.json && cat $R/summary.json
find $R -name "*.csv" -size +20M -delete
