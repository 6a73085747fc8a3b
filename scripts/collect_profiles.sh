# Copy the judged evidence of a scripts/runs/gpu_r2_final.sh run from gpurun_out/ (scratch,
# merged back by gpurun) into profiles/ (tracked).  Run here, after the GPU call.
#   kernel-trace summaries : profiles/<round>_kt_<W>_kernel_stats.csv + the bench line of that run
#   PMC passes             : profiles/<round>_pmc_{fetch,write}_<W>.csv + profiles/pmc_traffic.json
#   default bench          : profiles/<round>_bench.log
set -e
cd "$(dirname "$0")/.."
P=${1:-r02}
for d in gpurun_out/prof/kt_*/; do
  W=$(basename "$d"); W=${W#kt_}
  cp "$d/kt_kernel_stats.csv" "profiles/${P}_kt_${W}_kernel_stats.csv"
  cp "gpurun_out/prof/kt_${W}.log" "profiles/${P}_kt_${W}_bench.log"
done
for d in gpurun_out/prof/pmcf_*/; do
  W=$(basename "$d"); W=${W#pmcf_}
  cp "$d/pmc_counter_collection.csv" "profiles/${P}_pmc_fetch_${W}.csv"
  cp "gpurun_out/prof/pmcw_${W}/pmc_counter_collection.csv" "profiles/${P}_pmc_write_${W}.csv"
done
[ -f gpurun_out/pmc_traffic.json ] && cp gpurun_out/pmc_traffic.json profiles/pmc_traffic.json
[ -f gpurun_out/bench_r.log ] && cp gpurun_out/bench_r.log "profiles/${P}_bench.log"
ls -la profiles | head -60
