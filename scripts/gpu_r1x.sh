# LDS pressure of the classify kernels (one pass of 8 SQ counters)
set -o pipefail
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
P3="SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_CMD_FIFO_FULL SQ_LDS_DATA_FIFO_FULL SQ_LDS_ADDR_CONFLICT SQ_INSTS_LDS"
for W in M1500 IMIX S64; do
  timeout -s KILL 90 rocprofv3 --pmc $P3 -d gpurun_out/prof/sq3_$W -o pmc --output-format csv -- python3 scripts/pmc_run.py $W 20 > gpurun_out/prof/sq3_$W.log 2>&1; rc=$?
  echo "sq3 $W rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0
