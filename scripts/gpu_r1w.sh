# SQ counters of the S13 classify kernel (two passes of 8 SQ counters each)
set -o pipefail
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA"
P2="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_BUSY_CU_CYCLES"
for W in M1500 IMIX S64; do
  timeout -s KILL 90 rocprofv3 --pmc $P1 -d gpurun_out/prof/sq1_$W -o pmc --output-format csv -- python3 scripts/pmc_run.py $W 20 > gpurun_out/prof/sq1_$W.log 2>&1; rc=$?
  echo "sq1 $W rc=$rc"; [ $rc -ne 0 ] && exit $rc
  timeout -s KILL 90 rocprofv3 --pmc $P2 -d gpurun_out/prof/sq2_$W -o pmc --output-format csv -- python3 scripts/pmc_run.py $W 20 > gpurun_out/prof/sq2_$W.log 2>&1; rc=$?
  echo "sq2 $W rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0
