# SQ counters (two 8-counter passes) for the ring and single-launch kernels; CSVs under gpurun_out/sq
set -o pipefail
mkdir -p gpurun_out/sq
export TMPDIR=/tmp
for W in ${SQ_W:-IMIX M1500 IMIX_1}; do
  N=12; case $W in *_1) N=30 ;; esac
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY -d gpurun_out/sq/p1_$W -o pmc --output-format csv -- python3 scripts/pmc_run.py $W $N > gpurun_out/sq/p1_$W.log 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_SCA SQ_BUSY_CU_CYCLES -d gpurun_out/sq/p2_$W -o pmc --output-format csv -- python3 scripts/pmc_run.py $W $N > gpurun_out/sq/p2_$W.log 2>&1 || exit 1
  echo "sq $W ok"
done
