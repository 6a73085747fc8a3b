# TX rewrite variants: parity (tests/test_tx_csum.py) of each build, then alternated M1500_tx bench lines
set -o pipefail
mkdir -p gpurun_out
L=mos-networking-stack_amd/libmosrx.so
cp $L gpurun_out/.lib_orig.so
for v in b16 txc b16c; do
  cp ab/libmosrx_$v.so $L
  timeout -k 10 300 python -u -m pytest tests/test_tx_csum.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ab_pytest_$v.log 2>&1; rc=$?
  echo "== parity $v rc=$rc"; tail -1 gpurun_out/ab_pytest_$v.log
  [ $rc -ne 0 ] && { cp gpurun_out/.lib_orig.so $L; exit $rc; }
done
cp gpurun_out/.lib_orig.so $L
V="old b16 txc b16c" W="M1500_tx,M1500_1" bash scripts/gpu_ab.sh
