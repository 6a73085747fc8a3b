# BPF JIT wave-group A/B (ab/libmosrx_<v>.so): parity (tests/test_bpf.py) of each build, then alternated IMIX_bpf lines
set -o pipefail
mkdir -p gpurun_out
L=mos-networking-stack_amd/libmosrx.so
cp $L gpurun_out/.lib_orig.so
for v in ${PV:-g2 g4}; do
  cp ab/libmosrx_$v.so $L
  timeout -k 10 300 python -u -m pytest tests/test_bpf.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ab_pytest_$v.log 2>&1; rc=$?
  echo "== parity $v rc=$rc"; tail -1 gpurun_out/ab_pytest_$v.log
  [ $rc -ne 0 ] && { cp gpurun_out/.lib_orig.so $L; exit $rc; }
done
cp gpurun_out/.lib_orig.so $L
V="old ${PV:-g2 g4}" W="IMIX_bpf,IMIX_cls_bpf" bash scripts/gpu_ab.sh
