# SMALL tile size A/B (ab/libmosrx_<v>.so for v in $PV): parity of each build
# (no fused BPF: hipRTC builds the default tile), then alternated S64 ring /
# single-launch bench lines against ab/libmosrx_old.so
set -o pipefail
mkdir -p gpurun_out
L=mos-networking-stack_amd/libmosrx.so
cp $L gpurun_out/.lib_orig.so
for v in ${PV:-new v1024}; do
  cp ab/libmosrx_$v.so $L
  timeout -k 10 300 python -u -m pytest tests/test_parity_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "not bpf" > gpurun_out/ab_pytest_$v.log 2>&1; rc=$?
  echo "== parity $v rc=$rc"; tail -2 gpurun_out/ab_pytest_$v.log
  [ $rc -ne 0 ] && { cp gpurun_out/.lib_orig.so $L; exit $rc; }
done
cp gpurun_out/.lib_orig.so $L
V="old ${PV:-new v1024}" W="S64,S64_1,S64_hdr" bash scripts/gpu_ab.sh
