# SMALL tile frames-per-lane A/B: parity of each build (no fused BPF: hipRTC builds
# the default tile), then alternated S64 ring / single-launch bench lines
set -o pipefail
mkdir -p gpurun_out
L=mos-networking-stack_amd/libmosrx.so
cp $L gpurun_out/.lib_orig.so
timeout -k 10 200 python -u -c "
import bench, json
for k, t, g, n in (('S64', 2, 32, 8 << 20), ('M1500', 2, 1, 500000)):
    print(json.dumps(bench.measure_backend_threads(k, t, g, n, 0)), flush=True)
" > gpurun_out/mt_check.log 2>&1; rc=$?
tail -3 gpurun_out/mt_check.log; [ $rc -ne 0 ] && exit $rc
for v in new v1024; do
  cp ab/libmosrx_$v.so $L
  timeout -k 10 300 python -u -m pytest tests/test_parity_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "not bpf" > gpurun_out/ab_pytest_$v.log 2>&1; rc=$?
  echo "== parity $v rc=$rc"; tail -2 gpurun_out/ab_pytest_$v.log
  [ $rc -ne 0 ] && { cp gpurun_out/.lib_orig.so $L; exit $rc; }
done
cp gpurun_out/.lib_orig.so $L
V="old new v1024" W="S64,S64_1,S64_hdr" bash scripts/gpu_ab.sh
