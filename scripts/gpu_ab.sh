# A/B of library builds ab/libmosrx_<v>.so for v in $V (default: old new), alternated, 1-stream bench lines
set -o pipefail
mkdir -p gpurun_out
L=mos-networking-stack_amd/libmosrx.so
cp $L gpurun_out/.lib_orig.so
for r in 1 2; do
  for v in ${V:-old new}; do
    cp ab/libmosrx_$v.so $L
    timeout -k 10 200 python -u bench.py --workloads ${W:-M1500,IMIX,S64_queue} --streams 1 --no-cpu --no-e2e > gpurun_out/ab_$v.log 2>&1; rc=$?
    echo "== $v run $r"; grep "^\[bench\]" gpurun_out/ab_$v.log
    [ $rc -ne 0 ] && { cp gpurun_out/.lib_orig.so $L; exit $rc; }
  done
done
cp gpurun_out/.lib_orig.so $L
