cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/latprof
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --stats -d gpurun_out/latprof/s64g1 -o lp -- \
  python3 -u scripts/r6_latprof.py S64 1 60 > gpurun_out/latprof/s64g1.log 2>&1 || { tail -20 gpurun_out/latprof/s64g1.log; exit 1; }
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --stats -d gpurun_out/latprof/m1500g1 -o lp -- \
  python3 -u scripts/r6_latprof.py M1500 1 8.7 > gpurun_out/latprof/m1500g1.log 2>&1 || { tail -20 gpurun_out/latprof/m1500g1.log; exit 1; }
grep "offered" gpurun_out/latprof/*.log | cut -c1-400
