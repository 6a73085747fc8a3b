# which SQ counters exist on gfx950 (listing only)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > gpurun_out/counters.txt 2>&1; rc=$?
grep -o "SQ_[A-Z_0-9]*\|TA_[A-Z_0-9]*\|TCP_[A-Z_0-9]*\|TCC_[A-Z_0-9]*" gpurun_out/counters.txt | sort -u > gpurun_out/counter_names.txt
wc -l gpurun_out/counter_names.txt
exit $rc
