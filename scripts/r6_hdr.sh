# FETCH_SIZE / WRITE_SIZE of byte-known header-window kernels and of the IMIX_bpf row
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/hdr
./scripts/hdrprobe 1 > gpurun_out/hdr/sectors.txt || exit 1
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 90 rocprofv3 --pmc $c --output-format csv -d gpurun_out/hdr/$c -o p -- ./scripts/hdrprobe 24 > gpurun_out/hdr/probe_$c.log 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d gpurun_out/hdr/bpf_$c -o p -- python3 scripts/pmc_run.py IMIX_bpf 24 > gpurun_out/hdr/bpf_$c.log 2>&1 || exit 1
done
cat gpurun_out/hdr/sectors.txt
find gpurun_out/hdr -name "*counter_collection.csv" | head
