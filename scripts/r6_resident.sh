# round 6: resident-kernel probe; the kernel leaves by itself within 2 s
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6res
timeout -k 10 60 ./scripts/resident_probe > gpurun_out/r6res/probe.txt 2>&1; rc=$?
cat gpurun_out/r6res/probe.txt
exit $rc
