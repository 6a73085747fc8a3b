# round 6: soaks of the backend with direct (copy-free) groups on by default
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6soak
timeout -k 10 200 python3 -u scripts/soak_backend.py 150 61 > gpurun_out/r6soak/backend.log 2>&1 || { tail -30 gpurun_out/r6soak/backend.log; exit 1; }
tail -3 gpurun_out/r6soak/backend.log
timeout -k 10 150 python3 -u scripts/soak_threads.py 90 > gpurun_out/r6soak/threads.log 2>&1 || { tail -30 gpurun_out/r6soak/threads.log; exit 1; }
tail -3 gpurun_out/r6soak/threads.log
