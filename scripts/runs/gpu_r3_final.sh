#!/bin/bash
# round 3 final evidence: the whole -m gpu suite, smoke(), the driver's bench
# command (gpu_r3_full.sh), then PMC traffic + kernel traces of the main rows
# (gpu_r3_profiles.sh).  Any failure ends the script.
cd "${GRAFT_REPO_ROOT:-.}"
bash scripts/runs/gpu_r3_full.sh || exit $?
KT_W="${KT_W:-M1500 IMIX S64 M1500_1 IMIX_1 S64_1}" bash scripts/runs/gpu_r3_profiles.sh
