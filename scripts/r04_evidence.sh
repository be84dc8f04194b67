#!/bin/bash
# Round-4 evidence of the product tree in one GPU call: final_evidence.sh (GPU suite, smoke,
# bench + rocprof + PMC, kbench sweep, SQ breakdown, config-4 shard) and the config-3 seed
# sweep (|librfa - float64| and |librfa - pffft| every-bin statistics on four captures).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-r04g}
bash scripts/final_evidence.sh $TAG || exit $?
timeout -k 10 300 python -u scripts/config3_seed_sweep.py 3,5,7,11 > gpurun_out/seed_sweep_$TAG.txt 2>&1
rc=$?; echo "sweep rc=$rc"; grep -v amdgpu.ids gpurun_out/seed_sweep_$TAG.txt
exit $rc
