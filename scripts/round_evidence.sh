#!/bin/bash
# Round evidence in one GPU call: profile_round (bench + rocprof stats + 2 PMC passes)
# then the kernel micro-bench over all sizes/formats.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-r01}
bash scripts/profile_round.sh $TAG || exit $?
timeout -k 10 300 python scripts/kbench.py --sizes 1024,4096,8192,16384,65536,262144,1048576 --formats s8,f32 \
    > gpurun_out/kbench_$TAG.txt 2>&1
rc=$?; echo "kbench rc=$rc"; cat gpurun_out/kbench_$TAG.txt | tail -20
exit $rc
