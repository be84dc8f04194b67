#!/bin/bash
# GPU suite, then the tile-order ring epilogue (in-tree) vs the residue-major dword
# epilogue (alt/librfa_diag12.so, built before the change) inside one call.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${1:-b}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/pytest_gpu_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -6 gpurun_out/pytest_gpu_$TAG.log; [ $rc -ne 0 ] && exit $rc
for N in 65536 32768 131072; do
  bash scripts/ab_kbench.sh gpurun_out/tile_ab_${TAG}_$N.txt "--sizes $N --formats s8 --samples 32768000 --state" \
    "old|RFA_LIB=alt/librfa_diag12.so" "tile|" "old2|RFA_LIB=alt/librfa_diag12.so" "tile2|" || exit $?
done
