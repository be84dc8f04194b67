#!/bin/bash
# Column-order ring state update A/B in ONE GPU call: state GPU tests (incl. the
# tiled kernel's parity cases), then large-N step time with state_tile_kernel vs
# the storage-order kernels (RFA_STATE_TILE=0).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${1:-tile}
timeout -k 10 400 python -u -m pytest tests/test_gpu_state.py -x -q --timeout 120 --timeout-method thread \
    -p no:cacheprovider > gpurun_out/pytest_state_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_state_$TAG.log; [ $rc -ne 0 ] && exit $rc
bash scripts/ab_kbench.sh gpurun_out/state_tile_ab_$TAG.txt \
    "--sizes 262144,524288,1048576 --formats s8 --samples 16777216 --state --iters 50" \
    "tile|" "storage|RFA_STATE_TILE=0" "tile2|" || exit $?
