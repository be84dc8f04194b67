#!/bin/bash
# State-update overlap A/B in ONE GPU call: the state GPU tests (incl. the
# RFA_STATE_OVERLAP parity cases), then config-3 step time with the peak / EMA
# update serial vs overlapped on a second stream, and the 1 M small-batch state
# kernel (state4_kernel vs the scalar one).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${1:-ov}
timeout -k 10 400 python -u -m pytest tests/test_gpu_state.py -x -q --timeout 120 --timeout-method thread \
    -p no:cacheprovider > gpurun_out/pytest_state_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_state_$TAG.log; [ $rc -ne 0 ] && exit $rc
bash scripts/ab_kbench.sh gpurun_out/state_overlap_ab_$TAG.txt \
    "--sizes 65536 --formats s8 --samples 32768000 --state --iters 200 --no-prof" \
    "serial|" "ov2|RFA_STATE_OVERLAP=2" "ov2lazy|RFA_STATE_OVERLAP=2 RFA_STATE_JOIN=lazy" \
    "ov3lazy|RFA_STATE_OVERLAP=3 RFA_STATE_JOIN=lazy" "ov4lazy|RFA_STATE_OVERLAP=4 RFA_STATE_JOIN=lazy" \
    "ov2lazy_nf|RFA_STATE_OVERLAP=2 RFA_STATE_JOIN=lazy RFA_STATE_FUSED=0" "serial2|" || exit $?
bash scripts/ab_kbench.sh gpurun_out/state4_ab_$TAG.txt \
    "--sizes 262144,1048576 --formats s8 --samples 16777216 --state --iters 50" \
    "state4|" "scalar|RFA_STATE_SCALAR=1" || exit $?
