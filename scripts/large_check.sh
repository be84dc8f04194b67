#!/bin/bash
# Large-N (2^18..2^20) check: parity subset, then kernel split with rows and with the ring.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-l02}
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_state.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "1048576 or 262144 or 524288 or large or retune" > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_$TAG.log
[ $rc -ge 124 ] && exit $rc
scripts/prof_kbench.sh ${TAG}_rows "--sizes 262144,1048576 --formats s8,f32 --iters 10" || exit $?
scripts/prof_kbench.sh ${TAG}_ring "--sizes 262144,1048576 --formats s8,f32 --iters 10 --state" || exit $?
