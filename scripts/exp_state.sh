#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -x -p no:cacheprovider > gpurun_out/pytest_state.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_state.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python scripts/kbench.py --sizes 8192,16384,32768,65536,131072 --formats s8,f32 --state || exit $?
timeout -k 10 200 python scripts/kbench.py --sizes 65536 --formats s8,u8,s16,f32,f32p || exit $?
