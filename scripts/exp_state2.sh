#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -x -p no:cacheprovider > gpurun_out/pytest_s2.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_s2.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python scripts/kbench.py --sizes 16384,65536 --formats s8 --state || exit $?
timeout -k 10 200 python scripts/kbench.py --sizes 16384,65536 --formats s8 --state --no-prof || exit $?
timeout -k 10 200 python scripts/kbench.py --sizes 16384,65536 --formats s8 --no-prof || exit $?
