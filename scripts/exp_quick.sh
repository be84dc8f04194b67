#!/bin/bash
# parity tests then kernel timings (args passed to kbench)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -x -p no:cacheprovider > gpurun_out/pytest_quick.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_quick.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python scripts/kbench.py "$@"
