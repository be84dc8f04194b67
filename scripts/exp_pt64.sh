#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_pt64.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_pt64.log; [ $rc -ne 0 ] && exit $rc
for d in 0 256 0 256; do echo "== DIAG $d"; RFA_DIAG=$d timeout -k 10 120 python scripts/kbench.py --sizes 16384,65536 --formats s8 --iters 20 --samples 32768000 2>&1 | grep -v amdgpu.ids || exit 1; done
