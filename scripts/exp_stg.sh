#!/bin/bash
# LDS-DMA staged input (STG) vs register loads: parity tests first, then kernel bench A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_stg.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_stg.log; [ $rc -ne 0 ] && exit $rc
for st in 1 0; do echo "== RFA_STAGE=$st"; RFA_STAGE=$st timeout -k 10 200 python scripts/kbench.py --sizes 8192,16384,32768,65536 --formats s8,s16 --iters 20 2>&1 | grep -v amdgpu.ids || exit 1; done
echo "== state bench"; timeout -k 10 200 python scripts/kbench.py --sizes 65536 --formats s8 --state 2>&1 | grep -v amdgpu.ids
