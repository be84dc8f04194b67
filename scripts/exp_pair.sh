#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_pair.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_pair.log; [ $rc -ne 0 ] && exit $rc
for p in 1 0; do echo "== RFA_PAIR=$p"; RFA_PAIR=$p timeout -k 10 200 python scripts/kbench.py --sizes 65536 --formats s8,u8 --iters 20 2>&1 | grep -v amdgpu.ids || exit 1; done
echo "== state bench"; timeout -k 10 200 python scripts/kbench.py --sizes 65536 --formats s8 --state 2>&1 | grep -v amdgpu.ids
rm -f gpurun_out/stamps_p.bin
RFA_STAMPS_FILE=gpurun_out/stamps_p.bin timeout -k 10 120 python scripts/kbench.py --sizes 65536 --formats s8 --iters 3 --no-prof 2>&1 | grep -v amdgpu.ids || exit 1
python3 scripts/stamps.py gpurun_out/stamps_p.bin; rm -f gpurun_out/stamps_p.bin
