#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -x -p no:cacheprovider > gpurun_out/pytest_32k.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_32k.log; [ $rc -ne 0 ] && exit $rc
for L in 15 14; do
  echo "== RFA_WIDE_LOGM=$L"
  RFA_WIDE_LOGM=$L timeout -k 10 200 python scripts/kbench.py --sizes 32768,65536,131072 --formats s8,s16,f32 || exit $?
done
RFA_WIDE_LOGM=14 timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -m gpu -q -x -p no:cacheprovider -k "32768 or 65536 or 131072" > gpurun_out/pytest_32k_14.log 2>&1
echo "logm14 parity rc=$?"; tail -2 gpurun_out/pytest_32k_14.log
timeout -k 10 300 python scripts/host_rate.py || exit $?
