#!/bin/bash
# PT=32 vs PT=64 wide kernel: parity (default PT) then kernel timings for both.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -x -p no:cacheprovider > gpurun_out/pytest_pt.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_pt.log; [ $rc -ge 124 ] && exit $rc
for pt in 32 64; do
  RFA_PT=$pt timeout -k 10 200 python scripts/kbench.py --sizes 8192,16384,32768,65536,131072 --formats s8,s16,f32 > gpurun_out/kb_pt$pt.log 2>&1
  rc=$?; echo "PT=$pt rc=$rc"; cat gpurun_out/kb_pt$pt.log; [ $rc -ne 0 ] && exit $rc
done
RFA_PT=64 timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -m gpu -q -x -p no:cacheprovider > gpurun_out/pytest_pt64.log 2>&1
echo "pt64 pytest rc=$?"; tail -3 gpurun_out/pytest_pt64.log
