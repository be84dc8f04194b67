#!/bin/bash
# Channel-mean cost (FftProcessor.kt:143-157, one lane per frame summing its channel's
# bins in order): 64 K s8 B = 500 + EMA / peak step with squelch channels of 0, 200,
# 1000, 8000 and 32000 bins.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out/chan_${1:-a}.txt; : > $OUT
for k in 0 200 1000 8000 32000; do
  echo "== channel bins $k" | tee -a $OUT
  timeout -k 10 120 python -u scripts/kbench.py --sizes 65536 --formats s8 --samples 32768000 --state --channel-bins $k \
    2>&1 | grep -v amdgpu.ids | tee -a $OUT
  rc=${PIPESTATUS[0]}; [ $rc -ne 0 ] && exit $rc
done
for k in 0 100000 1048576; do  # 1 M, 16 frames: up to the full band
  echo "== 1M channel bins $k" | tee -a $OUT
  timeout -k 10 120 python -u scripts/kbench.py --sizes 1048576 --formats s8 --samples 16777216 --state --channel-bins $k \
    --iters 5 2>&1 | grep -v amdgpu.ids | tee -a $OUT
  rc=${PIPESTATUS[0]}; [ $rc -ne 0 ] && exit $rc
done
exit 0
