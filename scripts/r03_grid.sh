#!/bin/bash
# Is the 64 K kernel bound by the synchronised HBM bursts of all CUs?  Same kernel on
# 256 / 192 / 128 / 64 workgroups (A/B build, RFA_WIDE_GRID): per-item phase stamps.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${1:-a}
for g in 256 128 64 192; do
  rm -f gpurun_out/stamps_grid${g}_$TAG.bin
  RFA_LIB=alt/librfa_ab.so RFA_WIDE_GRID=$g RFA_STAMPS_FILE=gpurun_out/stamps_grid${g}_$TAG.bin timeout -k 10 120 \
    python -u scripts/kbench.py --sizes 65536 --formats s8 --samples 32768000 --state --iters 8 2>&1 | grep -v amdgpu.ids
  rc=${PIPESTATUS[0]}; echo "grid $g rc=$rc"; [ $rc -ne 0 ] && exit $rc
  python scripts/stamps.py gpurun_out/stamps_grid${g}_$TAG.bin > gpurun_out/stamps_grid${g}_$TAG.txt
done
