#!/bin/bash
# Phase stamps (DIAG 32 build) for s8 kernels: exp_stamps.sh "N1 N2 ..." [samples]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
SIZES=${1:-"16384 65536"}; SAMPLES=${2:-16777216}
for n in $SIZES; do
  rm -f gpurun_out/stamps_$n.bin
  RFA_STAMPS_FILE=gpurun_out/stamps_$n.bin timeout -k 10 120 python scripts/kbench.py --sizes $n --formats s8 --iters 3 --no-prof --samples $SAMPLES 2>&1 | grep -v amdgpu.ids || exit 1
  python3 scripts/stamps.py gpurun_out/stamps_$n.bin || exit 1
  rm -f gpurun_out/stamps_$n.bin
done
