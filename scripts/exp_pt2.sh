#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for pt in 32 64; do
  echo "== PT=$pt"
  RFA_PT=$pt timeout -k 10 200 python scripts/precision.py || exit $?
  RFA_PT=$pt timeout -k 10 200 python scripts/kbench.py --sizes 16384,65536 --formats s8 --samples 67108864 || exit $?
done
