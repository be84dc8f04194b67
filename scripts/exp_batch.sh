#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for sm in 16777216 33554432 67108864; do
  for p in 1 0; do echo "== samples $sm PAIR=$p"; RFA_PAIR=$p timeout -k 10 200 python scripts/kbench.py --sizes 16384,65536 --formats s8 --iters 10 --samples $sm 2>&1 | grep -v amdgpu.ids || exit 1; done
done
