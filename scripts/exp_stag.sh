#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for st in 0 12000 24000; do
  for p in 1 0; do echo "== PAIR=$p STAGGER=$st"; RFA_PAIR=$p RFA_STAGGER_NS=$st timeout -k 10 200 python scripts/kbench.py --sizes 65536 --formats s8 --iters 10 --samples 134217728 2>&1 | grep -v amdgpu.ids || exit 1; done
done
