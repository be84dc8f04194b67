#!/bin/bash
# A/B: start delay of the second half of the 64 K persistent grid (RFA_STAGGER_NS), B = 500 frames, state on.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for ns in 0 2000 5000 10000 0; do
  echo "== RFA_STAGGER_NS=$ns"
  RFA_STAGGER_NS=$ns timeout -k 10 120 python3 scripts/kbench.py --sizes 65536 --formats s8 --samples 32768000 --iters 40 --state | grep -v amdgpu.ids || exit $?
done
