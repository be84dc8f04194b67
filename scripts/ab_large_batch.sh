#!/bin/bash
# A/B: large-N scratch batch size (RFA_DIT_SCRATCH_MB) at N = 1 M, ring + state.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for mb in 128 64 32; do
  echo "== scratch $mb MB"
  RFA_DIT_SCRATCH_MB=$mb timeout -k 10 120 python3 scripts/kbench.py --sizes 1048576 --formats s8,f32 --samples 67108864 --iters 10 --state || exit $?
done
