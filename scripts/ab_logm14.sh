#!/bin/bash
# A/B: 64 K as 4 residues of 16 K (two workgroups per CU, RFA_WIDE_LOGM=14) vs 2 residues of 32 K,
# both with the residue-major ring, B = 500, state on.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for lm in 15 14 15 14; do
  echo "== RFA_WIDE_LOGM=$lm"
  RFA_WIDE_LOGM=$lm timeout -k 10 120 python3 scripts/kbench.py --sizes 65536 --formats s8,f32 --samples 32768000 --iters 40 --state | grep -v amdgpu.ids || exit $?
done
