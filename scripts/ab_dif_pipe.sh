#!/bin/bash
# A/B: pipelined persistent large-N front kernel, frame groups RFA_DIF_PIPE (0 = one block per tile).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for p in 0 2 4 6 8 16; do
  echo "== RFA_DIF_PIPE=$p"
  RFA_DIF_PIPE=$p timeout -k 10 120 python3 scripts/kbench.py --sizes 262144,1048576 --formats s8 --iters 20 --state | grep -v amdgpu.ids || exit $?
done
