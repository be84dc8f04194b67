#!/bin/bash
# A/B: large-N front kernel ablations (alt/librfa_abl*.so) vs the in-tree build, kernel stats per variant.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for v in base abl1 abl2; do
  lib=""; [ $v != base ] && lib="RFA_LIB=alt/librfa_$v.so"
  scripts/prof_kbench.sh dif_$v "--sizes 1048576 --formats s8,f32 --iters 10 --state" $lib || exit $?
done
