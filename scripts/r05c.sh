#!/bin/bash
# Round-5 call c: same-call A/B of static wave priorities in the 64 K kernel (waves 8-15 or 0-7 at prio 1).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
bash scripts/ab_kbench.sh gpurun_out/r05c_ab.txt "--sizes 65536 --formats s8,f32 --samples 32768000 --state" \
  "base|RFA_LIB=abv/librfa_base5.so" "prio1|RFA_LIB=abv/librfa_prio1.so" "prio2|RFA_LIB=abv/librfa_prio2.so" \
  "base_b|RFA_LIB=abv/librfa_base5.so" "prio1_b|RFA_LIB=abv/librfa_prio1.so" "prio2_b|RFA_LIB=abv/librfa_prio2.so"
