#!/bin/bash
# A/B kernel timings inside ONE GPU call (boxes differ by up to +-10 %, so
# variants are only ever compared within a call).
#
# usage: scripts/ab_kbench.sh OUT "KBENCH_ARGS" "label|ENV=v ENV2=v" ["label|..."]...
#   e.g. scripts/ab_kbench.sh gpurun_out/ab.txt "--sizes 65536 --formats s8 --samples 32768000" \
#          "base|RFA_LIB=alt/librfa_base.so" "new|" "rmajor|RFA_DIAG=64"
# Each variant runs scripts/kbench.py once under its environment; the first
# failing variant (timeout, crash) ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$1; shift
ARGS=$1; shift
mkdir -p "$(dirname "$OUT")"
: > "$OUT"
for v in "$@"; do
  label=${v%%|*}; envs=${v#*|}
  echo "== $label ($envs)" | tee -a "$OUT"
  # shellcheck disable=SC2086
  env $envs timeout -k 10 120 python -u scripts/kbench.py $ARGS 2>&1 | grep -v amdgpu.ids | tee -a "$OUT"
  rc=${PIPESTATUS[0]}
  if [ "$rc" -ne 0 ]; then echo "variant $label rc=$rc" | tee -a "$OUT"; exit "$rc"; fi
done
