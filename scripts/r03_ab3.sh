#!/bin/bash
# Round-3 64 K kernel changes, three interleaved rounds per variant (one call):
# old = round-2 epilogue (dword ring stores), tile = 16-B store-tile ring order,
# tw = + unfused pass-1/2 twiddle reads, cw (in-tree) = + complex-window residue-1 pre-stage.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
V=()
for rnd in 1 2 3; do
  V+=("old$rnd|RFA_LIB=alt/librfa_old.so" "tile$rnd|RFA_LIB=alt/librfa_tile.so" "tw$rnd|RFA_LIB=alt/librfa_tw.so" "cw$rnd|")
done
bash scripts/ab_kbench.sh gpurun_out/ab3_${1:-a}.txt "--sizes 65536 --formats s8 --samples 32768000 --state" "${V[@]}"
