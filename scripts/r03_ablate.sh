#!/bin/bash
# 64 K store ablations in one call (A/B build alt/librfa_diag12.so, -DRFA_DIAG_STG12).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
L=alt/librfa_diag12.so
bash scripts/ab_kbench.sh gpurun_out/store_ablation_${1:-a}.txt "--sizes 65536 --formats s8 --samples 32768000 --state" \
  "full|RFA_LIB=$L" "no_stores|RFA_LIB=$L RFA_DIAG=2" "x4_tile_stores|RFA_LIB=$L RFA_DIAG=64" \
  "stream_only|RFA_LIB=$L RFA_DIAG=12" "stream_only_no_stores|RFA_LIB=$L RFA_DIAG=14" \
  "stream_only_x4|RFA_LIB=$L RFA_DIAG=76" "full_again|RFA_LIB=$L"
