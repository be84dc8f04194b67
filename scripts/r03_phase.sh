#!/bin/bash
# Two 16 K workgroups per CU (persistent, LDS-staged): does a phase offset between them
# (RFA_PHASE_NS: the grid's second half starts late) let their phases interleave?
# 4096 frames = 8 items per workgroup; two interleaved rounds, one call.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
V=()
for rnd in 1 2; do
  for ns in 0 4500 9000 13500; do V+=("phase${ns}_$rnd|RFA_LIB=alt/librfa_ab.so RFA_PHASE_NS=$ns"); done
done
bash scripts/ab_kbench.sh gpurun_out/phase_${1:-a}.txt "--sizes 16384 --formats s8 --samples 67108864" "${V[@]}"
