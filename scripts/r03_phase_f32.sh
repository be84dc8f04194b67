#!/bin/bash
# Round-3 A/B: start offset for half of the first-round workgroups of the one-item-per-
# workgroup wide kernels (64 K cf32, whose items load their 512 KB frame in a burst, and
# the 1 M pair's kernel B), RFA_PHASE_NS on the A/B build; two interleaved rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
V=()
for rnd in 1 2; do
  for ns in 0 4000 8000 12000 16000; do V+=("phase${ns}_$rnd|RFA_LIB=alt/librfa_ab.so RFA_PHASE_NS=$ns"); done
done
bash scripts/ab_kbench.sh gpurun_out/phase_f32.txt "--sizes 65536,1048576 --formats f32,s8 --samples 32768000 --state" "${V[@]}"
