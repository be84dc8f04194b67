#!/bin/bash
# 64 K kernel probes in one call (A/B build alt/librfa_diag.so, -DRFA_DIAG_STG12):
# phase stamps with and without window loads (stamp 7 = the pre-stage barrier), then
# ablations, every variant twice in interleaved order.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${1:-e}
L=alt/librfa_diag.so
K="--sizes 65536 --formats s8 --samples 32768000 --state"
for d in ${STAMPS:-0 16}; do
  rm -f gpurun_out/stamps_${TAG}_$d.bin
  RFA_LIB=$L RFA_DIAG=$d RFA_STAMPS_FILE=gpurun_out/stamps_${TAG}_$d.bin timeout -k 10 120 python -u scripts/kbench.py \
    $K --iters 8 > /dev/null 2>&1
  rc=$?; echo "stamps diag $d rc=$rc"; [ $rc -ne 0 ] && exit $rc
  python scripts/stamps.py gpurun_out/stamps_${TAG}_$d.bin > gpurun_out/stamps_${TAG}_$d.txt
done
V=()
for rnd in 1 2; do
  V+=("full$rnd|RFA_LIB=$L" "nowin$rnd|RFA_LIB=$L RFA_DIAG=16" "nobfly$rnd|RFA_LIB=$L RFA_DIAG=4"
      "noxchg$rnd|RFA_LIB=$L RFA_DIAG=8" "stream$rnd|RFA_LIB=$L RFA_DIAG=12" "stream_nowin$rnd|RFA_LIB=$L RFA_DIAG=28"
      "nostores$rnd|RFA_LIB=$L RFA_DIAG=2" "intree$rnd|")
done
bash scripts/ab_kbench.sh gpurun_out/probe_${TAG}.txt "$K" "${V[@]}"
