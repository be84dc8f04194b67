#!/bin/bash
# GPU suite on the in-tree build, then 64 K / 32 K / 128 K A/B of the round-3 kernel
# changes (old = round-2 epilogue, tile = tile-order ring stores, tw = + unfused twiddle
# reads, in-tree = + complex-window pre-stage), then phase stamps of the in-tree kernel.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${1:-c}
[ "${SKIP_PYTEST:-0}" = 1 ] || timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/pytest_gpu_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -8 gpurun_out/pytest_gpu_$TAG.log; [ $rc -ne 0 ] && exit $rc
bash scripts/ab_kbench.sh gpurun_out/ab_${TAG}_64k.txt "--sizes 65536 --formats s8 --samples 32768000 --state" \
  "old|RFA_LIB=alt/librfa_old.so" "tile|RFA_LIB=alt/librfa_tile.so" "tw|RFA_LIB=alt/librfa_tw.so" "cw|" \
  "nt|RFA_LIB=alt/librfa_st_nt.so" "sc1|RFA_LIB=alt/librfa_st_sc1.so" "old2|RFA_LIB=alt/librfa_old.so" "cw2|" || exit $?
bash scripts/ab_kbench.sh gpurun_out/ab_${TAG}_other.txt "--sizes 32768,131072 --formats s8,f32 --samples 32768000 --state" \
  "old|RFA_LIB=alt/librfa_old.so" "cw|" || exit $?
rm -f gpurun_out/stamps_$TAG.bin
RFA_LIB=alt/librfa_ab.so RFA_STAMPS_FILE=gpurun_out/stamps_$TAG.bin timeout -k 10 120 python -u scripts/kbench.py \
  --sizes 65536 --formats s8 --samples 32768000 --state --iters 8 > /dev/null 2>&1
rc=$?; echo "stamps rc=$rc"; [ $rc -ne 0 ] && exit $rc
python scripts/stamps.py gpurun_out/stamps_$TAG.bin | tee gpurun_out/stamps_$TAG.txt
