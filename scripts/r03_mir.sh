#!/bin/bash
# Mirrored-lane 64 K kernel: GPU parity suite (64 K parity, ring, state, framing), A/B
# against the pair / complex-window pre-stage (alt/librfa_nomir.so), three interleaved
# rounds, 64 K s8 and u8; phase stamps of the mirrored kernel (alt/librfa_ab.so).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${1:-a}
[ "${SKIP_PYTEST:-0}" = 1 ] || timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
    -k "65536 or 64k or config3 or ring or state or framing or jni" > gpurun_out/pytest_mir_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_mir_$TAG.log; [ $rc -ne 0 ] && exit $rc
V=()
for rnd in 1 2 3; do V+=("nomir$rnd|RFA_LIB=alt/librfa_nomir.so" "mir$rnd|"); done
bash scripts/ab_kbench.sh gpurun_out/ab_mir_$TAG.txt "--sizes 65536 --formats s8,u8 --samples 32768000 --state" "${V[@]}" || exit $?
rm -f gpurun_out/stamps_mir_$TAG.bin
RFA_LIB=alt/librfa_ab.so RFA_STAMPS_FILE=gpurun_out/stamps_mir_$TAG.bin timeout -k 10 120 python -u scripts/kbench.py \
  --sizes 65536 --formats s8 --samples 32768000 --state --iters 8 > /dev/null 2>&1
rc=$?; echo "stamps rc=$rc"; [ $rc -ne 0 ] && exit $rc
python scripts/stamps.py gpurun_out/stamps_mir_$TAG.bin > gpurun_out/stamps_mir_$TAG.txt
