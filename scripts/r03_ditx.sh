#!/bin/bash
# Per-round exchange + pass (RFA_DITX, in-tree) vs contiguous-quarter rounds then the
# whole pass (alt/librfa_noditx.so): 64 K parity subset, three interleaved rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${1:-a}
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
    -k "65536 or 64k or config3 or framing or state_sequence or u8" > gpurun_out/pytest_ditx_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_ditx_$TAG.log; [ $rc -ne 0 ] && exit $rc
V=(); for rnd in 1 2 3; do V+=("noditx_$rnd|RFA_LIB=alt/librfa_noditx.so" "ditx_$rnd|"); done
bash scripts/ab_kbench.sh gpurun_out/ditx_$TAG.txt "--sizes 65536 --formats s8 --samples 32768000 --state" "${V[@]}"
