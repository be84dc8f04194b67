#!/bin/bash
# RFA_SPLIT_WHOLE A/B in ONE GPU call: GPU suite on alt/librfa_whole.so, then
# 16 K / 32 K one-residue kernels in-tree vs whole-frame-in-region-B staging.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
RFA_LIB=alt/librfa_whole.so timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 \
    --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_whole.log 2>&1
rc=$?; echo "pytest(whole) rc=$rc"; tail -3 gpurun_out/pytest_whole.log; [ $rc -ne 0 ] && exit $rc
bash scripts/ab_kbench.sh gpurun_out/split_whole_ab.txt "--sizes 8192,16384,32768 --formats s8,u8 --iters 40" \
    "intree|" "whole|RFA_LIB=alt/librfa_whole.so" "intree2|" "whole2|RFA_LIB=alt/librfa_whole.so" || exit $?
