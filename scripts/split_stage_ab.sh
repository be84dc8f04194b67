#!/bin/bash
# RFA_SPLIT_STAGE A/B in ONE GPU call: the whole GPU suite on the split-staging
# build (alt/librfa_split.so), then 64 K kernel time in-tree vs split.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
RFA_LIB=alt/librfa_split.so timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 \
    --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_split.log 2>&1
rc=$?; echo "pytest(split) rc=$rc"; tail -3 gpurun_out/pytest_split.log; [ $rc -ne 0 ] && exit $rc
bash scripts/ab_kbench.sh gpurun_out/split_stage_ab.txt "--sizes 65536 --formats s8,u8 --samples 32768000 --state --iters 100" \
    "intree|" "split|RFA_LIB=alt/librfa_split.so" "intree2|" "split2|RFA_LIB=alt/librfa_split.so" || exit $?
