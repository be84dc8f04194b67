#!/bin/bash
# Round-4 A/B, same call: the 64 K float-input pre-stage with its loads two chunks ahead
# (alt/librfa_d2.so, -DRFA_PRE_DIST_F32=2) against one chunk (alt/librfa_d1.so, same tree).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${1:-r04y}
export TMPDIR=/tmp RFA_W64_FORMATS=0
V=()
for rnd in 1 2 3; do V+=("d1_$rnd|RFA_LIB=alt/librfa_d1.so" "d2_$rnd|RFA_LIB=alt/librfa_d2.so"); done
bash scripts/ab_kbench.sh gpurun_out/dist_ab_$TAG.txt "--sizes 65536 --formats f32,f32p" "${V[@]}" || exit $?
bash scripts/ab_kbench.sh gpurun_out/dist_ab_state_$TAG.txt "--sizes 65536 --formats f32 --samples 32768000 --state" "${V[@]}" || exit $?
RFA_LIB=alt/librfa_d2.so timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread -p no:cacheprovider \
    tests/test_gpu_parity.py -k "65536" > gpurun_out/pytest_d2_$TAG.log 2>&1
rc=$?; echo "pytest d2 rc=$rc"; tail -2 gpurun_out/pytest_d2_$TAG.log
