#!/bin/bash
# Round-4 A/B, same call: the large-N front kernel with 512-column blocks (alt/librfa_bw512.so,
# -DRFA_DIF_BW=512: one D table per 8 waves, 4 waves per SIMD) against the same tree's A/B build
# (alt/librfa_ab4.so, 256-column blocks); 1 M parity through the 512-column build.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${1:-r04n}
export TMPDIR=/tmp RFA_W64_FORMATS=0
V=()
for rnd in 1 2 3; do V+=("bw256_$rnd|RFA_LIB=alt/librfa_ab4.so" "bw512_$rnd|RFA_LIB=alt/librfa_bw512.so"); done
bash scripts/ab_kbench.sh gpurun_out/bw_ab_$TAG.txt "--sizes 262144,524288,1048576 --formats s8" "${V[@]}" || exit $?
bash scripts/ab_kbench.sh gpurun_out/bw_ab_state_$TAG.txt "--sizes 1048576 --formats s8 --samples 16777216 --state" "${V[@]}" || exit $?
RFA_LIB=alt/librfa_bw512.so timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread -p no:cacheprovider \
    tests/test_gpu_parity.py tests/test_gpu_state.py -k "1048576 or 524288 or 262144 or large_n or column_order" > gpurun_out/pytest_bw512_$TAG.log 2>&1
rc=$?; echo "pytest bw512 rc=$rc"; tail -3 gpurun_out/pytest_bw512_$TAG.log
exit 0
