#!/bin/bash
# Round-5 call r: 8 K one-round exchanges (RFA_WIDE_KR1: M-sized buffer, 2 workgroups per CU,
# half the barriers) vs the product's two-round form: 8 K parity on the build, same-call A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
RFA_LIB=abv/librfa_kr1.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "8192" -q --timeout 120 --timeout-method thread > gpurun_out/r05r_pytest.txt 2>&1; rc=$?; tail -1 gpurun_out/r05r_pytest.txt; grep FAILED gpurun_out/r05r_pytest.txt; [ $rc -eq 0 ] || exit $rc
A="--sizes 8192 --formats s8,f32 --samples 134217728"
bash scripts/ab_kbench.sh gpurun_out/r05r_ab.txt "$A" "base|RFA_LIB=abv/librfa_sb1.so" "kr1|RFA_LIB=abv/librfa_kr1.so" "base_b|RFA_LIB=abv/librfa_sb1.so" "kr1_b|RFA_LIB=abv/librfa_kr1.so"
