#!/bin/bash
# Round-5 call f: in-grid state v4 (pipelined unit loads; tail 1 / unbounded / 4 units): diagnostics,
# state tests on the build, same-call A/B of the 64 K step vs the baseline.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
RFA_LIB=abv/librfa_igs4d.so timeout -k 10 200 python scripts/igs_debug.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r05g_debug.txt &&
RFA_LIB=abv/librfa_igs4.so timeout -k 10 400 python -u -m pytest tests/test_gpu_state.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r05g_pytest.txt 2>&1; rc=$?; tail -1 gpurun_out/r05g_pytest.txt; [ $rc -eq 0 ] &&
bash scripts/ab_kbench.sh gpurun_out/r05g_ab.txt "--sizes 65536 --formats s8,f32 --samples 32768000 --state" \
  "base|RFA_LIB=abv/librfa_base.so" "igs4|RFA_LIB=abv/librfa_igs4.so" "igs4u|RFA_LIB=abv/librfa_igs4u.so" "igs4t4|RFA_LIB=abv/librfa_igs4t4.so" \
  "base_b|RFA_LIB=abv/librfa_base.so" "igs4_b|RFA_LIB=abv/librfa_igs4.so" "igs4u_b|RFA_LIB=abv/librfa_igs4u.so" "igs4t4_b|RFA_LIB=abv/librfa_igs4t4.so"
