#!/bin/bash
# Round-5 call f: in-grid state v3 (compare-exchange tickets, tail wait 0 / 5 us): diagnostics,
# state tests on the build, same-call A/B of the 64 K step vs the baseline.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
RFA_LIB=abv/librfa_igs3d.so timeout -k 10 200 python scripts/igs_debug.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r05f_debug.txt &&
RFA_LIB=abv/librfa_igs3.so timeout -k 10 400 python -u -m pytest tests/test_gpu_state.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r05f_pytest.txt 2>&1; rc=$?; tail -1 gpurun_out/r05f_pytest.txt; [ $rc -eq 0 ] &&
bash scripts/ab_kbench.sh gpurun_out/r05f_ab.txt "--sizes 65536 --formats s8,f32 --samples 32768000 --state" \
  "base|RFA_LIB=abv/librfa_base.so" "igs3|RFA_LIB=abv/librfa_igs3.so" "igs3w|RFA_LIB=abv/librfa_igs3w.so" \
  "base_b|RFA_LIB=abv/librfa_base.so" "igs3_b|RFA_LIB=abv/librfa_igs3.so" "igs3w_b|RFA_LIB=abv/librfa_igs3w.so"
