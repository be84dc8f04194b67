#!/bin/bash
# Round-5 call b: C-ABI per-call cost, state/parity GPU tests on the in-grid state build,
# same-call A/B of the 64 K step (HEAD vs in-grid off vs on), then the bench line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 ./tools/call_bench 4000 1 > gpurun_out/r05b_call1.json 2>&1 && cat gpurun_out/r05b_call1.json &&
timeout -k 10 120 ./tools/call_bench 100 64 > gpurun_out/r05b_call64.json 2>&1 && cat gpurun_out/r05b_call64.json &&
timeout -k 10 400 python -u -m pytest tests/test_gpu_state.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r05b_pytest.txt 2>&1; rc=$?; tail -3 gpurun_out/r05b_pytest.txt; [ $rc -eq 0 ] &&
bash scripts/ab_kbench.sh gpurun_out/r05b_ab.txt "--sizes 65536 --formats s8,f32 --samples 32768000 --state" \
  "base|RFA_LIB=abv/librfa_base.so" "igs_off|RFA_LIB=abv/librfa_igs.so RFA_IGS=0" "igs_on|RFA_LIB=abv/librfa_igs.so" \
  "base2|RFA_LIB=abv/librfa_base.so" "igs_on2|RFA_LIB=abv/librfa_igs.so" "pf|RFA_LIB=abv/librfa_pf.so" "pf_off|RFA_LIB=abv/librfa_pf.so RFA_IGS=0" &&
timeout -k 10 600 python -u bench.py --cpu-seconds 3 > gpurun_out/r05b_bench.json 2> gpurun_out/r05b_bench.err; rc=$?; tail -c 400 gpurun_out/r05b_bench.json; exit $rc
