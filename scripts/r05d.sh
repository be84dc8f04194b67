#!/bin/bash
# Round-5 call d: in-grid state v2 (noinline 16-B-load units, -DRFA_IGS=1): state + parity tests on
# that build, same-call A/B of the 64 K step against the product build, then its bench line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
RFA_LIB=abv/librfa_igs2.so timeout -k 10 400 python -u -m pytest tests/test_gpu_state.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r05d_pytest.txt 2>&1; rc=$?; tail -2 gpurun_out/r05d_pytest.txt; [ $rc -eq 0 ] &&
bash scripts/ab_kbench.sh gpurun_out/r05d_ab.txt "--sizes 65536 --formats s8,f32 --samples 32768000 --state" \
  "base|RFA_LIB=abv/librfa_base5.so" "igs2|RFA_LIB=abv/librfa_igs2.so" "igs2_off|RFA_LIB=abv/librfa_igs2.so RFA_IGS=0" \
  "base_b|RFA_LIB=abv/librfa_base5.so" "igs2_b|RFA_LIB=abv/librfa_igs2.so" &&
NOC="--cpu-seconds 0 --f32-steps 0 --c5-steps 0 --c2-steps 0 --c4-steps 0 --demod-steps 0 --host-fed-calls 0"
RFA_LIB=abv/librfa_igs2.so timeout -k 10 300 python -u bench.py $NOC > gpurun_out/r05d_bench_igs2.json 2>&1; tail -c 300 gpurun_out/r05d_bench_igs2.json;
RFA_LIB=abv/librfa_base5.so timeout -k 10 300 python -u bench.py $NOC > gpurun_out/r05d_bench_base.json 2>&1; tail -c 300 gpurun_out/r05d_bench_base.json
