#!/bin/bash
# Round-5 call e: in-grid state v2 on the WIDE kernel (A/B builds now default to it): diagnostics,
# state tests on that build, same-call A/B of the 64 K step vs the baseline, bench lines of both.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
RFA_LIB=abv/librfa_igs2d.so timeout -k 10 200 python scripts/igs_debug.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r05e_debug.txt &&
RFA_LIB=abv/librfa_igs2.so timeout -k 10 400 python -u -m pytest tests/test_gpu_state.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r05e_pytest.txt 2>&1; rc=$?; tail -1 gpurun_out/r05e_pytest.txt; [ $rc -eq 0 ] &&
bash scripts/ab_kbench.sh gpurun_out/r05e_ab.txt "--sizes 65536 --formats s8,f32 --samples 32768000 --state" \
  "base|RFA_LIB=abv/librfa_base.so" "igs2|RFA_LIB=abv/librfa_igs2.so" "igs2_off|RFA_LIB=abv/librfa_igs2.so RFA_IGS=0" \
  "base_b|RFA_LIB=abv/librfa_base.so" "igs2_b|RFA_LIB=abv/librfa_igs2.so" &&
NOC="--cpu-seconds 0 --f32-steps 0 --c5-steps 0 --c2-steps 0 --c4-steps 0 --demod-steps 0 --host-fed-calls 0" &&
RFA_LIB=abv/librfa_igs2.so timeout -k 10 300 python -u bench.py $NOC > gpurun_out/r05e_bench_igs2.json 2>&1 &&
RFA_LIB=abv/librfa_base.so timeout -k 10 300 python -u bench.py $NOC > gpurun_out/r05e_bench_base.json 2>&1 &&
RFA_LIB=abv/librfa_igs2.so timeout -k 10 300 python -u bench.py $NOC > gpurun_out/r05e_bench_igs2b.json 2>&1; rc=$?
for f in gpurun_out/r05e_bench_*.json; do python3 -c "
import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])"; done
exit $rc
