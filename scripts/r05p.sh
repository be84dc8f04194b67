#!/bin/bash
# Round-5 call p: state_fused_kernel walking the ring with 32-bit buffer offsets (one row down per
# frame, no per-frame modulo): state tests on the build, same-call A/B of the config-3 step, rocprof
# of the state kernel per build.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
RFA_LIB=abv/librfa_sb1.so timeout -k 10 400 python -u -m pytest tests/test_gpu_state.py -q --timeout 120 --timeout-method thread > gpurun_out/r05p_pytest.txt 2>&1; rc=$?; tail -1 gpurun_out/r05p_pytest.txt; grep FAILED gpurun_out/r05p_pytest.txt; [ $rc -eq 0 ] || exit $rc
A="--sizes 65536 --formats s8,f32 --samples 32768000 --state"
bash scripts/ab_kbench.sh gpurun_out/r05p_ab.txt "$A" "sb0|RFA_LIB=abv/librfa_sb0.so" "sb1|RFA_LIB=abv/librfa_sb1.so" "sb1u8|RFA_LIB=abv/librfa_sb1u8.so" \
  "sb0_b|RFA_LIB=abv/librfa_sb0.so" "sb1_b|RFA_LIB=abv/librfa_sb1.so" "sb1u8_b|RFA_LIB=abv/librfa_sb1u8.so" || exit 1
for L in sb0 sb1 sb1u8; do
  RFA_LIB=abv/librfa_$L.so timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r05p_prof_$L -o run -- python scripts/kbench.py --sizes 65536 --formats s8 --samples 32768000 --state --iters 20 > gpurun_out/r05p_prof_$L.log 2>&1 || exit 1
done
python3 - <<'PY'
import csv, glob
for L in ("sb0", "sb1", "sb1u8"):
    f = glob.glob(f"gpurun_out/r05p_prof_{L}/**/run_kernel_stats.csv", recursive=True) + glob.glob(f"gpurun_out/r05p_prof_{L}/run_kernel_stats.csv")
    for r in csv.DictReader(open(f[0])):
        if "rfa::" in r["Name"]: print(f"{L:6s} {r['Name'][:60]:60s} calls {r['Calls']:>4} avg {float(r['AverageNs'])/1000:8.2f} us")
PY
