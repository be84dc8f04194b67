#!/bin/bash
# Round-5 call n: 16-B write-through z stores in the per-tile large-N front kernel too (f32 / s16
# input): parity suites on the product build, same-call A/B vs the 8-B-store build (p2nost).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_state.py tests/test_gpu_seam.py -q --timeout 120 --timeout-method thread > gpurun_out/r05n_pytest.txt 2>&1; rc=$?; tail -1 gpurun_out/r05n_pytest.txt; grep FAILED gpurun_out/r05n_pytest.txt; [ $rc -eq 0 ] || exit $rc
A="--sizes 262144,1048576 --formats f32,s16 --samples 16777216 --state"
bash scripts/ab_kbench.sh gpurun_out/r05n_ab.txt "$A" "nost|RFA_LIB=abv/librfa_p2nost.so" "new|" "nost_b|RFA_LIB=abv/librfa_p2nost.so" "new_b|" || exit 1
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r05n_prof -o run -- python scripts/kbench.py --sizes 1048576 --formats f32 --samples 16777216 --state --iters 10 > gpurun_out/r05n_prof.log 2>&1 || exit 1
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/r05n_prof/**/run_kernel_stats.csv", recursive=True) + glob.glob("gpurun_out/r05n_prof/run_kernel_stats.csv")
for r in csv.DictReader(open(f[0])):
    if "rfa::" in r["Name"]: print(f"{r['Name'][:70]:70s} calls {r['Calls']:>4} avg {float(r['AverageNs'])/1000:8.2f} us")
PY
