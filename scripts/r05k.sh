#!/bin/bash
# Round-5 call k: the product build with the new large-N front kernel (LO = 6 split, 16-B sc1 z
# stores, misaligned 8-bit frames staged aligned): parity + state suites, same-call A/B vs the
# round-4 head build at 256 K / 512 K / 1 M, rocprof split of the 1 M pair.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_state.py tests/test_gpu_seam.py -q --timeout 120 --timeout-method thread > gpurun_out/r05k_pytest.txt 2>&1; rc=$?; tail -1 gpurun_out/r05k_pytest.txt; grep FAILED gpurun_out/r05k_pytest.txt; [ $rc -eq 0 ] || exit $rc
A="--sizes 262144,524288,1048576 --formats s8 --samples 16777216 --state"
bash scripts/ab_kbench.sh gpurun_out/r05k_ab.txt "$A" "base|RFA_LIB=abv/librfa_base.so" "new|" "base_b|RFA_LIB=abv/librfa_base.so" "new_b|" || exit 1
A1="--sizes 1048576 --formats s8 --samples 16777216 --state --iters 10"
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r05k_prof -o run -- python scripts/kbench.py $A1 > gpurun_out/r05k_prof.log 2>&1 || exit 1
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/r05k_prof/**/run_kernel_stats.csv", recursive=True) + glob.glob("gpurun_out/r05k_prof/run_kernel_stats.csv")
for r in csv.DictReader(open(f[0])):
    if "rfa::" in r["Name"]: print(f"{r['Name'][:70]:70s} calls {r['Calls']:>4} avg {float(r['AverageNs'])/1000:8.2f} us")
PY
