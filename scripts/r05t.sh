#!/bin/bash
# Round-5 call t: state_fused_kernel with 1024-thread blocks (one wave per chunk: every row load
# instruction is 1 KB contiguous of one row) vs 256 (four 256-B pieces of four rows): state tests on
# the build, same-call A/B, rocprof of the state kernel.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
RFA_LIB=abv/librfa_nt1024.so timeout -k 10 400 python -u -m pytest tests/test_gpu_state.py -q --timeout 120 --timeout-method thread > gpurun_out/r05t_pytest.txt 2>&1; rc=$?; tail -1 gpurun_out/r05t_pytest.txt; grep FAILED gpurun_out/r05t_pytest.txt; [ $rc -eq 0 ] || exit $rc
A="--sizes 65536 --formats s8 --samples 32768000 --state"
bash scripts/ab_kbench.sh gpurun_out/r05t_ab.txt "$A" "nt256|RFA_LIB=abv/librfa_nt256.so" "nt1024|RFA_LIB=abv/librfa_nt1024.so" "nt256_b|RFA_LIB=abv/librfa_nt256.so" "nt1024_b|RFA_LIB=abv/librfa_nt1024.so" || exit 1
for L in nt256 nt1024; do
  RFA_LIB=abv/librfa_$L.so timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r05t_prof_$L -o run -- python scripts/kbench.py $A --iters 20 > gpurun_out/r05t_prof_$L.log 2>&1 || exit 1
done
python3 - <<'PY'
import csv, glob
for L in ("nt256", "nt1024"):
    f = glob.glob(f"gpurun_out/r05t_prof_{L}/run_kernel_stats.csv")
    for r in csv.DictReader(open(f[0])):
        if "rfa::" in r["Name"]: print(f"{L:7s} {r['Name'][:60]:60s} calls {r['Calls']:>4} avg {float(r['AverageNs'])/1000:8.2f} us")
PY
