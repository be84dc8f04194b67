#!/bin/bash
# Round-5 call q: ring tile stores without sc1 (write-back) -- does the state pass then read the
# ring faster (Infinity Cache) and does the FFT kernel lose?  Same-call A/B + rocprof split.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
A="--sizes 65536 --formats s8,f32 --samples 32768000 --state"
bash scripts/ab_kbench.sh gpurun_out/r05q_ab.txt "$A" "sb1|RFA_LIB=abv/librfa_sb1.so" "rsc0|RFA_LIB=abv/librfa_rsc0.so" "sb1_b|RFA_LIB=abv/librfa_sb1.so" "rsc0_b|RFA_LIB=abv/librfa_rsc0.so" || exit 1
for L in sb1 rsc0; do
  RFA_LIB=abv/librfa_$L.so timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r05q_prof_$L -o run -- python scripts/kbench.py --sizes 65536 --formats s8 --samples 32768000 --state --iters 20 > gpurun_out/r05q_prof_$L.log 2>&1 || exit 1
done
python3 - <<'PY'
import csv, glob
for L in ("sb1", "rsc0"):
    f = glob.glob(f"gpurun_out/r05q_prof_{L}/**/run_kernel_stats.csv", recursive=True) + glob.glob(f"gpurun_out/r05q_prof_{L}/run_kernel_stats.csv")
    for r in csv.DictReader(open(f[0])):
        if "rfa::" in r["Name"]: print(f"{L:6s} {r['Name'][:60]:60s} calls {r['Calls']:>4} avg {float(r['AverageNs'])/1000:8.2f} us")
PY
