#!/bin/bash
# Round-4 A/B, same call: the ring's 16-B tile stores with sc1 (write-through, the line leaves the
# XCD L2, MI355X_MICROARCH.md store flavours) so 128 KB of ring per item stops evicting the window
# tables and staged frames: alt/librfa_sc1.so (-DRFA_ST_SC1) against alt/librfa_ab5.so (same
# tree); FETCH_SIZE of both at the headline workload; the headline bench line of both.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${1:-r04x}
export TMPDIR=/tmp RFA_W64_FORMATS=0
V=()
for rnd in 1 2 3; do V+=("ab5_$rnd|RFA_LIB=alt/librfa_ab5.so" "sc1_$rnd|RFA_LIB=alt/librfa_sc1.so"); done
bash scripts/ab_kbench.sh gpurun_out/sc1_ab_$TAG.txt "--sizes 32768,65536,131072 --formats s8,f32 --samples 32768000 --state" "${V[@]}" || exit $?
for v in ab5 sc1; do
  rm -rf gpurun_out/pmcsc_${v}_$TAG
  RFA_LIB=alt/librfa_$v.so timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmcsc_${v}_$TAG -o p -- \
      python3 scripts/kbench.py --iters 3 --sizes 65536 --formats s8 --samples 32768000 --state > gpurun_out/pmcsc_${v}_$TAG.log 2>&1 || { echo "pmc $v failed"; exit 1; }
  python3 - "$v" "$TAG" <<'PY'
import csv, glob, statistics, sys
v, tag = sys.argv[1:3]
f = glob.glob(f"gpurun_out/pmcsc_{v}_{tag}/**/*counter_collection.csv", recursive=True)[0]
vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(f)) if r["Counter_Name"] == "FETCH_SIZE" and "fft_wide_kernel" in r["Kernel_Name"]]
print(v, "FETCH bytes per launch (x2 gfx950 correction):", round(2 * statistics.median(vals) * 1024))
PY
done | tee -a gpurun_out/sc1_ab_$TAG.txt
NOC="--cpu-seconds 0 --f32-steps 0 --c5-steps 0 --c2-steps 0 --c4-steps 0 --demod-steps 0"
for rnd in 1 2; do for v in ab5 sc1; do
  RFA_LIB=alt/librfa_$v.so timeout -k 10 300 python bench.py $NOC > gpurun_out/bench_${v}_$TAG.json 2> gpurun_out/bench_${v}_$TAG.err || exit $?
  python3 -c "import json;d=json.load(open('gpurun_out/bench_${v}_$TAG.json'));print('bench $v', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'])" | tee -a gpurun_out/sc1_ab_$TAG.txt
done; done
RFA_LIB=alt/librfa_sc1.so timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread -p no:cacheprovider \
    tests/test_gpu_parity.py tests/test_gpu_state.py -k "65536 or 32768 or 131072 or config3" > gpurun_out/pytest_sc1_$TAG.log 2>&1
rc=$?; echo "pytest sc1 rc=$rc"; tail -2 gpurun_out/pytest_sc1_$TAG.log
