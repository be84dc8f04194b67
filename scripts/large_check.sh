#!/bin/bash
# Large-N (2^18..2^20) check: parity subset, then kernel split with rows and with the ring.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-l02}
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_state.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "1048576 or 262144 or 524288 or large or retune" > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_$TAG.log
[ $rc -ge 124 ] && exit $rc
scripts/prof_kbench.sh ${TAG}_rows "--sizes 262144,1048576 --formats s8,f32 --iters 10" || exit $?
scripts/prof_kbench.sh ${TAG}_ring "--sizes 262144,1048576 --formats s8,f32 --iters 10 --state" || exit $?
# HBM traffic per launch of the large-N kernels (ring + state), one --pmc pass per counter
for c in FETCH_SIZE WRITE_SIZE; do
  rm -rf "gpurun_out/pmc_${TAG}_$c"
  timeout -s KILL 90 rocprofv3 --pmc $c --output-format csv -d "gpurun_out/pmc_${TAG}_$c" -o p -- \
      python3 scripts/kbench.py --sizes 1048576 --formats s8,f32 --iters 3 --state > "gpurun_out/pmc_${TAG}_$c.log" 2>&1 || exit $?
  python3 - "$TAG" "$c" <<'PY'
import csv, glob, sys, collections
tag, c = sys.argv[1:3]
f = sorted(glob.glob(f"gpurun_out/pmc_{tag}_{c}/**/*counter_collection.csv", recursive=True))
acc = collections.defaultdict(list)
for r in csv.DictReader(open(f[-1])):
    if "rfa::" in r["Kernel_Name"] and r["Counter_Name"] == c:
        acc[r["Kernel_Name"][:80]].append(float(r["Counter_Value"]))
for k, v in acc.items():
    v = v[len(v) // 2:]
    mb = sum(v) / len(v) * 1024 / 1e6 * (2 if c == "FETCH_SIZE" else 1)
    print(f"{c:10s} {mb:9.1f} MB/launch (x{len(v)}, FETCH doubled per the guide)  {k}")
PY
done
