#!/bin/bash
# Config-5 (1 M-point) evidence: kernel split (rocprofv3 stats) and per-kernel
# FETCH_SIZE / WRITE_SIZE (separate --pmc passes), for kbench at N = 1 M.
# usage: scripts/prof_large.sh TAG [FORMATS]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=$1; FMTS=${2:-s8,f32}
mkdir -p gpurun_out
scripts/prof_kbench.sh "$TAG" "--sizes 1048576 --formats $FMTS --iters 10" || exit $?
for c in FETCH_SIZE WRITE_SIZE; do
  rm -rf "gpurun_out/pmc_${TAG}_$c"
  timeout -s KILL 90 rocprofv3 --pmc $c --output-format csv -d "gpurun_out/pmc_${TAG}_$c" -o p -- \
      python3 scripts/kbench.py --sizes 1048576 --formats $FMTS --iters 3 > "gpurun_out/pmc_${TAG}_$c.log" 2>&1
  rc=$?; [ $rc -ne 0 ] && { echo "pmc $c rc=$rc"; exit $rc; }
  python3 - "$TAG" "$c" <<'PY'
import csv, glob, sys, collections
tag, c = sys.argv[1:3]
f = sorted(glob.glob(f"gpurun_out/pmc_{tag}_{c}/**/*counter_collection.csv", recursive=True))
acc = collections.defaultdict(list)
for r in csv.DictReader(open(f[-1])):
    if "rfa::" in r["Kernel_Name"] and r["Counter_Name"] == c:
        acc[r["Kernel_Name"][:90]].append(float(r["Counter_Value"]))
for k, v in acc.items():
    v = v[len(v) // 2:]  # the later launches (after warmup)
    mb = sum(v) / len(v) * 1024 / 1e6 * (2 if c == "FETCH_SIZE" else 1)
    print(f"{c:10s} {mb:9.1f} MB/launch (x{len(v)}; FETCH doubled per the guide)  {k}")
PY
done
