#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for d in 0 64; do echo "== DIAG $d"; RFA_DIAG=$d timeout -k 10 120 python scripts/kbench.py --sizes 65536 --formats s8 --iters 20 2>&1 | grep -v amdgpu.ids || exit 1; done
for d in 0 64; do
  rm -rf gpurun_out/pmcw_amp$d
  RFA_DIAG=$d timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmcw_amp$d -o p -- python3 scripts/kbench.py --sizes 65536 --formats s8 --iters 3 > /dev/null 2>&1 || { echo "pmc $d failed"; exit 1; }
  python3 - $d <<'PY'
import csv, glob, sys
f = glob.glob(f"gpurun_out/pmcw_amp{sys.argv[1]}/**/*counter_collection.csv", recursive=True)[0]
v = [float(r["Counter_Value"]) for r in csv.DictReader(open(f)) if "fft_" in r["Kernel_Name"]]
print("DIAG", sys.argv[1], "WRITE_SIZE MB per launch", [round(x * 1024 / 1e6, 1) for x in v])
PY
done
