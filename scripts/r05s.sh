#!/bin/bash
# Round-5 call s: config-4 SQ record (8 K s8, 64 batches of 256 frames per launch) on the final
# build, plus FETCH / WRITE passes for the same kernel.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
bash scripts/pmc_breakdown.sh r05s_8k "--sizes 8192 --formats s8 --samples 134217728" > gpurun_out/sq_r05s_8k.txt 2>&1 || { tail -5 gpurun_out/sq_r05s_8k.txt; exit 1; }
tail -1 gpurun_out/sq_r05s_8k.txt | cut -c1-300
for c in FETCH_SIZE WRITE_SIZE; do
  rm -rf gpurun_out/pmc_r05s_$c
  timeout -s KILL 90 rocprofv3 --pmc $c --output-format csv -d gpurun_out/pmc_r05s_$c -o p -- python3 scripts/kbench.py --sizes 8192 --formats s8 --samples 134217728 --iters 3 > gpurun_out/pmc_r05s_$c.log 2>&1 || exit 1
done
python3 - <<'PY'
import csv, glob
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    f = sorted(glob.glob(f"gpurun_out/pmc_r05s_{c}/**/*counter_collection.csv", recursive=True))
    v = [float(r["Counter_Value"]) for r in csv.DictReader(open(f[-1])) if "fft_wide_kernel" in r["Kernel_Name"] and r["Counter_Name"] == c]
    v = v[len(v) // 2:]
    print(c, round(sum(v) / len(v) * 1024 / 1e6 * (2 if c == "FETCH_SIZE" else 1), 1), "MB per launch (FETCH doubled per the guide)", len(v))
PY
