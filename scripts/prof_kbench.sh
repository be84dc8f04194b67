#!/bin/bash
# rocprofv3 kernel-trace stats of scripts/kbench.py for one variant.
# usage: scripts/prof_kbench.sh TAG "KBENCH_ARGS" [ENV=v ...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=$1; ARGS=$2; shift 2
mkdir -p gpurun_out
rm -rf "gpurun_out/prof_$TAG"
# shellcheck disable=SC2086
env "$@" timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d "gpurun_out/prof_$TAG" -o run -- \
    python3 scripts/kbench.py $ARGS > "gpurun_out/prof_$TAG.log" 2>&1
rc=$?
echo "== $TAG rc=$rc"; grep -E "N=" "gpurun_out/prof_$TAG.log"
f=$(find "gpurun_out/prof_$TAG" -name "*kernel_stats.csv" | head -1)
[ -n "$f" ] && python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows:
    if "rfa::" in r["Name"] or "anonymous" in r["Name"] and "ddc" in r["Name"]:
        print(f'{float(r["AverageNs"])/1e3:9.1f} us avg  x{r["Calls"]:>5}  {r["Name"][:110]}')
PY
exit $rc
