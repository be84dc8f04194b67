#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for lib in default nt default nt; do
  if [ $lib = nt ]; then export RFA_LIB=$PWD/scripts/librfa_nt.so; else unset RFA_LIB; fi
  echo "== $lib"; timeout -k 10 200 python bench.py --cpu-seconds 0 --steps 30 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])" || exit 1
  timeout -k 10 120 python scripts/kbench.py --sizes 16384,65536 --formats s8 --iters 20 --samples 32768000 2>&1 | grep -v amdgpu.ids || exit 1
done
