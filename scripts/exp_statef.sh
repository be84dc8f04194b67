#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_sf.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_sf.log; [ $rc -ne 0 ] && exit $rc
for f in 1 0; do for c in 8 16 32; do echo "== fused $f chunks $c"; RFA_STATE_FUSED=$f RFA_STATE_CHUNKS=$c timeout -k 10 200 python bench.py --cpu-seconds 0 --steps 20 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])" || exit 1; done; done
