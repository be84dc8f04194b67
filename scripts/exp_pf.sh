#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_pf.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_pf.log; [ $rc -ne 0 ] && exit $rc
for p in 1 0 1 0; do echo "== PREFETCH=$p"; RFA_PREFETCH=$p timeout -k 10 120 python scripts/kbench.py --sizes 65536 --formats s8,u8 --iters 20 --samples 32768000 2>&1 | grep -v amdgpu.ids || exit 1; done
for p in 1 0; do echo "== bench PREFETCH=$p"; RFA_PREFETCH=$p timeout -k 10 200 python bench.py --cpu-seconds 0 --steps 20 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])" || exit 1; done
