#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_dq.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_dq.log; [ $rc -ne 0 ] && exit $rc
for cfg in 1 0 1 0; do
  echo "== DQ=$cfg"; RFA_DQ=$cfg timeout -k 10 120 python scripts/kbench.py --sizes 4096,8192,16384,32768,65536 --formats s8,s16 --iters 20 --samples 32768000 2>&1 | grep -v amdgpu.ids || exit 1
done
for d in 1 0; do echo "== bench DQ=$d"; RFA_DQ=$d timeout -k 10 200 python bench.py --cpu-seconds 0 --steps 20 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])" || exit 1; done
