#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for d in 0 16 64; do echo "== DIAG $d"; RFA_DIAG=$d timeout -k 10 120 python scripts/kbench.py --sizes 65536 --formats s8 --iters 20 --samples 32768000 2>&1 | grep -v amdgpu.ids || exit 1; done
echo "== WIDE_LOGM=14"; RFA_WIDE_LOGM=14 timeout -k 10 120 python scripts/kbench.py --sizes 65536 --formats s8 --iters 20 --samples 32768000 2>&1 | grep -v amdgpu.ids || exit 1
