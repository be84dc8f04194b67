#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for d in 0 1 2 3 4 8 12 16 19 31; do echo "== DIAG $d"; RFA_DIAG=$d timeout -k 10 120 python scripts/kbench.py --sizes 16384 --formats s8 --iters 20 2>&1 | grep -v amdgpu.ids || exit 1; done
echo "== persist 2"; RFA_PERSIST=2 timeout -k 10 120 python scripts/kbench.py --sizes 16384,65536 --formats s8 --iters 20 2>&1 | grep -v amdgpu.ids || exit 1
echo "== persist 2 stagger 3000"; RFA_PERSIST=2 RFA_STAGGER_NS=3000 timeout -k 10 120 python scripts/kbench.py --sizes 16384 --formats s8 --iters 20 2>&1 | grep -v amdgpu.ids || exit 1
