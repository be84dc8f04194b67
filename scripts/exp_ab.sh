#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for c in 8 16 4; do echo "== default lib, state chunks $c"; RFA_STATE_CHUNKS=$c timeout -k 10 120 python scripts/kbench.py --sizes 65536 --formats s8 --state || exit $?; done
echo "== PRE_DIST=2"; RFA_LIB=$PWD/scripts/librfa_d2.so timeout -k 10 200 python scripts/kbench.py --sizes 32768,65536,131072 --formats s8,s16,f32 || exit $?
echo "== PRE_DIST=1"; timeout -k 10 200 python scripts/kbench.py --sizes 32768,65536,131072 --formats s8,s16,f32 || exit $?
