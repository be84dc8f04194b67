#!/bin/bash
# Round-4 A/B, same call: pass-2 twiddles of the 8 K / 16 K kernels from a direct table in global
# memory (alt/librfa_p2d.so, -DRFA_P2DIRECT=1) against the same tree without it (alt/librfa_ab4.so)
# and head; config 4 on both; parity of the 8 K / 16 K cases through the p2d build.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${1:-r04n}
export TMPDIR=/tmp RFA_W64_FORMATS=0
V=()
for rnd in 1 2 3; do V+=("head_$rnd|RFA_LIB=alt/librfa_head.so" "ab4_$rnd|RFA_LIB=alt/librfa_ab4.so" "p2d_$rnd|RFA_LIB=alt/librfa_p2d.so"); done
bash scripts/ab_kbench.sh gpurun_out/p2d_ab_$TAG.txt "--sizes 8192,16384 --formats s8,f32" "${V[@]}" || exit $?
RFA_LIB=alt/librfa_p2d.so timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread -p no:cacheprovider \
    tests/test_gpu_parity.py -k "8192 or 16384 or hann or fixture or n8192 or n16384" > gpurun_out/pytest_p2d_$TAG.log 2>&1
rc=$?; echo "pytest p2d rc=$rc"; tail -3 gpurun_out/pytest_p2d_$TAG.log; [ $rc -gt 1 ] && exit $rc
NOC="--cpu-seconds 0 --f32-steps 0 --c5-steps 0 --c2-steps 0 --c4-steps 0 --demod-steps 0"
for rnd in 1 2; do for v in "ab4|alt/librfa_ab4.so" "p2d|alt/librfa_p2d.so"; do
  l=${v%%|*}; lib=${v#*|}
  RFA_LIB=$lib timeout -k 10 300 python bench.py --mode shard $NOC > gpurun_out/shard_${l}_$TAG.json 2> gpurun_out/shard_${l}_$TAG.err || exit $?
  python3 -c "import json;d=json.load(open('gpurun_out/shard_${l}_$TAG.json'));print('shard $l', d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'])"
done; done
