#!/bin/bash
# Round-4 A/B, same call: 8 K A-table alias (4 workgroups per CU) and the W_8 sqrt(1/2) fusion.
#   head  = the committed tree before both (alt/librfa_head.so)
#   w8off = alias only (-DRFA_W8_FMA=0, A/B build)
#   new   = alias + W_8 fusion (in-tree librfa.so)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${1:-r04h}
export TMPDIR=/tmp
V=()
for rnd in 1 2 3; do
  V+=("head_$rnd|RFA_LIB=alt/librfa_head.so" "w8off_$rnd|RFA_LIB=alt/librfa_w8off.so RFA_W64_FORMATS=0" "new_$rnd|")
done
bash scripts/ab_kbench.sh gpurun_out/c4_ab_$TAG.txt "--sizes 8192,16384,65536 --formats s8,f32" "${V[@]}" || exit $?
NOC="--cpu-seconds 0 --f32-steps 0 --c5-steps 0 --c2-steps 0 --c4-steps 0 --demod-steps 0"
for v in "head|alt/librfa_head.so" "new|"; do
  l=${v%%|*}; lib=${v#*|}
  RFA_LIB=$lib timeout -k 10 300 python bench.py --mode shard $NOC > gpurun_out/shard_${l}_$TAG.json 2> gpurun_out/shard_${l}_$TAG.err
  rc=$?; echo "shard $l rc=$rc"; python3 -c "import json;d=json.load(open('gpurun_out/shard_${l}_$TAG.json'));print('$l', d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'])"; [ $rc -ne 0 ] && exit $rc
done
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_gpu_$TAG.log
exit $rc
