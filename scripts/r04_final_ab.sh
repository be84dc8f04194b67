#!/bin/bash
# Round-4 final A/B, same call: head (before the round-4 kernel changes) vs this tree, kernel and
# step at 8 K .. 64 K, the 64 K headline workload (500 frames + state), config 4, the GPU suite.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${1:-r04l}
export TMPDIR=/tmp
V=()
for rnd in 1 2 3; do V+=("head_$rnd|RFA_LIB=alt/librfa_head.so" "new_$rnd|"); done
bash scripts/ab_kbench.sh gpurun_out/final_ab_$TAG.txt "--sizes 8192,16384,32768,65536 --formats s8,f32" "${V[@]}" || exit $?
bash scripts/ab_kbench.sh gpurun_out/final_ab_state_$TAG.txt "--sizes 65536 --formats s8,f32 --samples 32768000 --state" "${V[@]}" || exit $?
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_gpu_$TAG.log; [ $rc -ne 0 ] && exit $rc
NOC="--cpu-seconds 0 --f32-steps 0 --c5-steps 0 --c2-steps 0 --c4-steps 0 --demod-steps 0"
for rnd in 1 2; do for v in "head|alt/librfa_head.so" "new|"; do
  l=${v%%|*}; lib=${v#*|}
  RFA_LIB=$lib timeout -k 10 300 python bench.py --mode shard $NOC > gpurun_out/shard_${l}_$TAG.json 2> gpurun_out/shard_${l}_$TAG.err || exit $?
  python3 -c "import json;d=json.load(open('gpurun_out/shard_${l}_$TAG.json'));print('shard $l', d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'])"
  RFA_LIB=$lib timeout -k 10 300 python bench.py $NOC > gpurun_out/bench_${l}_$TAG.json 2> gpurun_out/bench_${l}_$TAG.err || exit $?
  python3 -c "import json;d=json.load(open('gpurun_out/bench_${l}_$TAG.json'));print('bench $l', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'])"
done; done
