#!/bin/bash
# Round-4 last call: one-residue 8-bit frames unstaged (this tree) against the evidenced build
# (alt/librfa_prev.so, librfa 2ca174cf), kernel and config 4; then the round evidence of this tree.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${1:-r04z}
export TMPDIR=/tmp
V=()
for rnd in 1 2 3; do V+=("prev_$rnd|RFA_LIB=alt/librfa_prev.so" "new_$rnd|"); done
bash scripts/ab_kbench.sh gpurun_out/unstage_ab_$TAG.txt "--sizes 8192,16384,32768,65536 --formats s8,u8" "${V[@]}" || exit $?
NOC="--cpu-seconds 0 --f32-steps 0 --c5-steps 0 --c2-steps 0 --c4-steps 0 --demod-steps 0"
for rnd in 1 2; do for v in "prev|alt/librfa_prev.so" "new|"; do
  l=${v%%|*}; lib=${v#*|}
  RFA_LIB=$lib timeout -k 10 300 python bench.py --mode shard $NOC > gpurun_out/shard_${l}_$TAG.json 2> gpurun_out/shard_${l}_$TAG.err || exit $?
  python3 -c "import json;d=json.load(open('gpurun_out/shard_${l}_$TAG.json'));print('shard $l', d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'])" | tee -a gpurun_out/unstage_ab_$TAG.txt
done; done
bash scripts/r04_evidence.sh $TAG
