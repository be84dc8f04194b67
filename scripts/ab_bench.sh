#!/bin/bash
# Generic same-call A/B of prebuilt A/B libraries (scripts/build_variant.sh NAME -> abv/librfa_NAME.so):
# the 64 K-path parity subset on every variant but `base`, then the bench line (500 x 64 K s8,
# EMA + peak, kernel + state pass) interleaved over ROUNDS rounds.  Kernel us = algorithmic bytes /
# achieved.  usage: scripts/ab_bench.sh OUT "base v1 v2" ROUNDS
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/$1; VARS=$2; ROUNDS=${3:-3}
mkdir -p $O
export TMPDIR=/tmp
for v in $VARS; do
  [ $v = base ] && continue
  RFA_LIB=abv/librfa_$v.so timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_state.py \
      tests/test_gpu_properties.py -x -q --timeout 120 --timeout-method thread -m gpu -k "65536 or config3 or 64k" \
      > $O/pytest_$v.txt 2>&1 || { echo "pytest $v rc=$?"; tail -30 $O/pytest_$v.txt; exit 1; }
  echo "$v: $(tail -1 $O/pytest_$v.txt)"
done
B="--steps 10 --warmup 2 --f32-steps 0 --c5-steps 0 --c2-steps 0 --c4-steps 0 --demod-steps 0 --host-fed-calls 0 --cpu-seconds 0"
for i in $(seq 1 $ROUNDS); do
  for v in $VARS; do
    RFA_LIB=abv/librfa_$v.so timeout -k 10 120 python bench.py $B > $O/${v}_$i.json 2> $O/${v}_$i.err || { echo "$v rc=$?"; tail -3 $O/${v}_$i.err; exit 1; }
    python3 - $O/${v}_$i.json ${v}_$i <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]
print(f"{sys.argv[2]:>12}: {d['value']:9.0f} Msps  {d['ms_per_step']:7.3f} ms/step  kernel {r['alg_bytes_per_launch']/r['achieved']/1e3:6.1f} us")
PY
  done
done
exit 0
