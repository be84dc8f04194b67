#!/bin/bash
# Round 6 call g: wave-owned staging of the 64 K 8-bit frame halves (RFA_STG_OWN: each wave stages
# the samples its own threads read, so the item-start wait has no barrier) and the item-start wait
# that leaves the 8 ring tile stores in flight (RFA_STG_W8), A/B builds against base: parity of
# the 64 K paths on each variant, then bench lines interleaved over three rounds.
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/r06g_ab
mkdir -p $O
export TMPDIR=/tmp
for v in own ownw8 w8; do
  RFA_LIB=abv/librfa_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_state.py \
      tests/test_gpu_properties.py -x -q --timeout 120 --timeout-method thread -m gpu > $O/pytest_$v.txt 2>&1 \
      || { echo "pytest $v rc=$?"; tail -30 $O/pytest_$v.txt; exit 1; }
  echo "$v: $(tail -1 $O/pytest_$v.txt)"
done
B="--steps 10 --warmup 2 --f32-steps 0 --c5-steps 0 --c2-steps 0 --c4-steps 0 --demod-steps 0 --host-fed-calls 0 --cpu-seconds 0"
run() {
  local tag=$1 lib=$2
  RFA_LIB=abv/librfa_$lib.so timeout -k 10 120 python bench.py $B > $O/$tag.json 2> $O/$tag.err || { echo "$tag rc=$?"; tail -3 $O/$tag.err; exit 1; }
  python3 - $O/$tag.json $tag <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]
print(f"{sys.argv[2]:>10}: {d['value']:9.0f} Msps  {d['ms_per_step']:7.3f} ms/step  kernel {r['alg_bytes_per_launch']/r['achieved']/1e3:6.1f} us")
PY
}
for i in 1 2 3; do
  for v in base w8 own ownw8; do run ${v}_$i $v; done
done
exit 0
