#!/bin/bash
# Round 6 call l: wave-owned staging for the one-residue 8/16-bit kernels (RFA_STG_OWN1, 8 K ... 32 K),
# A/B build against base: parity of those sizes on the variant, then kbench (s8 / u8 / s16, 8 K, 16 K,
# 32 K, 32.8 M samples per launch) and the config-4 bench companion, interleaved over three rounds.
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/r06l_ab
mkdir -p $O
export TMPDIR=/tmp
RFA_LIB=abv/librfa_own1.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_state.py \
    tests/test_gpu_framing.py -x -q --timeout 120 --timeout-method thread -m gpu -k "8192 or 16384 or 32768 or config4 or config2 or 1024" \
    > $O/pytest_own1.txt 2>&1 || { echo "pytest rc=$?"; tail -30 $O/pytest_own1.txt; exit 1; }
echo "own1: $(tail -1 $O/pytest_own1.txt)"
V=()
for i in 1 2 3; do V+=("base$i|RFA_LIB=abv/librfa_base.so" "own1_$i|RFA_LIB=abv/librfa_own1.so"); done
bash scripts/ab_kbench.sh $O/kbench.txt "--sizes 8192,16384,32768 --formats s8,u8,s16 --samples 32768000 --iters 30" "${V[@]}" > /dev/null || exit 1
grep -E "^==|N=" $O/kbench.txt
B="--steps 10 --warmup 2 --f32-steps 0 --c5-steps 0 --c2-steps 0 --demod-steps 0 --host-fed-calls 0 --cpu-seconds 0"
for i in 1 2 3; do
  for v in base own1; do
    RFA_LIB=abv/librfa_$v.so timeout -k 10 180 python bench.py $B > $O/c4_${v}_$i.json 2> $O/c4_${v}_$i.err || { echo "c4 $v rc=$?"; tail -3 $O/c4_${v}_$i.err; exit 1; }
    python3 - $O/c4_${v}_$i.json ${v}_$i <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
c = d["config4"]
print(f"config4 {sys.argv[2]:>8}: {c['value']:9.0f} Msps  frac {c['roofline_frac']:.4f}  (bench line {d['value']:9.0f})")
PY
  done
done
exit 0
