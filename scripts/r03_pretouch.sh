#!/bin/bash
# Round-3 A/B: L2 pre-touch of the 64 K frame's late half (RFA_PRETOUCH 1 / 2, alt/
# builds from scripts/build_variant.sh) against the same-source base build: parity of
# the config-3 state test on each variant, then three interleaved kbench rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in pt1 pt2; do
  RFA_LIB=alt/librfa_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_state.py tests/test_gpu_parity.py -m gpu -x -q \
      --timeout 120 --timeout-method thread -p no:cacheprovider -k "65536 or config3" > gpurun_out/pt_parity_$v.log 2>&1
  rc=$?; echo "parity $v rc=$rc"; tail -1 gpurun_out/pt_parity_$v.log; [ $rc -ne 0 ] && exit $rc
done
V=()
for rnd in 1 2 3; do
  for v in base pt1 pt2; do V+=("${v}_$rnd|RFA_LIB=alt/librfa_$v.so"); done
done
bash scripts/ab_kbench.sh gpurun_out/pretouch_ab.txt "--sizes 65536 --formats s8,u8 --samples 32768000 --state" "${V[@]}"
