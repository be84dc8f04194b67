#!/bin/bash
# Round-3 A/B: LDS address bases (RFA_XBASE: per-round exchange write base; RFA_XBASE_PRE:
# own base for the staged second half in the pre-stage), alt/ builds, parity on the
# full variant, three interleaved rounds over the configs' kernels.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in xb_pre xb_all; do
  RFA_LIB=alt/librfa_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_state.py -m gpu -x -q \
      --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/xb_parity_$v.log 2>&1
  rc=$?; echo "parity $v rc=$rc"; tail -1 gpurun_out/xb_parity_$v.log; [ $rc -ne 0 ] && exit $rc
done
V=()
for rnd in 1 2 3; do
  for v in xb_none xb_pre xb_all; do V+=("${v}_$rnd|RFA_LIB=alt/librfa_$v.so"); done
done
bash scripts/ab_kbench.sh gpurun_out/xbase_ab.txt "--sizes 8192,16384,65536 --formats s8,f32 --samples 32768000" "${V[@]}"
