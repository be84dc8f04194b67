#!/bin/bash
# Round-3 A/B: residue-1 pre-stage as interleaved cmac2 pairs (RFA_CMAC2X2; hipcc padded each link
# of a single chain with s_nop 0) on top of the pre-stage LDS base; xb_none = the tree before both.
# Parity of the default build, then three interleaved rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_state.py -m gpu -x -q \
    --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/cm_parity.log 2>&1
rc=$?; echo "parity rc=$rc"; tail -1 gpurun_out/cm_parity.log; [ $rc -ne 0 ] && exit $rc
V=()
for rnd in 1 2 3; do
  for v in xb_none cm0 cm1; do V+=("${v}_$rnd|RFA_LIB=alt/librfa_$v.so"); done
done
bash scripts/ab_kbench.sh gpurun_out/cmac_ab.txt "--sizes 65536 --formats s8,u8 --samples 32768000 --state" "${V[@]}"
