#!/bin/bash
# Round-3 A/B: the 64 K residue-1 complex window (twiddle folded into the window, fft_wide.hip
# prestage CW) for interleaved cf32 input too (RFA_CWIN_FMT=3; 28 B of spills in that instance):
# parity of the cwf3 build on the f32 fixtures and config-3 state, three interleaved kbench rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
RFA_LIB=alt/librfa_cwf3.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_state.py -m gpu -x -q \
    --timeout 120 --timeout-method thread -p no:cacheprovider -k "f32 or 65536 or config3" > gpurun_out/cwf_parity.log 2>&1
rc=$?; echo "parity rc=$rc"; tail -4 gpurun_out/cwf_parity.log; [ $rc -ne 0 ] && exit $rc
V=()
for rnd in 1 2 3; do
  for v in cwf2 cwf3; do V+=("${v}_$rnd|RFA_LIB=alt/librfa_$v.so"); done
done
bash scripts/ab_kbench.sh gpurun_out/cw_f32_ab.txt "--sizes 65536 --formats f32 --samples 32768000 --state" "${V[@]}"
# second A/B in the same call: per-round exchange write base in the 16 K kernel only (RFA_XBASE16)
RFA_LIB=alt/librfa_xb16.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q \
    --timeout 120 --timeout-method thread -p no:cacheprovider -k "16384" > gpurun_out/xb16_parity.log 2>&1
rc=$?; echo "parity xb16 rc=$rc"; tail -1 gpurun_out/xb16_parity.log; [ $rc -ne 0 ] && exit $rc
V=()
for rnd in 1 2 3; do
  for v in cwf2 xb16; do V+=("${v}_$rnd|RFA_LIB=alt/librfa_$v.so"); done
done
bash scripts/ab_kbench.sh gpurun_out/xb16_ab.txt "--sizes 16384 --formats f32,s8 --samples 67108864" "${V[@]}"
