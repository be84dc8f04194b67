#!/bin/bash
# Round-3 A/B: interleaved cf32 at 8 K / 16 K / 32 K with the first half of the next frame staged by LDS-DMA
# after exchange 1 (RFA_QSTAGE_H, fft_wide.hip QSTB) vs direct loads; parity of the qh1 build, then
# three interleaved kbench rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
RFA_LIB=alt/librfa_qh1.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_state.py tests/test_gpu_jni.py -m gpu -x -q \
    --timeout 120 --timeout-method thread -p no:cacheprovider -k "f32 or 8192 or 16384 or 32768 or config" \
    > gpurun_out/qh_parity.log 2>&1
rc=$?; echo "parity rc=$rc"; tail -1 gpurun_out/qh_parity.log; [ $rc -ne 0 ] && exit $rc
V=()
for rnd in 1 2 3; do
  for v in qh0 qh1; do V+=("${v}_$rnd|RFA_LIB=alt/librfa_$v.so"); done
done
bash scripts/ab_kbench.sh gpurun_out/qstage_h_ab.txt "--sizes 8192,16384,32768 --formats f32 --samples 33554432" "${V[@]}"
