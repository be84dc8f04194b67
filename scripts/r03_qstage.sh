#!/bin/bash
# Round-3 A/B: 64 K interleaved cf32 with the next frame's first quarter of each half staged by
# LDS-DMA after exchange 1 (RFA_QSTAGE, fft_wide.hip QST) vs direct loads only; parity of the
# in-tree build (GPU parity + state suites), then three interleaved kbench rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_state.py tests/test_gpu_jni.py -m gpu -x -q \
    --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/qs_parity.log 2>&1
rc=$?; echo "parity rc=$rc"; tail -1 gpurun_out/qs_parity.log; [ $rc -ne 0 ] && exit $rc
V=()
for rnd in 1 2 3; do
  for v in qs0 qs1; do V+=("${v}_$rnd|RFA_LIB=alt/librfa_$v.so"); done
done
bash scripts/ab_kbench.sh gpurun_out/qstage_ab.txt "--sizes 65536 --formats f32,s8 --samples 32768000 --state" "${V[@]}"
