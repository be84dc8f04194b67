#!/bin/bash
# Round-3 A/B: large-N kernel B with the first half of its next item's z_s staged by LDS-DMA after
# exchange 1 (RFA_QSTAGE_B, fft_wide.hip QSTB; persistent grid) vs direct loads; parity of the
# in-tree build on the large-N tests, then three interleaved kbench rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_state.py tests/test_gpu_jni.py -m gpu -x -q \
    --timeout 120 --timeout-method thread -p no:cacheprovider -k "large or 262144 or 524288 or 1048576 or column" \
    > gpurun_out/qb_parity.log 2>&1
rc=$?; echo "parity rc=$rc"; tail -1 gpurun_out/qb_parity.log; [ $rc -ne 0 ] && exit $rc
V=()
for rnd in 1 2 3; do
  for v in qb0 qb1; do V+=("${v}_$rnd|RFA_LIB=alt/librfa_$v.so"); done
done
bash scripts/ab_kbench.sh gpurun_out/qstage_b_ab.txt "--sizes 262144,524288,1048576 --formats s8,f32 --samples 16777216 --state" "${V[@]}"
