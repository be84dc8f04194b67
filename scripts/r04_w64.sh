#!/bin/bash
# Round-4 first call: the wave-decoupled 64 K kernel (fft_w64.hip).  GPU suite on the new
# library, then a same-call A/B of the kernel against the round-3 library (alt/librfa_base.so,
# built from the round-3 commit) and the two-round exchange-0 form (RFA_W64_X0R=2 on the A/B
# build), two interleaved rounds, then rocprof kernel stats of the new kernel.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${1:-r04a}
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/pytest_gpu_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -6 gpurun_out/pytest_gpu_$TAG.log; [ $rc -ne 0 ] && exit $rc
V=()
for rnd in 1 2; do
  V+=("base_$rnd|RFA_LIB=alt/librfa_base.so" "w64x4_$rnd|" "w64x2_$rnd|RFA_LIB=alt/librfa_ab.so RFA_W64_X0R=2")
done
bash scripts/ab_kbench.sh gpurun_out/w64_ab_$TAG.txt "--sizes 65536 --formats s8,u8,f32 --samples 32768000 --state" "${V[@]}" \
    || exit $?
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o k -- \
    python -u scripts/kbench.py --sizes 65536 --formats s8,f32 --samples 32768000 --state --iters 10 \
    > gpurun_out/prof_$TAG.log 2>&1
rc=$?; echo "rocprof rc=$rc"; find gpurun_out/prof_$TAG -name "*kernel_stats.csv" | head -2
