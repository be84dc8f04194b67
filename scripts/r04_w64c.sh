#!/bin/bash
# Round-4 third call: the balanced exchange 0 (fft_w64.hip exchange0_bal).  GPU suite, same-call
# A/B against the round-3 library and the writer-wave exchange forms (RFA_W64_X0R=3: four
# rounds through A, =2: two rounds through A + B; A/B build), per-wave phase stamps.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${1:-r04d}
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/pytest_gpu_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_gpu_$TAG.log; [ $rc -ne 0 ] && exit $rc
V=()
for rnd in 1 2; do
  V+=("base_$rnd|RFA_LIB=alt/librfa_base.so" "bal_$rnd|" "x0r3_$rnd|RFA_LIB=alt/librfa_ab.so RFA_W64_X0R=3" "x0r2_$rnd|RFA_LIB=alt/librfa_ab.so RFA_W64_X0R=2")
done
bash scripts/ab_kbench.sh gpurun_out/w64_ab_$TAG.txt "--sizes 65536 --formats s8,f32 --samples 32768000 --state" "${V[@]}" || exit $?
rm -f gpurun_out/stamps_$TAG.bin
RFA_LIB=alt/librfa_ab.so RFA_STAMPS_FILE=gpurun_out/stamps_$TAG.bin timeout -k 10 120 python -u scripts/kbench.py \
    --sizes 65536 --formats s8 --samples 32768000 --state --iters 2 > gpurun_out/stamps_$TAG.log 2>&1
rc=$?; echo "stamps rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/stamps_$TAG.log; exit $rc; }
python3 scripts/stamps_w64.py gpurun_out/stamps_$TAG.bin > gpurun_out/stamps_$TAG.txt 2>&1; cat gpurun_out/stamps_$TAG.txt
