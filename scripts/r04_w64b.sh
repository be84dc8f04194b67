#!/bin/bash
# Round-4 second call: why the wave-decoupled 64 K kernel is not faster.  Per-wave phase stamps
# (DIAG 32 on the A/B build), SQ counters of the new kernel and of the round-3 kernel, and a
# same-call A/B (round-3 library / new default / two-round exchange 0).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${1:-r04b}
export TMPDIR=/tmp
rm -f gpurun_out/stamps_$TAG.bin
RFA_LIB=alt/librfa_ab.so RFA_STAMPS_FILE=gpurun_out/stamps_$TAG.bin timeout -k 10 120 python -u scripts/kbench.py \
    --sizes 65536 --formats s8 --samples 32768000 --state --iters 2 > gpurun_out/stamps_$TAG.log 2>&1
rc=$?; echo "stamps rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/stamps_$TAG.log; exit $rc; }
python3 scripts/stamps_w64.py gpurun_out/stamps_$TAG.bin > gpurun_out/stamps_$TAG.txt 2>&1; cat gpurun_out/stamps_$TAG.txt
bash scripts/pmc_breakdown.sh ${TAG}_new "--sizes 65536 --formats s8 --samples 32768000 --state" || exit $?
: RFA_LIB=alt/librfa_base.so bash scripts/pmc_breakdown.sh ${TAG}_base "--sizes 65536 --formats s8 --samples 32768000 --state" || exit $?
exit 0
V=()
for rnd in 1 2; do
  V+=("base_$rnd|RFA_LIB=alt/librfa_base.so" "w64x4_$rnd|" "w64x2_$rnd|RFA_LIB=alt/librfa_ab.so RFA_W64_X0R=2")
done
bash scripts/ab_kbench.sh gpurun_out/w64_ab_$TAG.txt "--sizes 65536 --formats s8,f32 --samples 32768000 --state" "${V[@]}"
