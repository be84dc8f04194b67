#!/bin/bash
# Round-4 probes, same call: LDS-DMA staging on / off at 8 K .. 32 K s8 (A/B build, RFA_STAGE),
# SQ counters of the 8 K s8 kernel at config 4's shape, and FETCH / WRITE of the 64 K cf32 kernel
# (500 frames + state, per launch).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${1:-r04m}
export TMPDIR=/tmp RFA_W64_FORMATS=0
V=()
for rnd in 1 2 3; do V+=("stg_$rnd|RFA_LIB=alt/librfa_ab4.so" "nostg_$rnd|RFA_LIB=alt/librfa_ab4.so RFA_STAGE=0"); done
bash scripts/ab_kbench.sh gpurun_out/stage_ab_$TAG.txt "--sizes 8192,16384,32768 --formats s8" "${V[@]}" || exit $?
bash scripts/pmc_breakdown.sh ${TAG}_8k "--sizes 8192 --formats s8 --samples 33554432" > gpurun_out/sq8k_$TAG.txt 2>&1
rc=$?; echo "sq8k rc=$rc"; tail -1 gpurun_out/sq8k_$TAG.txt; [ $rc -ne 0 ] && exit $rc
for c in FETCH_SIZE WRITE_SIZE; do
  rm -rf gpurun_out/pmcf32_${c}_$TAG
  timeout -s KILL 90 rocprofv3 --pmc $c --output-format csv -d gpurun_out/pmcf32_${c}_$TAG -o p -- \
      python3 scripts/kbench.py --iters 3 --sizes 65536 --formats f32 --samples 32768000 --state > gpurun_out/pmcf32_${c}_$TAG.log 2>&1 || { echo "pmc $c failed"; exit 1; }
done
F=$(find gpurun_out/pmcf32_FETCH_SIZE_$TAG -name "*counter_collection.csv" | head -1)
W=$(find gpurun_out/pmcf32_WRITE_SIZE_$TAG -name "*counter_collection.csv" | head -1)
python3 scripts/pmc_summary.py "$F" "$W" f32_65536_500 fft_wide_kernel gpurun_out/pmc_f32_$TAG.json "profiles/$TAG"
