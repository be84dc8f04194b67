#!/bin/bash
# Round evidence on one GPU: default bench line (with cpu_baseline), rocprofv3
# kernel-trace stats of the same command, and two separate PMC passes
# (FETCH_SIZE, WRITE_SIZE) for the HBM traffic of the main kernel.
# usage: scripts/profile_round.sh TAG [extra bench args]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r01}; shift || true
EXTRA="$*"
fatal() { [ "$1" -ne 0 ]; }
timeout -k 10 420 python bench.py $EXTRA > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench_$TAG.json; tail -3 gpurun_out/bench_$TAG.err; fatal $rc && exit $rc
rm -rf gpurun_out/prof_$TAG gpurun_out/pmcf_$TAG gpurun_out/pmcw_$TAG
timeout -k 10 420 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- \
    python3 bench.py --cpu-seconds 0 --f32-steps 0 --c5-steps 0 --c2-steps 0 --c4-steps 0 --demod-steps 0 $EXTRA > gpurun_out/prof_$TAG.log 2>&1
rc=$?; echo "rocprof stats rc=$rc"; fatal $rc && { tail -5 gpurun_out/prof_$TAG.log; exit $rc; }
find gpurun_out/prof_$TAG -name "*kernel_stats.csv" -exec cat {} \;
SHORT="--cpu-seconds 0 --f32-steps 0 --c5-steps 0 --c2-steps 0 --c4-steps 0 --demod-steps 0 --steps 2 --warmup 1 --calls-per-step 4"
timeout -k 10 420 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmcf_$TAG -o run -- \
    python3 bench.py $SHORT $EXTRA > gpurun_out/pmcf_$TAG.log 2>&1
rc=$?; echo "pmc fetch rc=$rc"; fatal $rc && { tail -5 gpurun_out/pmcf_$TAG.log; exit $rc; }
timeout -k 10 420 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmcw_$TAG -o run -- \
    python3 bench.py $SHORT $EXTRA > gpurun_out/pmcw_$TAG.log 2>&1
rc=$?; echo "pmc write rc=$rc"; fatal $rc && { tail -5 gpurun_out/pmcw_$TAG.log; exit $rc; }
F=$(find gpurun_out/pmcf_$TAG -name "*counter_collection.csv" | head -1)
W=$(find gpurun_out/pmcw_$TAG -name "*counter_collection.csv" | head -1)
python3 scripts/pmc_summary.py "$F" "$W" s8_65536_500 fft_wide_kernel gpurun_out/pmc_traffic_$TAG.json "profiles/$TAG" || true
exit 0
