#!/bin/bash
# Round-end evidence of the final tree in ONE GPU call: round_evidence.sh (GPU
# suite, smoke, bench + rocprof stats + FETCH/WRITE PMC passes, kbench sweep),
# the SQ counter breakdown of the 64 K kernel (VALU busy / wave wait for
# profiles/sq_valu.json), and the config-4 shard mode on one GPU.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${1:-r02e}
bash scripts/round_evidence.sh $TAG || exit $?
bash scripts/pmc_breakdown.sh $TAG "--sizes 65536 --formats s8 --samples 32768000 --state" > gpurun_out/sq_$TAG.txt 2>&1
rc=$?; echo "sq rc=$rc"; tail -2 gpurun_out/sq_$TAG.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --mode shard --cpu-seconds 0 --f32-steps 0 --c5-steps 0 --demod-steps 0 \
    > gpurun_out/bench_shard_$TAG.json 2> gpurun_out/bench_shard_$TAG.err
rc=$?; echo "shard rc=$rc"; cat gpurun_out/bench_shard_$TAG.json; exit $rc
