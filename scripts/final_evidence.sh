#!/bin/bash
# Round-end evidence of the final tree in ONE GPU call: round_evidence.sh (GPU
# suite, smoke, bench + rocprof stats + FETCH/WRITE PMC passes, kbench sweep),
# the SQ counter breakdown of the 64 K kernel (VALU busy / wave wait for
# profiles/sq_valu.json), and the config-4 shard mode on one GPU.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${1:-r03a}
bash scripts/round_evidence.sh $TAG || exit $?
bash scripts/pmc_breakdown.sh $TAG "--sizes 65536 --formats s8 --samples 32768000 --state" > gpurun_out/sq_$TAG.txt 2>&1
rc=$?; echo "sq rc=$rc"; tail -2 gpurun_out/sq_$TAG.txt; [ $rc -ne 0 ] && exit $rc
NOC="--cpu-seconds 0 --f32-steps 0 --c5-steps 0 --c2-steps 0 --c4-steps 0 --demod-steps 0"
timeout -k 10 300 python bench.py --mode shard $NOC > gpurun_out/bench_shard_$TAG.json 2> gpurun_out/bench_shard_$TAG.err
rc=$?; echo "shard rc=$rc"; cat gpurun_out/bench_shard_$TAG.json; [ $rc -ne 0 ] && exit $rc
# config 4 (256 x 8192 s8 batches, 64 per rfa_process_batches call): kernel split of the same command
rm -rf gpurun_out/prof_shard_$TAG
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_shard_$TAG -o run -- \
    python3 bench.py --mode shard $NOC --steps 10 > gpurun_out/prof_shard_$TAG.log 2>&1
rc=$?; echo "shard rocprof rc=$rc"; find gpurun_out/prof_shard_$TAG -name "*kernel_stats.csv" -exec cat {} \;
exit $rc
