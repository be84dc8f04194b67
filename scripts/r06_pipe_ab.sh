#!/bin/bash
# Round 6: CU-mask census, pipelined-state tests, and the bench A/B over state CUs
# (rfa_set_pipelined), every GPU step under its own time limit.
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/r06a
mkdir -p $O
export TMPDIR=/tmp
CENSUS_ONLY=1 timeout -k 10 60 ./scripts/ubench_cumask > $O/census.txt 2>&1 || { echo "census rc=$?"; exit 1; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_state.py -x -v --timeout 200 --timeout-method thread -k "pipelined" \
    > $O/pytest_pipelined.txt 2>&1 || { echo "pytest rc=$?"; tail -30 $O/pytest_pipelined.txt; exit 1; }
B="--steps 10 --warmup 2 --f32-steps 0 --c5-steps 0 --c2-steps 0 --c4-steps 0 --demod-steps 0 --host-fed-calls 0 --cpu-seconds 0"
for i in 1 2; do
  for c in 0 16 24 32; do
    timeout -k 10 120 python bench.py $B --state-cus $c > $O/bench_c${c}_$i.json 2> $O/bench_c${c}_$i.err || { echo "bench $c rc=$?"; exit 1; }
    python - $O/bench_c${c}_$i.json $c <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(f"state_cus {sys.argv[2]:>3}: {d['value']:.0f} Msps  {d['ms_per_step']:.3f} ms/step  kernel {d['roofline']['achieved']:.0f} GB/s")
PY
  done
done
cd /tmp && timeout -k 10 180 rocprofv3 --kernel-trace --stats -d /root/repo/$O/prof24 -o run -- python3 /root/repo/bench.py $B --state-cus 24 > /root/repo/$O/prof24.log 2>&1 || echo "rocprof rc=$?"
exit 0
