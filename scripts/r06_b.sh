#!/bin/bash
# Round 6 call b: parity vs the exact-twiddle pffft (configs 2-5), and the state-load cache-policy A/B
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/r06b
mkdir -p $O
export TMPDIR=/tmp
B="--steps 10 --warmup 2 --f32-steps 0 --c5-steps 0 --c2-steps 0 --c4-steps 0 --demod-steps 0 --host-fed-calls 0 --cpu-seconds 0"
for i in 1 2; do
  for v in base stnt; do
    RFA_LIB=abv/librfa_$v.so timeout -k 10 120 python bench.py $B > $O/bench_${v}_$i.json 2> $O/bench_${v}_$i.err || { echo "bench $v rc=$?"; exit 1; }
    python - $O/bench_${v}_$i.json $v <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(f"{sys.argv[2]:>6}: {d['value']:.0f} Msps  {d['ms_per_step']:.3f} ms/step  kernel {d['roofline']['achieved']:.0f} GB/s")
PY
  done
done
RFA_LIB=abv/librfa_stnt.so timeout -k 10 120 python bench.py $B --state-cus 32 > $O/bench_stnt_pipe32.json 2>&1 && tail -c 300 $O/bench_stnt_pipe32.json | head -c 300; echo
timeout -k 10 1200 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -k "no_worse" \
    > $O/pytest_no_worse.txt 2>&1; echo "pytest rc=$?"; grep -E "passed|failed|exact|seed" $O/pytest_no_worse.txt | tail -40
exit 0
