#!/bin/bash
# Round 6 call o: the round's 64 K kernel changes end to end, same call: the product library before
# them (commit b3477ce), after the wave-owned staging (203fe6f) and the final product (in-tree), bench
# line (500 x 64 K s8, EMA + peak) interleaved over five rounds.
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/r06o_ab
mkdir -p $O
export TMPDIR=/tmp
B="--steps 10 --warmup 2 --f32-steps 0 --c5-steps 0 --c2-steps 0 --c4-steps 0 --demod-steps 0 --host-fed-calls 0 --cpu-seconds 0"
for i in 1 2 3 4 5; do
  for v in b3477ce 203fe6f final; do
    L=abv/librfa_$v.so; [ $v = final ] && L=rfanalyzer_amd/librfa.so
    RFA_LIB=$L timeout -k 10 120 python bench.py $B > $O/${v}_$i.json 2> $O/${v}_$i.err || { echo "$v rc=$?"; tail -3 $O/${v}_$i.err; exit 1; }
    python3 - $O/${v}_$i.json ${v}_$i <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]
print(f"{sys.argv[2]:>10}: {d['value']:9.0f} Msps  {d['ms_per_step']:7.3f} ms/step  kernel {r['alg_bytes_per_launch']/r['achieved']/1e3:6.1f} us")
PY
  done
done
exit 0
