#!/bin/bash
# Round 6 call r: wave-owned staging of the 64 K cf32 kernel's staged quarters (RFA_STG_OWNQ) read from the
# bench's f32 companion line (64 K f32, 500 frames, EMA + peak; --f32-steps 10), base vs ownq over four rounds
# (kbench's per-process spread hid it in call m).
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/r06r_ab
mkdir -p $O
export TMPDIR=/tmp
B="--steps 4 --warmup 2 --f32-steps 10 --c5-steps 0 --c2-steps 0 --c4-steps 0 --demod-steps 0 --host-fed-calls 0 --cpu-seconds 0"
for i in 1 2 3 4; do
  for v in base ownq; do
    RFA_LIB=abv/librfa_$v.so timeout -k 10 180 python bench.py $B > $O/${v}_$i.json 2> $O/${v}_$i.err || { echo "$v rc=$?"; tail -3 $O/${v}_$i.err; exit 1; }
    python3 - $O/${v}_$i.json ${v}_$i <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
f = d["f32"]
print(f"{sys.argv[2]:>8}: f32 {f['value']:9.0f} Msps  frac {f['roofline_frac']:.4f}  kernel {f['kernel_ms']*1e3:6.1f} us | s8 line {d['value']:9.0f}")
PY
  done
done
exit 0
