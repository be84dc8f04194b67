#!/bin/bash
# Round 6 call t: wave-owned staging of QSTB's staged half (cf32 8 K ... 32 K one-residue frames and the
# large-N kernel B; RFA_STG_OWNB, A/B build) against base: parity of those paths on the variant, then the
# bench's config-2 / config-4 / config-5 companion lines, interleaved over four rounds.
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/r06t_ab
mkdir -p $O
export TMPDIR=/tmp
RFA_LIB=abv/librfa_ownb.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_state.py \
    -x -q --timeout 120 --timeout-method thread -m gpu -k "f32 or config2 or config5 or 1048576 or large or 262144 or 524288" \
    > $O/pytest_ownb.txt 2>&1 || { echo "pytest rc=$?"; tail -30 $O/pytest_ownb.txt; exit 1; }
echo "ownb: $(tail -1 $O/pytest_ownb.txt)"
B="--steps 2 --warmup 1 --f32-steps 0 --c5-steps 10 --c2-steps 10 --c4-steps 4 --demod-steps 0 --host-fed-calls 0 --cpu-seconds 0"
for i in 1 2 3 4; do
  for v in base ownb; do
    RFA_LIB=abv/librfa_$v.so timeout -k 10 240 python bench.py $B > $O/${v}_$i.json 2> $O/${v}_$i.err || { echo "$v rc=$?"; tail -3 $O/${v}_$i.err; exit 1; }
    python3 - $O/${v}_$i.json ${v}_$i <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
c2, c5, c4 = d["config2"], d["config5"], d.get("config4_f32", {})
print(f"{sys.argv[2]:>8}: config2 {c2['value']:9.0f} ({c2['kernel_ms']*1e3:6.1f} us)  config5 {c5['value']:9.0f} ({c5['kernel_ms']*1e3:6.1f} us)  config4_f32 {c4.get('value', 0):9.0f}")
PY
  done
done
exit 0
