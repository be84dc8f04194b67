#!/bin/bash
# Round 6 call f: the state pass co-resident beside the FFT (no CU masks): FFT compiled for 5 waves
# per SIMD (96 VGPRs, RFA_WIDE_WPE=5) so a state wave fits beside its workgroup on every CU; the state
# pass as partial + combine kernels (no LDS); pipelined ring flip; FFT streams at high priority.
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/r06f
mkdir -p $O
export TMPDIR=/tmp
B="--steps 10 --warmup 2 --f32-steps 0 --c5-steps 0 --c2-steps 0 --c4-steps 0 --demod-steps 0 --host-fed-calls 0 --cpu-seconds 0"
run() {  # tag lib extra-env... -- bench args
  local tag=$1 lib=$2; shift 2
  env RFA_LIB=abv/librfa_$lib.so "$@" timeout -k 10 120 python bench.py $B $PIPE > $O/$tag.json 2> $O/$tag.err || { echo "$tag rc=$?"; tail -3 $O/$tag.err; exit 1; }
  python3 - $O/$tag.json $tag <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(f"{sys.argv[2]:>22}: {d['value']:9.0f} Msps  {d['ms_per_step']:7.3f} ms/step")
PY
}
for i in 1 2; do
  PIPE="" run base_serial_$i base
  PIPE="" run wpe5_serial_$i wpe5
  PIPE="--state-cus 8" run wpe5_nomask_fused_$i wpe5 RFA_PIPE_NOMASK=1
  PIPE="--state-cus 8" run wpe5_nomask_split_$i wpe5 RFA_PIPE_NOMASK=1 RFA_STATE_FUSED=0
  PIPE="--state-cus 8" run base_nomask_split_$i base RFA_PIPE_NOMASK=1 RFA_STATE_FUSED=0
done
cd /tmp && RFA_LIB=/root/repo/abv/librfa_wpe5.so RFA_PIPE_NOMASK=1 RFA_STATE_FUSED=0 timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv \
    -d /root/repo/$O/prof -o run -- python3 /root/repo/bench.py $B --state-cus 8 > /root/repo/$O/prof.log 2>&1 || echo "rocprof rc=$?"
exit 0
