#!/bin/bash
# Round-4 A/B, same call (A/B builds with RFA_W64_FORMATS=0 so 64 K takes the wide kernel):
#   head   = before the round-4 kernel changes (alt/librfa_head.so)
#   base4  = 8 K A-table alias + the W_8 DFT form for 8/16-bit frames (fft_w8.h)
#   xst    = base4 + exchange stores from one write base per round as single ds_write_b64
#   notail = xst + the lane index opaque per item (A/B build of this tree, RFA_TAIL_STATE=0)
#   new    = notail + the tail-overlapped state update (in-tree librfa.so)
# then the GPU suite, the determinism / alignment check, config 4 and the headline bench line
# (head vs new).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${1:-r04k}
export TMPDIR=/tmp RFA_W64_FORMATS=0
V=()
for rnd in 1 2 3; do
  V+=("head_$rnd|RFA_LIB=alt/librfa_head.so" "base4_$rnd|RFA_LIB=alt/librfa_base4.so RFA_TAIL_STATE=0"
      "xst_$rnd|RFA_LIB=alt/librfa_xst.so RFA_TAIL_STATE=0" "notail_$rnd|RFA_LIB=alt/librfa_tail.so RFA_TAIL_STATE=0" "new_$rnd|")
done
bash scripts/ab_kbench.sh gpurun_out/vadd2_ab_$TAG.txt "--sizes 8192,16384,32768,65536 --formats s8,f32" "${V[@]}" || exit $?
bash scripts/ab_kbench.sh gpurun_out/tail_ab_$TAG.txt "--sizes 65536 --formats s8,f32 --samples 32768000 --state" "${V[@]}" || exit $?
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_gpu_$TAG.log; [ $rc -gt 1 ] && exit $rc
timeout -k 10 120 python -u scripts/determinism_check.py 1048576 32768 65536 2>&1 | grep -v amdgpu.ids | tee gpurun_out/determinism_$TAG.txt
NOC="--cpu-seconds 0 --f32-steps 0 --c5-steps 0 --c2-steps 0 --c4-steps 0 --demod-steps 0"
for v in "head|alt/librfa_head.so" "new|"; do
  l=${v%%|*}; lib=${v#*|}
  RFA_LIB=$lib timeout -k 10 300 python bench.py --mode shard $NOC > gpurun_out/shard_${l}_$TAG.json 2> gpurun_out/shard_${l}_$TAG.err
  rc=$?; echo "shard $l rc=$rc"; [ $rc -ne 0 ] && exit $rc
  python3 -c "import json;d=json.load(open('gpurun_out/shard_${l}_$TAG.json'));print('shard $l', d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'])"
  RFA_LIB=$lib timeout -k 10 300 python bench.py $NOC > gpurun_out/bench_${l}_$TAG.json 2> gpurun_out/bench_${l}_$TAG.err
  rc=$?; echo "bench $l rc=$rc"; [ $rc -ne 0 ] && exit $rc
  python3 -c "import json;d=json.load(open('gpurun_out/bench_${l}_$TAG.json'));print('bench $l', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'])"
done
