#!/bin/bash
# Round-4 A/B, same call: 64 K / 128 K residues rotated by the round (alt/librfa_rot.so,
# -DRFA_RES_ROTATE=1: every persistent workgroup alternates the residue-0 / residue-1 pre-stages)
# against the same tree (alt/librfa_ab6.so); headline bench line of both; parity through rot.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${1:-r04w}
export TMPDIR=/tmp RFA_W64_FORMATS=0
V=()
for rnd in 1 2 3; do V+=("ab6_$rnd|RFA_LIB=alt/librfa_ab6.so" "rot_$rnd|RFA_LIB=alt/librfa_rot.so"); done
bash scripts/ab_kbench.sh gpurun_out/rot_ab_$TAG.txt "--sizes 65536,131072 --formats s8,f32 --samples 32768000 --state" "${V[@]}" || exit $?
bash scripts/ab_kbench.sh gpurun_out/rot_ab_nostate_$TAG.txt "--sizes 65536 --formats s8,f32" "${V[@]}" || exit $?
NOC="--cpu-seconds 0 --f32-steps 0 --c5-steps 0 --c2-steps 0 --c4-steps 0 --demod-steps 0"
for rnd in 1 2; do for v in ab6 rot; do
  RFA_LIB=alt/librfa_$v.so timeout -k 10 300 python bench.py $NOC > gpurun_out/bench_${v}_$TAG.json 2> gpurun_out/bench_${v}_$TAG.err || exit $?
  python3 -c "import json;d=json.load(open('gpurun_out/bench_${v}_$TAG.json'));print('bench $v', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'])" | tee -a gpurun_out/rot_ab_$TAG.txt
done; done
RFA_LIB=alt/librfa_rot.so timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread -p no:cacheprovider \
    tests/test_gpu_parity.py tests/test_gpu_state.py tests/test_gpu_framing.py -k "65536 or 131072 or config3 or rtlsdr" > gpurun_out/pytest_rot_$TAG.log 2>&1
rc=$?; echo "pytest rot rc=$rc"; tail -2 gpurun_out/pytest_rot_$TAG.log
