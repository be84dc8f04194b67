#!/bin/bash
# Round-4: balanced exchange 0 timing (same call: round-3 library, balanced default, writer-wave
# forms X0R=3 / X0R=2 on the A/B build), per-wave stamps, config-3 seed sweep.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${1:-r04f}
export TMPDIR=/tmp
V=()
for rnd in 1 2; do
  V+=("base_$rnd|RFA_LIB=alt/librfa_base.so" "bal_$rnd|" "x0r3_$rnd|RFA_LIB=alt/librfa_ab.so RFA_W64_X0R=3" "x0r2_$rnd|RFA_LIB=alt/librfa_ab.so RFA_W64_X0R=2")
  V+=("bal_p1_$rnd|RFA_LIB=alt/librfa_ab.so RFA_W64_PRIO=1" "bal_p2_$rnd|RFA_LIB=alt/librfa_ab.so RFA_W64_PRIO=2" "bal_p3_$rnd|RFA_LIB=alt/librfa_ab.so RFA_W64_PRIO=3")
  V+=("bal_prew_$rnd|RFA_LIB=alt/librfa_ab.so RFA_W64_PREW=1" "x0r3_prew_$rnd|RFA_LIB=alt/librfa_ab.so RFA_W64_PREW=1 RFA_W64_X0R=3")
  V+=("old64_$rnd|RFA_LIB=alt/librfa_ab.so RFA_W64_FORMATS=0")
done
bash scripts/ab_kbench.sh gpurun_out/w64_ab_$TAG.txt "--sizes 65536 --formats s8,f32 --samples 32768000 --state" "${V[@]}" || exit $?
rm -f gpurun_out/stamps_$TAG.bin
RFA_LIB=alt/librfa_ab.so RFA_STAMPS_FILE=gpurun_out/stamps_$TAG.bin timeout -k 10 120 python -u scripts/kbench.py \
    --sizes 65536 --formats s8 --samples 32768000 --state --iters 2 > gpurun_out/stamps_$TAG.log 2>&1
rc=$?; echo "stamps rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/stamps_$TAG.log; exit $rc; }
python3 scripts/stamps_w64.py gpurun_out/stamps_$TAG.bin > gpurun_out/stamps_$TAG.txt 2>&1; cat gpurun_out/stamps_$TAG.txt
timeout -k 10 300 python -u scripts/config3_seed_sweep.py 3,5,7,11 > gpurun_out/seed_sweep_$TAG.txt 2>&1
rc=$?; echo "sweep rc=$rc"; cat gpurun_out/seed_sweep_$TAG.txt | grep -v amdgpu.ids
