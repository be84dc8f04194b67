#!/bin/bash
# Round 6 call m: wave-owned staging of the 64 K cf32 kernel's two staged quarters (RFA_STG_OWNQ, A/B
# build) against the product build: 64 K parity on the variant, then kbench (64 K f32 / f32p, 500
# frames, EMA + peak) interleaved over three rounds.
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/r06m_ab
mkdir -p $O
export TMPDIR=/tmp
RFA_LIB=abv/librfa_ownq.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_state.py \
    tests/test_gpu_properties.py -x -q --timeout 120 --timeout-method thread -m gpu -k "65536 or config3 or 64k" \
    > $O/pytest_ownq.txt 2>&1 || { echo "pytest rc=$?"; tail -30 $O/pytest_ownq.txt; exit 1; }
echo "ownq: $(tail -1 $O/pytest_ownq.txt)"
V=()
for i in 1 2 3; do V+=("base$i|RFA_LIB=abv/librfa_base.so" "ownq$i|RFA_LIB=abv/librfa_ownq.so"); done
bash scripts/ab_kbench.sh $O/kbench.txt "--sizes 65536 --formats f32,f32p,s8 --samples 32768000 --iters 30 --state" "${V[@]}" > /dev/null || exit 1
grep -E "^==|N=" $O/kbench.txt
exit 0
