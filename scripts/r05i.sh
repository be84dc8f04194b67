#!/bin/bash
# Round-5 call i: config-5 kernel A (dif_front_pipe_kernel) variants -- twiddle split 64 (D table
# 16 KB: 4 blocks per CU), 16-B z stores -- parity of the large-N tests on each, same-call A/B of
# the 1 M pair (16 s8 frames, ring + state), frame-group sweep, rocprof split per library.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for L in lo6 lo6st st16; do
  RFA_LIB=abv/librfa_$L.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "large_n or n1048576 or 1048576 or 262144" --deselect "tests/test_gpu_parity.py::test_all_sizes_and_formats_vs_oracle[f32-1048576]" -q --timeout 120 --timeout-method thread > gpurun_out/r05i_pytest_$L.txt 2>&1; rc=$?; echo "$L: $(tail -1 gpurun_out/r05i_pytest_$L.txt)"; [ $rc -le 1 ] || exit $rc  # 1 = a test failed (recorded): the A/B still runs
done
A="--sizes 1048576 --formats s8 --samples 16777216 --state"
bash scripts/ab_kbench.sh gpurun_out/r05i_ab.txt "$A" \
  "base|RFA_LIB=abv/librfa_base.so" "lo6|RFA_LIB=abv/librfa_lo6.so" "lo6_g8|RFA_LIB=abv/librfa_lo6.so RFA_DIF_PIPE=8" \
  "lo6_g4|RFA_LIB=abv/librfa_lo6.so RFA_DIF_PIPE=4" "lo6st|RFA_LIB=abv/librfa_lo6st.so" "st16|RFA_LIB=abv/librfa_st16.so" \
  "base_b|RFA_LIB=abv/librfa_base.so" "lo6_b|RFA_LIB=abv/librfa_lo6.so" "lo6_g8_b|RFA_LIB=abv/librfa_lo6.so RFA_DIF_PIPE=8" \
  "lo6st_b|RFA_LIB=abv/librfa_lo6st.so" "st16_b|RFA_LIB=abv/librfa_st16.so" || exit 1
for L in base lo6 lo6st; do
  RFA_LIB=abv/librfa_$L.so timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/r05i_prof_$L -o run -- python scripts/kbench.py $A --iters 10 > gpurun_out/r05i_prof_$L.log 2>&1 || exit 1
done
for L in base lo6 lo6st; do echo "== $L"; f=$(find gpurun_out/r05i_prof_$L -name "*kernel_stats.csv" | head -1); head -6 "$f" | cut -d, -f1-4; done
