#!/bin/bash
# Round-5 call j: config-5 kernel A variants (fp contraction off in fft_large.hip): twiddle split
# 64 (lo6, lo6w4 = capped at 128 VGPRs), 16-B z stores with / without sc1 (lo6sc / lo6wb);
# large-N parity per library (failures recorded), same-call A/B, rocprof split.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for L in lo6 lo6w4 lo6sc lo6wb; do
  RFA_LIB=abv/librfa_$L.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "large_n or 1048576 or 262144" -q --timeout 120 --timeout-method thread > gpurun_out/r05j_pytest_$L.txt 2>&1; rc=$?; echo "$L: $(tail -1 gpurun_out/r05j_pytest_$L.txt) $(grep FAILED gpurun_out/r05j_pytest_$L.txt | tr '\n' ' ')"; [ $rc -le 1 ] || exit $rc
done
A="--sizes 1048576 --formats s8 --samples 16777216 --state"
bash scripts/ab_kbench.sh gpurun_out/r05j_ab.txt "$A" \
  "base|RFA_LIB=abv/librfa_base.so" "lo6|RFA_LIB=abv/librfa_lo6.so" "lo6_g8|RFA_LIB=abv/librfa_lo6.so RFA_DIF_PIPE=8" \
  "lo6w4|RFA_LIB=abv/librfa_lo6w4.so" "lo6w4_g8|RFA_LIB=abv/librfa_lo6w4.so RFA_DIF_PIPE=8" \
  "lo6sc|RFA_LIB=abv/librfa_lo6sc.so" "lo6sc_g8|RFA_LIB=abv/librfa_lo6sc.so RFA_DIF_PIPE=8" \
  "lo6wb|RFA_LIB=abv/librfa_lo6wb.so" "lo6wb_g8|RFA_LIB=abv/librfa_lo6wb.so RFA_DIF_PIPE=8" \
  "base_b|RFA_LIB=abv/librfa_base.so" "lo6_b|RFA_LIB=abv/librfa_lo6.so" "lo6_g8_b|RFA_LIB=abv/librfa_lo6.so RFA_DIF_PIPE=8" \
  "lo6w4_b|RFA_LIB=abv/librfa_lo6w4.so" "lo6w4_g8_b|RFA_LIB=abv/librfa_lo6w4.so RFA_DIF_PIPE=8" \
  "lo6sc_b|RFA_LIB=abv/librfa_lo6sc.so" "lo6sc_g8_b|RFA_LIB=abv/librfa_lo6sc.so RFA_DIF_PIPE=8" \
  "lo6wb_b|RFA_LIB=abv/librfa_lo6wb.so" "lo6wb_g8_b|RFA_LIB=abv/librfa_lo6wb.so RFA_DIF_PIPE=8" || exit 1
for L in base lo6w4 lo6sc; do
  RFA_LIB=abv/librfa_$L.so timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r05j_prof_$L -o run -- python scripts/kbench.py $A --iters 10 > gpurun_out/r05j_prof_$L.log 2>&1 || exit 1
done
for L in base lo6w4 lo6sc; do echo "== $L"; f=$(find gpurun_out/r05j_prof_$L -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && head -6 "$f" | cut -d, -f1-5; done
exit 0
