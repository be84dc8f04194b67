#!/bin/bash
# Round-5 call o: wave-local exchange sync in fft_rows_kernel (N <= 1024: one wave per sub-FFT, no
# workgroup barrier): parity of the small sizes on the build, same-call A/B vs the barrier form.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
RFA_LIB=abv/librfa_ws1.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_jni.py tests/test_gpu_seam.py tests/test_gpu_framing.py -q --timeout 120 --timeout-method thread > gpurun_out/r05o_pytest.txt 2>&1; rc=$?; tail -1 gpurun_out/r05o_pytest.txt; grep FAILED gpurun_out/r05o_pytest.txt; [ $rc -eq 0 ] || exit $rc
A="--sizes 64,256,512,1024,2048 --formats s8,f32 --samples 16777216"
bash scripts/ab_kbench.sh gpurun_out/r05o_ab.txt "$A" "ws0|RFA_LIB=abv/librfa_ws0.so" "ws1|RFA_LIB=abv/librfa_ws1.so" "ws0_b|RFA_LIB=abv/librfa_ws0.so" "ws1_b|RFA_LIB=abv/librfa_ws1.so"
