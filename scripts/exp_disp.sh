#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_display.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_disp.log 2>&1
rc=$?; echo "display tests rc=$rc"; grep -E "PASS|FAIL|Error|assert" gpurun_out/pytest_disp.log | head -30; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_all.log 2>&1
rc=$?; echo "all gpu tests rc=$rc"; tail -2 gpurun_out/pytest_all.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --cpu-seconds 2 > gpurun_out/bench_disp.json 2> gpurun_out/bench_disp.err; rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench_disp.json; tail -3 gpurun_out/bench_disp.err
exit $rc
