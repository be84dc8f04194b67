#!/bin/bash
# Round-3 validation call: GPU parity suite, every-bin survey, default bench line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${1:-r03}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/pytest_gpu_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_gpu_$TAG.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u scripts/full_row_check.py > gpurun_out/full_row_$TAG.txt 2>&1
rc=$?; echo "full_row rc=$rc"; grep -v amdgpu.ids gpurun_out/full_row_$TAG.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench_$TAG.json; exit $rc
