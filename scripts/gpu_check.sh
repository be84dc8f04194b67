#!/bin/bash
# One GPU-box session: parity tests, smoke, short bench, rocprofv3 kernel stats.
# Stops at the first step that ends in a signal/timeout/crash (rc >= 124 or rc == 134/139).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r01}
STEPS=${STEPS:-all}
fatal() { [ "$1" -ge 124 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }

if [[ "$STEPS" == all || "$STEPS" == *test* ]]; then
  timeout -k 10 900 python -m pytest tests -m gpu -q -x -p no:cacheprovider > gpurun_out/pytest_gpu_$TAG.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu_$TAG.log
  if fatal $rc; then exit $rc; fi
fi
if [[ "$STEPS" == all || "$STEPS" == *smoke* ]]; then
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1
  rc=$?; echo "smoke rc=$rc"; tail -3 gpurun_out/smoke_$TAG.log
  if fatal $rc; then exit $rc; fi
fi
if [[ "$STEPS" == all || "$STEPS" == *bench* ]]; then
  timeout -k 10 400 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
  rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench_$TAG.json; tail -3 gpurun_out/bench_$TAG.err
  if fatal $rc; then exit $rc; fi
fi
if [[ "$STEPS" == all || "$STEPS" == *prof* ]]; then
  rm -rf gpurun_out/prof_$TAG
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- \
      python3 bench.py --cpu-seconds 0 ${BENCH_ARGS:-} > gpurun_out/prof_$TAG.log 2>&1
  rc=$?; echo "rocprof rc=$rc"; tail -3 gpurun_out/prof_$TAG.log
  find gpurun_out/prof_$TAG -name "*kernel_stats.csv" -exec cat {} \; | head -20
  if fatal $rc; then exit $rc; fi
fi
exit 0
