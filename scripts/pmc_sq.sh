#!/bin/bash
# SQ stall breakdown of the main kernel (one --pmc pass, no tracing domains).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-sq}; shift
rm -rf gpurun_out/pmcsq_$TAG
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS \
   --output-format csv -d gpurun_out/pmcsq_$TAG -o run -- python3 scripts/kbench.py --iters 3 "$@" > gpurun_out/pmcsq_$TAG.log 2>&1
rc=$?; echo "pmc sq rc=$rc"; exit $rc
