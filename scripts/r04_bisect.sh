#!/bin/bash
# Round-4 bisect: run-to-run determinism and the two failing parity tests per library.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${1:-r04j}
export RFA_W64_FORMATS=0
for v in "head|alt/librfa_head.so" "w8all|alt/librfa_w8all.so" "notid|alt/librfa_notid.so" "new|"; do
  l=${v%%|*}; lib=${v#*|}
  echo "== $l"
  RFA_LIB=$lib timeout -k 10 120 python -u scripts/determinism_check.py 1048576 32768 65536 2>&1 | grep -v amdgpu.ids
  rc=${PIPESTATUS[0]}; [ $rc -ne 0 ] && { echo "det rc=$rc"; exit $rc; }
  RFA_LIB=$lib timeout -k 10 200 python -u -m pytest -q --timeout 120 --timeout-method thread -p no:cacheprovider \
     "tests/test_gpu_parity.py::test_large_n_front_kernel_alignment_paths" "tests/test_gpu_parity.py::test_cf32_staged_next_item_across_workgroup_items" \
     "tests/test_gpu_parity.py::test_all_sizes_and_formats_vs_oracle" 2>&1 | grep -E "passed|failed|FAILED|assert " | head -12
done
