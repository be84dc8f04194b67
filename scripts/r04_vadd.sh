#!/bin/bash
# Round-4 A/B, same call: exchange stores without per-store address adds (one write base per
# round, unfused ds_write_b64) + the lane index opaque per item (no hoisted-base spills), and the
# DFTs' W_8 form limited to the wide kernel's own frames.
#   head  = before the 8 K alias and the W_8 fusion (alt/librfa_head.so)
#   w8all = alias + W_8 fusion everywhere (alt/librfa_w8all.so, the r04h "new")
#   new   = this tree (in-tree librfa.so)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${1:-r04i}
export TMPDIR=/tmp
V=()
for rnd in 1 2 3; do
  V+=("head_$rnd|RFA_LIB=alt/librfa_head.so" "w8all_$rnd|RFA_LIB=alt/librfa_w8all.so" "new_$rnd|")
done
bash scripts/ab_kbench.sh gpurun_out/vadd_ab_$TAG.txt "--sizes 8192,16384,32768,65536,1048576 --formats s8,f32" "${V[@]}" || exit $?
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_gpu_$TAG.log
exit $rc
