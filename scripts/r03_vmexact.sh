#!/bin/bash
# Round-3 A/B: the staged kernels' item-start wait exactly past the previous item's epilogue
# stores (RFA_VMEXACT: vmcnt(8) / vmcnt(40)) instead of draining them (vmcnt(0) / (32)); parity
# of the in-tree build (GPU parity + state suites), then three interleaved kbench rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_state.py -m gpu -x -q \
    --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/vm_parity.log 2>&1
rc=$?; echo "parity rc=$rc"; tail -1 gpurun_out/vm_parity.log; [ $rc -ne 0 ] && exit $rc
V=()
for rnd in 1 2 3; do
  for v in vm0 vm1; do V+=("${v}_$rnd|RFA_LIB=alt/librfa_$v.so"); done
done
bash scripts/ab_kbench.sh gpurun_out/vmexact_ab.txt "--sizes 8192,16384,65536 --formats s8,u8 --samples 32768000 --state" "${V[@]}"
