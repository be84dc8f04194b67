#!/bin/bash
# Round evidence in one GPU call: GPU parity tests + smoke, profile_round (bench +
# rocprof stats + 2 PMC passes), then the kernel micro-bench over sizes/formats.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${1:-r01}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_gpu_$TAG.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/smoke_$TAG.log; [ $rc -ne 0 ] && exit $rc
bash scripts/profile_round.sh $TAG || exit $?
timeout -k 10 300 python scripts/kbench.py --sizes 1024,4096,8192,16384,32768,65536,131072,262144,1048576 --formats s8,f32 \
    > gpurun_out/kbench_$TAG.txt 2>&1
rc=$?; echo "kbench rc=$rc"; grep -v amdgpu.ids gpurun_out/kbench_$TAG.txt
exit $rc
