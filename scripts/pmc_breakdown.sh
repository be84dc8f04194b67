#!/bin/bash
# SQ / LDS / memory-pipe breakdown of the main FFT kernel, one counter group per
# rocprofv3 --pmc pass.  usage: pmc_breakdown.sh TAG "kbench args"
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=$1; ARGS=$2
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE" \
           "SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_MISC SQ_INSTS_SMEM SQ_ACTIVE_INST_FLAT SQ_LDS_IDX_ACTIVE SQ_LDS_UNALIGNED_STALL"; do
  i=$((i+1))
  rm -rf gpurun_out/pmcb_${TAG}_$i
  timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/pmcb_${TAG}_$i -o p -- python3 scripts/kbench.py --iters 3 $ARGS > gpurun_out/pmcb_${TAG}_$i.log 2>&1 || { echo "pmc pass $i failed"; tail -3 gpurun_out/pmcb_${TAG}_$i.log; exit 1; }
done
python3 - "$TAG" <<'PY'
import csv, glob, sys, collections
tag = sys.argv[1]
acc = collections.defaultdict(list)
for f in sorted(glob.glob(f"gpurun_out/pmcb_{tag}_*/**/*counter_collection.csv", recursive=True)):
    for r in csv.DictReader(open(f)):
        if "fft_" in r["Kernel_Name"] or "fft64_kernel" in r["Kernel_Name"]:
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
print(tag, {k: round(sum(v) / len(v)) for k, v in sorted(acc.items())})
PY
