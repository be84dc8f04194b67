#!/bin/bash
# Per-sample instruction budget of the streaming FFT kernels: one rocprofv3
# --pmc pass per (format, N) over scripts/kbench.py (500 x 64 K samples per launch), SQ
# instruction counts + VALU-active cycles + wave waits + GPU cycles, and the kernel time of the
# same run (HIP events).  Output: gpurun_out/r06sq/table.txt
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r06sq
mkdir -p $O
CNT="SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAVE_CYCLES GRBM_GUI_ACTIVE"
for cfg in "s8 1024" "s8 8192" "s8 16384" "s8 65536" "f32 1024" "f32 8192" "f32 16384" "f32 65536" "s8 65536 --state"; do
  set -- $cfg
  tag="$1_$2${3:+_state}"
  rm -rf $O/p_$tag
  timeout -s KILL 120 rocprofv3 --pmc $CNT --output-format csv -d $O/p_$tag -o p -- \
      python3 scripts/kbench.py --iters 3 --samples 32768000 --formats $1 --sizes $2 ${3:-} > $O/p_$tag.log 2>&1 \
      || { echo "pmc $tag failed"; tail -3 $O/p_$tag.log; exit 1; }
  timeout -k 10 120 python3 scripts/kbench.py --iters 10 --samples 32768000 --formats $1 --sizes $2 ${3:-} > $O/t_$tag.log 2>&1 \
      || { echo "time $tag failed"; exit 1; }
done
python3 scripts/sq_table.py $O > $O/table.txt && cat $O/table.txt
