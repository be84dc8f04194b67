#!/bin/bash
# Round 6 call c: XCD-cluster exchange microbenchmark, the per-sample instruction budget (SQ), and
# the config-5 split-batch overlap A/B (RFA_DIF_SPLIT, A/B build), every GPU step time-limited.
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/r06c
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 120 ./scripts/ubench_cluster > $O/cluster.txt 2>&1 || { echo "cluster rc=$?"; cat $O/cluster.txt; exit 1; }
cat $O/cluster.txt
for i in 1 2; do
  for sp in 0 1; do
    RFA_LIB=abv/librfa_base.so RFA_DIF_SPLIT=$sp timeout -k 10 120 python3 scripts/kbench.py --sizes 1048576 --formats s8 \
        --samples 16777216 --iters 30 --state > $O/c5_split${sp}_$i.txt 2>&1 || { echo "c5 $sp rc=$?"; exit 1; }
    echo "split=$sp $(grep N= $O/c5_split${sp}_$i.txt)"
  done
done
./scripts/r06_sq_table.sh > $O/sq.log 2>&1 || { echo "sq rc=$?"; tail -5 $O/sq.log; exit 1; }
cat gpurun_out/r06sq/table.txt
exit 0
