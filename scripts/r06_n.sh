#!/bin/bash
# Round 6 call n: code-placement control.  The same 64 K s8 kernel ISA in six libraries (the in-tree
# product, A/B builds base / base2 / ownq, and pad1 / pad2 = base2 plus an unused kernel ahead of the
# others), kbench 64 K s8 500 frames + state, interleaved over three rounds: how far do identical
# kernels differ by library alone?
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/r06n_ab
mkdir -p $O
export TMPDIR=/tmp
V=()
for i in 1 2 3; do
  V+=("product$i|RFA_LIB=rfanalyzer_amd/librfa.so" "base$i|RFA_LIB=abv/librfa_base.so" "base2_$i|RFA_LIB=abv/librfa_base2.so"
      "ownq$i|RFA_LIB=abv/librfa_ownq.so" "pad1_$i|RFA_LIB=abv/librfa_pad1.so" "pad2_$i|RFA_LIB=abv/librfa_pad2.so")
done
bash scripts/ab_kbench.sh $O/kbench.txt "--sizes 65536 --formats s8 --samples 32768000 --iters 30 --state" "${V[@]}" > /dev/null || exit 1
grep -E "^==|N=" $O/kbench.txt
exit 0
