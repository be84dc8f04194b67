#!/bin/bash
# Round 6 call d: the co-scheduled re-read cluster form (64 K as four 16 K residues on one XCD,
# A/B build -DRFA_RES16K=1) vs the product 32 K-residue kernel: parity spot check + kernel A/B.
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/r06d
mkdir -p $O
export TMPDIR=/tmp
RFA_LIB=abv/librfa_res16k.so timeout -k 10 180 python3 - > $O/res16k_parity.txt 2>&1 <<'PY' || { echo "parity rc=$?"; cat $O/res16k_parity.txt; exit 1; }
import sys
sys.path.insert(0, "tests")
import numpy as np, oracle, signals, golden_util as gu, rfanalyzer_amd as rfa
for fmt, code in (("s8", oracle.IN_S8), ("f32", oracle.IN_F32_INTERLEAVED)):
    n, b = 65536, 24
    data = signals.frames_bytes(n, b, fmt, 3, tones=((0.1234, 0.4), (-0.377, 0.01)), noise=0.05)
    with rfa.SpectrumEngine(n, "blackman", fmt, ring_rows=0) as e:
        rows = e.process(data, b)
    ref = oracle.spectrum_rows(data, code, n, b, None, oracle.WIN_BLACKMAN)
    d = gu.full_row_diff(rows, ref, bar=None)
    print(f"res16k {fmt}: max |librfa - float64| over every bin {d:.4f} dB, deep-bin error {gu.deep_bin_error(rows, ref):.3e}")
    assert d <= 0.1
PY
cat $O/res16k_parity.txt
for i in 1 2; do
  for v in base res16k; do
    RFA_LIB=abv/librfa_$v.so timeout -k 10 120 python3 scripts/kbench.py --sizes 65536 --formats s8,f32 --samples 32768000 \
        --iters 20 > $O/kb_${v}_$i.txt 2>&1 || { echo "kbench $v rc=$?"; tail -3 $O/kb_${v}_$i.txt; exit 1; }
    grep N= $O/kb_${v}_$i.txt | sed "s/^/$v: /"
  done
done
exit 0
