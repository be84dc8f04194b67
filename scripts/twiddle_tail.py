"""is the config-3 tail |librfa - pffft| pffft's own float-argument twiddles?

For each config-3 capture (500 x 64 K s8 Blackman frames, seeds golden_util.CONFIG3_SEEDS) it
computes three CPU row sets -- the float64 transform (oracle/liborc.so), the reference's pffft
(oracle/_ref/libpffft_ref.so) and the same pffft with exact-angle twiddle tables
(oracle/_ref/libpffft_exact.so, oracle/exact_twiddle.c) -- and prints, per capture:
  |pffft - pffft_exact|, |pffft_exact - float64|, |pffft - float64| (max, share > 0.01 dB, deep-bin
  error) and, when --rows DIR holds librfa's rows of the same captures (rows_seed{S}.npy, written
  by tests/test_gpu_parity.py with RFA_SAVE_ROWS=DIR), |librfa - pffft_exact| and |librfa - float64|.

--config 2 / 4 / 5 runs the same three-way comparison on those batches (16 K cf32 Hann x 1024,
8 K s8 x 256, 1 M s8 x 16) and prints the counts the GPU tests compare (share > 0.01 dB, 1e-6
quantile) for pffft and pffft_exact against float64.

usage: python scripts/twiddle_tail.py [--config 3] [--seeds 3 5 7 11] [--frames 500] [--rows DIR]
"""
from __future__ import annotations

import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import oracle  # noqa: E402  (test infrastructure: this is a diagnostic script)
import golden_util as gu  # noqa: E402
import signals  # noqa: E402


def stats(a, b):
    return (f"max {gu.full_row_diff(a, b, bar=None):.4f} dB, share>0.01 {gu.exceed_fraction(a, b):.2e}, "
            f"1e-6 q {gu.tail_quantile(a, b):.4f}")


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--seeds", type=int, nargs="*", default=list(gu.CONFIG3_SEEDS))
    ap.add_argument("--frames", type=int, default=500)
    ap.add_argument("--rows", default=None)
    ap.add_argument("--config", type=int, default=3, choices=(2, 3, 4, 5))
    args = ap.parse_args()
    # the batches of tests/test_gpu_parity.py test_config{2,3,4,5}_no_worse_than_reference
    n, b, fmt, code, win = {2: (16384, 1024, "f32", oracle.IN_F32_INTERLEAVED, oracle.WIN_HANN),
                            3: (65536, args.frames, "s8", oracle.IN_S8, oracle.WIN_BLACKMAN),
                            4: (8192, 256, "s8", oracle.IN_S8, oracle.WIN_BLACKMAN),
                            5: (1 << 20, 16, "s8", oracle.IN_S8, oracle.WIN_BLACKMAN)}[args.config]
    print(f"config {args.config}: {b} x {n} {fmt}")
    for seed in args.seeds:
        if args.config == 2:
            data = signals.frames_bytes(n, b, "f32", seed, tones=((1000 / n, 0.5), (5000.5 / n, 0.05)), noise=0.01)
        else:
            data = signals.frames_bytes(n, b, "s8", seed, tones=((0.1234, 0.4), (-0.377, 0.01)), noise=0.05)
        f64 = oracle.spectrum_rows(data, code, n, b, None, win)
        ref = oracle.ref_spectrum_rows(data, code, n, b, None, win)
        ex = oracle.ref_spectrum_rows(data, code, n, b, None, win, exact_twiddles=True)
        de = {k: gu.deep_bin_error(v, f64) for k, v in (("pffft", ref), ("exact", ex))}
        print(f"seed {seed:2d}: |pffft - pffft_exact|  {stats(ref, ex)}")
        print(f"seed {seed:2d}: |pffft_exact - f64|    {stats(ex, f64)}; deep-bin error {de['exact']:.3e}")
        print(f"seed {seed:2d}: |pffft - f64|          {stats(ref, f64)}; deep-bin error {de['pffft']:.3e}")
        if args.rows:
            p = os.path.join(args.rows, f"rows_seed{seed}.npy")
            if os.path.exists(p):
                rows = np.load(p)
                print(f"seed {seed:2d}: |librfa - pffft_exact| {stats(rows, ex)}")
                print(f"seed {seed:2d}: |librfa - pffft|       {stats(rows, ref)}")
                print(f"seed {seed:2d}: |librfa - f64|         {stats(rows, f64)}; deep-bin error "
                      f"{gu.deep_bin_error(rows, f64):.3e}")
        sys.stdout.flush()


if __name__ == "__main__":
    main()
