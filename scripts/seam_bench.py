"""Legacy-seam plan timing (csrc/fft_seam.hip): wall time per rfa_seam_fft_ordered /
rfa_seam_fft_logmag_interleaved call (host arrays in and out, as the JNI symbols use it)
at lengths the streaming handle does not take.  Run under
`rocprofv3 --kernel-trace --stats` for the per-pass kernel durations; each pass moves
16 B per point (8 read, 8 written).

usage: python scripts/seam_bench.py [--reps 20]
"""
import argparse
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rfanalyzer_amd.engine import SeamPlan  # noqa: E402

SIZES = [48, 3888, 48000, 1 << 21, 3 << 20, 1 << 24, 1 << 26]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    for n in SIZES:
        x = np.random.default_rng(n).standard_normal(2 * n).astype(np.float32)
        reps = a.reps if n <= (1 << 22) else max(3, a.reps // 5)
        with SeamPlan(n) as p:
            plan = p.plan()
            p.fft_ordered(x)  # warm
            t0 = time.perf_counter()
            for _ in range(reps):
                p.fft_ordered(x)
            t_ord = (time.perf_counter() - t0) / reps
            p.fft_logmag(x)
            t0 = time.perf_counter()
            for _ in range(reps):
                p.fft_logmag(x)
            t_mag = (time.perf_counter() - t0) / reps
        print(f"n={n:>9} plan={plan} passes={len(plan)} ordered {t_ord * 1e3:9.3f} ms  logmag {t_mag * 1e3:9.3f} ms"
              f"  ({n / t_mag / 1e6:8.1f} Msamples/s host-to-host)", flush=True)


if __name__ == "__main__":
    main()
