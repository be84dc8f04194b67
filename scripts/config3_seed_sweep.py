#!/usr/bin/env python3
"""Every-bin parity on BASELINE config 3's batch (500 x 64 K s8 frames, Blackman) for several
synthetic captures (signals.frames_bytes seeds): librfa vs the float64 transform and vs the
reference's pffft, the reference's own error, and the share of bins beyond 0.01 dB.  The max
over 32.8 M bins is a tail statistic of fp32 rounding at the deepest bins and moves with the
data; this sweep shows by how much, for librfa and for pffft alike."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "tests", "golden")]


def main():
    import golden_util as gu
    import oracle
    import rfanalyzer_amd as rfa
    import signals
    n, b = 65536, 500
    seeds = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "3,5,7,11").split(",")]
    for sd in seeds:
        data = signals.frames_bytes(n, b, "s8", sd, tones=((0.1234, 0.4), (-0.377, 0.01)), noise=0.05)
        with rfa.SpectrumEngine(n, "blackman", "s8", ring_rows=0) as e:
            rows = e.process(data, b)
        ref64 = oracle.spectrum_rows(data, oracle.IN_S8, n, b, None, oracle.WIN_BLACKMAN)
        line = (f"seed {sd:3d}: |librfa - f64| max {gu.full_row_diff(rows, ref64, bar=None):.4f} dB, "
                f"share > 0.01 {gu.exceed_fraction(rows, ref64):.1e}")
        if oracle.ref_available():
            ref = oracle.ref_spectrum_rows(data, oracle.IN_S8, n, b)
            line += (f" | |librfa - pffft| max {gu.full_row_diff(rows, ref, bar=None):.4f}, share > 0.01 "
                     f"{gu.exceed_fraction(rows, ref):.1e}; |pffft - f64| max {gu.full_row_diff(ref, ref64, bar=None):.4f}, "
                     f"share > 0.01 {gu.exceed_fraction(ref, ref64):.1e}; beyond pffft's error "
                     f"{gu.full_row_bound(rows, ref, ref64):.4f}")
        print(line, flush=True)


if __name__ == "__main__":
    main()
