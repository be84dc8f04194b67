"""Debug: 64 K ring rows (rfa_get_ring, natural) vs the caller rows of the same frames."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
import numpy as np
import rfanalyzer_amd as rfa
import signals
for fmt in ("u8", "s8", "f32"):
    n, b = 65536, 5
    data = signals.frames_bytes(n, b, fmt, 7, tones=((0.11, 0.3),), noise=0.04)
    for rows_flag in (True, False):
        with rfa.SpectrumEngine(n, "blackman", fmt, ring_rows=6) as e:
            e.set_tuning(1, 2)
            rows = e.process(data, b, rows=rows_flag)
            ring, ri, wi = e.ring()
            pos = e.ring_positions()
        with rfa.SpectrumEngine(n, "blackman", fmt, ring_rows=0) as e2:
            ref = e2.process(data, b)
        for f in range(b):
            g = ring[(ri + (b - 1 - f)) % 6]
            bad = np.nonzero(np.abs(g - ref[f]) > 1e-3)[0]
            print(fmt, "rows" if rows_flag else "ring-only", "frame", f, "bad bins", bad.size,
                  bad[:12], (bad & 1)[:12] if bad.size else "", flush=True)
