#!/usr/bin/env python3
"""PCIe-inclusive rate of the host-buffer boundary (rfa_process_host: H2D copy
of raw IQ, kernels, D2H copy of the rows, synchronise), for DESIGN.md.  Not the
bench value: the bench starts with inputs resident in HBM."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import rfanalyzer_amd  # noqa: E402

for n, frames, fmt in [(65536, 256, "s8"), (16384, 1024, "s8"), (16384, 1024, "f32"), (1024, 4096, "s8")]:
    bps = {"s8": 2, "f32": 8}[fmt]
    data = np.random.default_rng(0).integers(-100, 100, n * frames * bps, dtype=np.int8)
    rows = np.empty(n * frames, np.float32)
    with rfanalyzer_amd.SpectrumEngine(n, "blackman", fmt, ring_rows=0) as e:
        e.process(data, frames)  # warm-up
        for rows_out in (True, False):
            t0 = time.perf_counter()
            it = 10
            for _ in range(it):
                e.process(data, frames, rows=rows_out)
            dt = (time.perf_counter() - t0) / it
            print(f"{fmt} N={n} frames={frames} rows_to_host={rows_out}: {n * frames / dt / 1e6:9.1f} Msamples/s "
                  f"({dt * 1e3:.2f} ms per batch, {n * frames * bps / dt / 1e9:.1f} GB/s of IQ in)", flush=True)
