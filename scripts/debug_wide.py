"""Compare wide vs narrow kernel complex outputs bin by bin (debug aid)."""
import os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import rfanalyzer_amd
for n in (8192, 16384):
    rng = np.random.default_rng(0)
    x = rng.standard_normal(2 * n).astype(np.float32)
    ref = np.fft.fft(x[0::2].astype(np.float64) + 1j * x[1::2])
    out = {}
    for k in ("narrow", "wide"):
        os.environ["RFA_KERNEL"] = k
        with rfanalyzer_amd.SpectrumEngine(n, "none", "f32", ring_rows=0) as e:
            c = e.fft_ordered(x)
        out[k] = c[0::2] + 1j * c[1::2]
        err = np.abs(out[k] - ref) / np.abs(ref).max()
        bad = np.nonzero(err > 1e-5)[0]
        print(n, k, "max rel err", err.max(), "bad bins", bad.size, bad[:16])
        if bad.size:
            M = n; TPF = M // 64
            tid = bad % TPF; b = (bad // TPF) % 4; t = bad // (M // 16)
            print("   tid", np.unique(tid)[:20], "b", np.unique(b), "t", np.unique(t))
            print("   sample got/ref", out[k][bad[:4]], ref[bad[:4]])
