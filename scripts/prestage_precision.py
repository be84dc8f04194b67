"""Precision of the 64 K pre-stage's residue-1 forms at the deepest bins (CPU, numpy).

Emulates in float32 the three ways the wide kernel can form
y_1[m] = (x[m] w[m] - x[m + M] w[m + M]) W_N^m  (N = 65536, M = 32768):
  cw      complex window: x[m] (w[m] W^m) + x[m + M] (-w[m + M] W^m), the products
          rounded once from double (fft_wide.hip prestage CW, the kept form)
  mir     d = x0 w0 - x1 w1, then d * pre_a[m mod 1024] * W_64^(m / 1024): a rounded
          per-thread table times a rounded compile-time constant (the round-2 form and
          the mirrored-lane experiment, profiles/r03/mirror_lanes_ab.txt)
  mirtab  d * W^m with W^m rounded once from double (a per-point table)
then an exact (float64) FFT, so only the pre-stage's rounding shows, against the float64
oracle rows of the config-3 batch (500 x 64 K s8 Blackman).  The constant W_64^t is
shared by 1024 points, so its rounding is coherent and lands in spurs ~75 dB (this
scale: 10 log10 |X|/N) under the strong tone -- on the deepest bins of the batch.
usage: python scripts/prestage_precision.py [frames]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "tests", "golden")]
import oracle  # noqa: E402
import signals  # noqa: E402

F32 = np.float32


def cmul32(a, b):
    ar, ai, br, bi = a.real.astype(F32), a.imag.astype(F32), b.real.astype(F32), b.imag.astype(F32)
    return (ar * br - ai * bi).astype(F32) + 1j * (ar * bi + ai * br).astype(F32)


def main():
    n, b = 65536, int(sys.argv[1]) if len(sys.argv) > 1 else 500
    m_ = n // 2
    data = signals.frames_bytes(n, b, "s8", 3, tones=((0.1234, 0.4), (-0.377, 0.01)), noise=0.05)
    ref64 = oracle.spectrum_rows(data, oracle.IN_S8, n, b, None, oracle.WIN_BLACKMAN)
    w = oracle.window(n).astype(F32) / F32(128)  # the engine's pre-scaled window (exact)
    raw = np.frombuffer(data, np.int8).reshape(b, n, 2).astype(F32)
    m = np.arange(m_)
    wd = np.exp(-2j * np.pi * m / n)
    pa = np.exp(-2j * np.pi * (m % 1024) / n).astype(np.complex64)
    c64 = np.exp(-2j * np.pi * (1024 * (m // 1024)) / n).astype(np.complex64)
    cw0 = (w[:m_].astype(float) * wd).astype(np.complex64)
    cw1 = (-w[m_:].astype(float) * wd).astype(np.complex64)
    res = {}
    for name in ("cw", "mir", "mirtab"):
        out = np.empty((b, m_))
        for fr in range(b):
            x0r, x0i, x1r, x1i = raw[fr, :m_, 0], raw[fr, :m_, 1], raw[fr, m_:, 0], raw[fr, m_:, 1]
            if name == "cw":
                re = (x0r * cw0.real).astype(F32)
                im = (x0r * cw0.imag).astype(F32)
                re = (re - x0i * cw0.imag).astype(F32)
                im = (im + x0i * cw0.real).astype(F32)
                re = (re + x1r * cw1.real).astype(F32)
                im = (im + x1r * cw1.imag).astype(F32)
                re = (re - x1i * cw1.imag).astype(F32)
                im = (im + x1i * cw1.real).astype(F32)
                y = re + 1j * im
            else:
                d = (x0r * w[:m_] - x1r.astype(float) * w[m_:]).astype(F32) + 1j * (
                    x0i * w[:m_] - x1i.astype(float) * w[m_:]).astype(F32)
                y = cmul32(cmul32(d, pa), c64) if name == "mir" else cmul32(d, wd.astype(np.complex64))
            out[fr] = 10 * np.log10(np.abs(np.fft.fft(y.astype(complex))) / n)
        res[name] = out
    k = 2 * np.arange(m_) + 1  # residue-1 bins, natural order; ref rows are fft-shifted
    ref = ref64[:, (k + n // 2) % n]
    order = np.argsort((ref - ref.mean(1, keepdims=True)), axis=None)[:2000]
    for name, out in res.items():
        d = np.abs(out - ref)
        deep = d.ravel()[order]
        print(f"{name:7s} all bins: max {d.max():.4f} dB  p99.99 {np.quantile(d, 0.9999):.2e} | "
              f"2000 deepest bins: max {deep.max():.4f} rms {np.sqrt((deep ** 2).mean()):.2e}")


if __name__ == "__main__":
    main()
