"""GPU: size-independent properties of the transform at the BASELINE sizes (64 K x 500 frames,
1 M), checked on the product path itself rather than against an oracle: Parseval and
linearity of the ordered complex spectrum (the reference's performFFT seam,
nativedsp.cpp:19-42), and three exact symmetries of the dB rows (nativedsp.cpp:72-79) through the
batched streaming path -- a power-of-two input scale adds exactly 10*log10(2) dB per factor 2, a
circular time shift leaves |X| unchanged, and a frequency shift by k0 bins rolls the fft-shifted
row by k0.  Window NONE for the symmetries (a window breaks shift invariance)."""
import numpy as np
import pytest

import golden_util as gu

pytestmark = pytest.mark.gpu

DB_2 = 10.0 * np.log10(2.0)  # row unit 10*log10(|X|/N): |X| doubles -> +3.0103 dB


def _cf32(n, frames, seed):
    rng = np.random.default_rng(seed)
    t = np.arange(n)
    x = np.empty((frames, n), np.complex64)
    for f in range(frames):
        k = rng.uniform(0, n)
        x[f] = (0.4 * np.exp(2j * np.pi * k * t / n) + 0.05 * (rng.standard_normal(n) + 1j * rng.standard_normal(n)))
    return x


def _interleave(x):
    out = np.empty(x.shape[:-1] + (2 * x.shape[-1],), np.float32)
    out[..., 0::2] = x.real
    out[..., 1::2] = x.imag
    return out


@pytest.mark.parametrize("n", [1024, 65536, 1 << 20])
def test_ordered_spectrum_parseval_and_linearity(rfa, n):
    """sum |X|^2 = N sum |x|^2 (relative 1e-5) and FFT(a x + b y) = a FFT(x) + b FFT(y) to fp32
    rounding (2e-6 of max |X|) on the ordered, unscaled complex spectrum."""
    x = _cf32(n, 2, n)
    a, b = np.float32(0.75), np.float32(-1.25)
    with rfa.SpectrumEngine(n, "none", "f32", ring_rows=0) as e:
        fx = e.fft_ordered(_interleave(x[0]))
        fy = e.fft_ordered(_interleave(x[1]))
        fz = e.fft_ordered(_interleave((a * x[0] + b * x[1]).astype(np.complex64)))
    cx = fx[0::2].astype(np.float64) + 1j * fx[1::2]
    cy = fy[0::2].astype(np.float64) + 1j * fy[1::2]
    cz = fz[0::2].astype(np.float64) + 1j * fz[1::2]
    e_time = np.sum(np.abs(x[0].astype(np.complex128)) ** 2)
    assert abs(np.sum(np.abs(cx) ** 2) / (n * e_time) - 1.0) <= 1e-5
    m = np.abs(cz).max()
    assert np.abs(cz - (float(a) * cx + float(b) * cy)).max() <= 2e-6 * m * np.sqrt(np.log2(n))


@pytest.mark.parametrize("n,frames", [(65536, 500), (1 << 20, 16)])
def test_rows_power_of_two_scale(rfa, n, frames):
    """x, 2x and x/4 through the batched path (cf32, window none, the config-3 / config-5 batch
    sizes): every arithmetic step scales by a power of two exactly, so every finite bin moves by
    exactly +10log10(2) and -2*10log10(2) dB up to the log's rounding (1e-4 dB)."""
    x = _interleave(_cf32(n, frames, 7))
    with rfa.SpectrumEngine(n, "none", "f32", ring_rows=0) as e:
        r1 = e.process(x.tobytes(), frames)
        r2 = e.process((2 * x).tobytes(), frames)
        r4 = e.process((x / 4).tobytes(), frames)
    fin = np.isfinite(r1)
    assert np.array_equal(fin, np.isfinite(r2)) and np.array_equal(fin, np.isfinite(r4))
    assert np.abs((r2 - r1)[fin] - DB_2).max() <= 1e-4
    assert np.abs((r4 - r1)[fin] + 2 * DB_2).max() <= 1e-4


@pytest.mark.parametrize("n,frames", [(65536, 500), (1 << 20, 16)])
def test_rows_time_shift_and_frequency_shift(rfa, n, frames):
    """Frame f and its circular time shift by d_f give the same dB row, and the frame multiplied
    by exp(2 pi i k0 n / N) = i^(q n) for k0 = q N / 4 (an exact quarter-turn per sample, so both
    inputs are exact in fp32) gives the row rolled by k0 bins -- within the transforms' own fp32
    rounding over the bins within the Parseval floor of the row level (golden_util.db_diff, the
    0.01 dB bar), with the peak bin exactly where the symmetry puts it.  Batched path at the
    BASELINE sizes.  (A general k0 needs a rounded input: its rounding noise alone reaches 0.012 dB
    at the floor bins of a 32.8 M-bin batch, measured.)"""
    x = _cf32(n, frames, 11)
    rng = np.random.default_rng(5)
    d = rng.integers(1, n, size=frames)
    q = rng.integers(1, 4, size=frames)
    k0 = q * (n // 4)
    t = np.arange(n)
    shifted = np.stack([np.roll(x[f], d[f]) for f in range(frames)]).astype(np.complex64)
    turn = np.array([1, 1j, -1, -1j], np.complex64)
    mixed = np.stack([x[f] * turn[(q[f] * t) % 4] for f in range(frames)])
    with rfa.SpectrumEngine(n, "none", "f32", ring_rows=0) as e:
        r0 = e.process(_interleave(x).tobytes(), frames)
        rs = e.process(_interleave(shifted).tobytes(), frames)
        rm = e.process(_interleave(mixed).tobytes(), frames)
    assert gu.db_diff(rs, r0) <= gu.DB_TOL
    rolled = np.stack([np.roll(r0[f], k0[f]) for f in range(frames)])
    assert gu.db_diff(rm, rolled) <= gu.DB_TOL
    np.testing.assert_array_equal(np.argmax(rs, 1), np.argmax(r0, 1))
    np.testing.assert_array_equal(np.argmax(rm, 1), np.argmax(rolled, 1))
