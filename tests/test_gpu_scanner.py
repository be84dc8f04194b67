"""GPU: newest-row window statistics (rfa_row_window_stats)
and the scanner functions built on them vs the Kotlin-semantics restatement
(oracle/scanner.py) on the ring row the device holds.  Peaks are bit-exact; the
averages are a double sum divided and rounded to float once, as the JVM's
FloatArray.average() -- only the order of the double additions differs, so the
float results agree to one ulp."""
import numpy as np
import pytest

import signals
from oracle import scanner as osc
from rfanalyzer_amd import scanner as sc

pytestmark = pytest.mark.gpu

N, R, F0, SR = 4096, 8, 433_000_000, 2_400_000


@pytest.fixture(scope="module")
def eng(rfa):
    e = rfa.SpectrumEngine(N, "blackman", "s8", ring_rows=R)
    e.set_tuning(F0, SR)
    e.process(signals.frames_bytes(N, 11, "s8", seed=33, tones=((0.21, 0.3), (0.37, 0.01), (-0.2, 0.002)),
                                   noise=0.01), 11, rows=False)
    yield e
    e.close()


def _newest_row(e):
    ring, ri, _ = e.ring()
    return ring[ri]


def _close(a, b):
    return np.all(np.abs(a.view(np.int32).astype(np.int64) - b.view(np.int32).astype(np.int64)) <= 1)


def test_window_stats_vs_kotlin(eng):
    row = _newest_row(eng)
    rng = np.random.default_rng(2)
    lo = rng.integers(0, N - 1, 300).astype(np.int32)
    hi = np.minimum(N - 1, lo + rng.integers(0, 400, 300)).astype(np.int32)
    lo, hi = np.concatenate([[0], lo]).astype(np.int32), np.concatenate([[N - 1], hi]).astype(np.int32)
    pk, av = eng.row_window_stats(lo, hi)
    epk, eav = osc.window_stats(row, lo, hi)
    np.testing.assert_array_equal(pk, epk)
    assert _close(av, eav)


@pytest.mark.parametrize("n", [65536, 131072, 1048576])
def test_window_stats_on_residue_major_ring(rfa, n):
    """The 64 K / 128 K ring is stored residue-major, the 1 M ring in the large-N kernel B's
    column order; the window kernel reads bins through ring_pos."""
    with rfa.SpectrumEngine(n, "blackman", "s8", ring_rows=3) as e:
        e.set_tuning(F0, SR)
        e.process(signals.frames_bytes(n, 4, "s8", seed=35, tones=((0.21, 0.3), (-0.2, 0.002)), noise=0.01), 4,
                  rows=False)
        row = _newest_row(e)
        rng = np.random.default_rng(5)
        lo = rng.integers(0, n - 1, 200).astype(np.int32)
        hi = np.minimum(n - 1, lo + rng.integers(0, 3000, 200)).astype(np.int32)
        pk, av = e.row_window_stats(lo, hi)
        epk, eav = osc.window_stats(row, lo, hi)
        np.testing.assert_array_equal(pk, epk)
        assert _close(av, eav)


def test_scanner_functions_match_restatement(eng):
    row = _newest_row(eng)
    # whole-row squelch level and detectSignal
    assert sc.average_signal_level(eng) == pytest.approx(float(osc.average(row)), rel=1e-6)
    got = sc.detect_signal(eng, -200.0, sc.PEAK_ONLY, -80.0, 5.0)
    assert got is not None and got[0] == float(osc.max_or_null(row))
    # detectSignalsInFFT: same frequencies detected, same peaks
    args = (F0, SR, 2_000_000, 12_500, -60.0, sc.PEAK_OR_AVERAGE, -90.0, 6.0, 0, 10 ** 12)
    found = sc.detect_signals_in_fft(eng, *args)
    freqs, lo, hi = sc.scan_windows(F0, SR, N, 2_000_000, 12_500, 0, 10 ** 12)
    epk, eav = osc.window_stats(row, lo, hi)
    thr = sc.effective_threshold(-60.0, -90.0, 6.0)
    exp = [f for f, p, a in zip(freqs, epk, eav) if p > thr or a > thr]
    assert [s.frequency for s in found] == exp and len(exp) > 0
    # IEM channels
    chans = [F0 + k * 100_000 for k in range(-14, 15)]
    det = sc.detect_iem_channels(eng, chans, F0, SR, -55.0)
    f2, lo2, hi2 = sc.iem_windows(F0, SR, N, chans)
    p2, _ = osc.window_stats(row, lo2, hi2)
    assert [d.channel_frequency for d in det] == [f for f, p in zip(f2, p2) if p > np.float32(-55.0)]


def test_bad_windows_rejected(eng, rfa):
    with pytest.raises(rfa.RfaError):
        eng.row_window_stats([5], [4])
    with pytest.raises(rfa.RfaError):
        eng.row_window_stats([0], [N])
