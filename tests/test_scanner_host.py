"""CPU: scanner window arithmetic (rfanalyzer_amd/scanner.py, MainViewModel.kt:861-929,
1462-1540) and the Kotlin FloatArray reductions restated in oracle/scanner.py."""
import numpy as np

from oracle import scanner as osc
from rfanalyzer_amd import scanner as sc

N, F0, SR = 4096, 433_000_000, 2_400_000


def test_bin_index_is_a_float_division():
    res = sc.resolution(SR, N)            # 2.4e6 / 4096 = 585.9375 exactly
    start = F0 - SR // 2
    assert sc.bin_index(F0, start, res) == N // 2
    assert sc.bin_index(start + 586, start, res) == 1  # 586 / 585.9375 = 1.0001 -> 1
    assert sc.bin_index(start - 1, start, res) == 0     # -0.0017 truncates toward zero


def test_scan_windows_cover_usable_band():
    freqs, lo, hi = sc.scan_windows(F0, SR, N, usable_bandwidth=2_000_000, step=25_000, scan_start=0,
                                    scan_end=10 ** 12)
    assert freqs[0] == F0 - 1_000_000 and freqs[-1] == F0 + 1_000_000
    assert len(freqs) == 81
    assert ((hi - lo) == 4).all()                      # +-2 bins inside the row
    assert lo.min() >= 0 and hi.max() < N


def test_iem_windows_half_width():
    freqs, lo, hi = sc.iem_windows(F0, SR, N, [F0 - 2_000_000, F0, F0 + 500_000])
    assert freqs == [F0, F0 + 500_000]                  # the first channel lies outside the row
    half = int(np.float32(100000) / np.float32(np.float32(SR) / np.float32(N)))  # 170
    assert (hi - lo == 2 * half).all()


def test_threshold_and_modes():
    assert sc.effective_threshold(-60, -80, 10) == np.float32(-60)
    assert sc.effective_threshold(-90, -80, 10) == np.float32(-70)
    assert sc._detected(sc.PEAK_ONLY, np.float32(-50), np.float32(-90), np.float32(-60))
    assert not sc._detected(sc.AVERAGE_ONLY, np.float32(-50), np.float32(-90), np.float32(-60))
    assert sc._detected(sc.PEAK_OR_AVERAGE, np.float32(-70), np.float32(-55), np.float32(-60))


def test_kotlin_reductions():
    row = np.array([-3.0, -1.0, -2.0, np.nan, -5.0], np.float32)
    assert osc.max_or_null(row[:3]) == np.float32(-1.0)
    assert np.isnan(osc.max_or_null(row))
    x = np.float32([0.1, 0.2, 0.3])
    assert osc.average(x) == np.float32((float(x[0]) + float(x[1]) + float(x[2])) / 3)
    pk, av = osc.window_stats(np.arange(10, dtype=np.float32), [0, 4], [3, 9])
    assert pk.tolist() == [3.0, 9.0] and av.tolist() == [1.5, 6.5]
