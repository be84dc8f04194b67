"""Scanner and squelch reductions of the newest waterfall row.

Host mirror of the reference's scanner helpers in ui/MainViewModel.kt (paths
relative to app/src/main/java/com/mantz_it/rfanalyzer/): the window arithmetic
and detection rules stay on the host in the reference's types (Long, Float,
Kotlin ``toInt()``), the reductions over the fft-shifted newest ring row run on
the device (``rfa_row_window_stats``) instead of on a JVM copy of the row.

* ``average_signal_level``   -- getAverageSignalLevel, MainViewModel.kt:1391-1413
* ``detect_signal``          -- detectSignal, MainViewModel.kt:1415-1457
* ``detect_signals_in_fft``  -- detectSignalsInFFT, MainViewModel.kt:1462-1540
* ``detect_iem_channels``    -- detectIEMChannelsInFFT, MainViewModel.kt:861-929
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

F32 = np.float32
PEAK_ONLY, AVERAGE_ONLY, PEAK_OR_AVERAGE = "PEAK_ONLY", "AVERAGE_ONLY", "PEAK_OR_AVERAGE"  # ScanDetectionMode


def kotlin_float_to_int(x: np.float32) -> int:
    """Kotlin Float.toInt(): truncation toward zero, NaN -> 0, saturating."""
    if np.isnan(x):
        return 0
    if x >= 2 ** 31 - 1:
        return 2 ** 31 - 1
    if x <= -(2 ** 31):
        return -(2 ** 31)
    return int(x)


@dataclass
class DiscoveredSignal:
    frequency: int
    peak_strength: float
    average_strength: float


@dataclass
class IEMDetectedChannel:
    channel_frequency: int
    peak_strength: float
    average_strength: float


def _detected(mode: str, peak: np.float32, avg: np.float32, thr: np.float32) -> bool:
    if mode == PEAK_ONLY:
        return bool(peak > thr)
    if mode == AVERAGE_ONLY:
        return bool(avg > thr)
    return bool(peak > thr or avg > thr)


def effective_threshold(threshold: float, noise_floor: float, margin: float) -> np.float32:
    """maxOf(threshold, noiseFloor + noiseFloorMargin) in Float."""
    s = F32(F32(noise_floor) + F32(margin))
    t = F32(threshold)
    return t if t >= s else s


def bin_index(frequency: int, start_frequency: int, resolution: np.float32) -> int:
    """((f - startFrequency) / frequencyResolution).toInt(): Long / Float is a Float division."""
    return kotlin_float_to_int(F32(F32(frequency - start_frequency) / resolution))


def resolution(sample_rate: int, n: int) -> np.float32:
    return F32(F32(sample_rate) / F32(n))  # sampleRate.toFloat() / fftSize


def scan_windows(center: int, sample_rate: int, n: int, usable_bandwidth: int, step: int, scan_start: int,
                 scan_end: int):
    """detectSignalsInFFT's loop (MainViewModel.kt:1490-1512): frequencies and +-2-bin windows."""
    res = resolution(sample_rate, n)
    start_frequency = center - sample_rate // 2
    usable_start = (sample_rate - usable_bandwidth) // 2
    usable_end = usable_start + usable_bandwidth
    f = max(scan_start, start_frequency + usable_start)
    end = min(scan_end, start_frequency + usable_end)
    freqs, lo, hi = [], [], []
    while f <= end:
        b = bin_index(f, start_frequency, res)
        if 0 <= b < n:
            freqs.append(f)
            lo.append(max(0, b - 2))
            hi.append(min(n - 1, b + 2))
        f += step
    return freqs, np.array(lo, np.int32), np.array(hi, np.int32)


def iem_windows(center: int, sample_rate: int, n: int, channel_frequencies):
    """detectIEMChannelsInFFT windows (MainViewModel.kt:884-898): +-max(5, (100000/res).toInt()) bins."""
    res = resolution(sample_rate, n)
    start_frequency = center - sample_rate // 2
    half = max(5, kotlin_float_to_int(F32(F32(100000) / res)))
    freqs, lo, hi = [], [], []
    for cf in channel_frequencies:
        b = bin_index(cf, start_frequency, res)
        if 0 <= b < n:
            freqs.append(cf)
            lo.append(max(0, b - half))
            hi.append(min(n - 1, b + half))
    return freqs, np.array(lo, np.int32), np.array(hi, np.int32)


def average_signal_level(engine) -> float:
    """Mean dB of the newest row (MainViewModel.kt:1391-1413)."""
    _, av = engine.row_window_stats([0], [engine.n - 1])
    return float(av[0])


def detect_signal(engine, threshold: float, mode: str, noise_floor: float, margin: float):
    """(peak, avg) of the newest row if detected, else None (MainViewModel.kt:1415-1457)."""
    pk, av = engine.row_window_stats([0], [engine.n - 1])
    thr = effective_threshold(threshold, noise_floor, margin)
    return (float(pk[0]), float(av[0])) if _detected(mode, pk[0], av[0], thr) else None


def detect_signals_in_fft(engine, center: int, sample_rate: int, usable_bandwidth: int, step: int, threshold: float,
                          mode: str, noise_floor: float, margin: float, scan_start: int, scan_end: int):
    """MainViewModel.kt:1462-1540 with the window reductions on the device."""
    freqs, lo, hi = scan_windows(center, sample_rate, engine.n, usable_bandwidth, step, scan_start, scan_end)
    if not freqs:
        return []
    pk, av = engine.row_window_stats(lo, hi)
    thr = effective_threshold(threshold, noise_floor, margin)
    return [DiscoveredSignal(f, float(p), float(a)) for f, p, a in zip(freqs, pk, av) if _detected(mode, p, a, thr)]


def detect_iem_channels(engine, channel_frequencies, center: int, sample_rate: int, threshold: float):
    """MainViewModel.kt:861-929: a channel is detected when its window peak exceeds the threshold."""
    freqs, lo, hi = iem_windows(center, sample_rate, engine.n, channel_frequencies)
    if not freqs:
        return []
    pk, av = engine.row_window_stats(lo, hi)
    return [IEMDetectedChannel(f, float(p), float(a)) for f, p, a in zip(freqs, pk, av) if p > F32(threshold)]
