"""TEST INFRASTRUCTURE ONLY -- restatement of the reference's scanner row reductions.

ui/MainViewModel.kt (app/src/main/java/com/mantz_it/rfanalyzer/):
getAverageSignalLevel (:1391-1413) and detectSignal (:1415-1457) over the whole
newest row, detectSignalsInFFT (:1462-1540) over +-2-bin windows per scan step,
detectIEMChannelsInFFT (:861-929) over +-max(5, (100000/res).toInt()) bins per
channel.  Kotlin's FloatArray.maxOrNull() (NaN wins) and FloatArray.average()
(sequential double sum / count, then toFloat()) are restated literally here, in
pure Python over a host copy of the row.
"""
from __future__ import annotations

import math

import numpy as np

F32 = np.float32


def max_or_null(xs) -> np.float32:
    """FloatArray.maxOrNull(): NaN if any element is NaN."""
    m = F32(xs[0])
    for x in xs[1:]:
        x = F32(x)
        if math.isnan(x) or math.isnan(m):
            m = F32(math.nan)
        elif x > m:
            m = x
    return m


def average(xs) -> np.float32:
    """FloatArray.average(): double accumulation in order, / count, then toFloat()."""
    s = 0.0
    for x in xs:
        s += float(x)
    return F32(s / len(xs))


def window_stats(row: np.ndarray, lo, hi):
    """(peak, avg) per inclusive window of one row."""
    pk = np.array([max_or_null(row[a:b + 1]) for a, b in zip(lo, hi)], np.float32)
    av = np.array([average(row[a:b + 1]) for a, b in zip(lo, hi)], np.float32)
    return pk, av
