"""TEST INFRASTRUCTURE ONLY -- pure-Python restatement of the display preprocessing.

Restates, operation by operation in the reference's types (Long, Double,
Float = numpy float32 scalars, Int), what the draw thread does with the
waterfall ring before drawing (paths relative to app/src/main/java/com/mantz_it/rfanalyzer/):

* ``AnalyzerSurface.drawPreprocessing`` (ui/AnalyzerSurface.kt:599-743): viewport
  start / end bins and pixels (:650-672), per pixel the mean of its bins summed in
  bin order (:693-705), the colour-map index truncated and clamped (:721-722),
  black outside the drawn range (:725), the boxcar time average of the newest
  L + 1 rows summed newest first (:710-714) with its path y and autoscale
  min / max (:663-665,713-718), the peak-hold y of row 0 (:707, -1 outside);
* ``createGqrxMap`` (ui/ColorMaps.kt:41-51) for realistic colour maps.

``draw_preprocess`` processes every row (what the lazy refresh converges to);
``Surface`` adds the reference's dirty-row bookkeeping (:619-640,678-684,735:
rows written since the last draw, everything after a viewport / scale / size
change, at most L + 6 rows per draw, the colour buffer persisting between draws)
with the marks FftProcessor sets (analyzer/FftProcessor.kt:181,193,215,219,223).
Pure-Python loops: small sizes only.
"""
from __future__ import annotations

import math

import numpy as np

from .processor import kotlin_float_to_int

F32 = np.float32
VERTICAL_SCALE_LOWER_BOUNDARY = F32(-100.0)  # database/AppStateRepository.kt:92
VERTICAL_SCALE_UPPER_BOUNDARY = F32(10.0)    # database/AppStateRepository.kt:93
BLACK = 0xFF000000                            # Color.rgb(0, 0, 0)


def argb(a: int, r: int, g: int, b: int) -> int:
    """android.graphics.Color.argb(int...) as an unsigned 32-bit value."""
    return ((a & 0xFF) << 24) | ((r & 0xFF) << 16) | ((g & 0xFF) << 8) | (b & 0xFF)


def _kdiv(a: int, b: int) -> int:
    """Kotlin Int division (truncates toward zero)."""
    q = abs(a) // abs(b)
    return q if (a >= 0) == (b >= 0) else -q


def gqrx_colormap() -> np.ndarray:
    """ColorMaps.kt:41-51 createGqrxMap(): 256 ARGB colours (Int arithmetic)."""
    out = []
    for i in range(256):
        if i < 20:
            c = argb(0xFF, 0, 0, 0)
        elif i < 70:
            c = argb(0xFF, 0, 0, _kdiv(140 * (i - 20), 50))
        elif i < 100:
            c = argb(0xFF, _kdiv(60 * (i - 70), 30), _kdiv(125 * (i - 70), 30), _kdiv(115 * (i - 70), 30) + 140)
        elif i < 150:
            c = argb(0xFF, _kdiv(195 * (i - 100), 50) + 60, _kdiv(130 * (i - 100), 50) + 125,
                     255 - _kdiv(255 * (i - 100), 50))
        elif i < 250:
            c = argb(0xFF, 255, 255 - _kdiv(255 * (i - 150), 100), 0)
        else:
            c = argb(0xFF, 255, _kdiv(255 * (i - 250), 5), _kdiv(255 * (i - 250), 5))
        out.append(c)
    return np.array(out, dtype=np.uint32)


def kotlin_double_to_int(x: float) -> int:
    """Kotlin Double.toInt(): truncation toward zero, NaN -> 0, saturating."""
    if math.isnan(x):
        return 0
    if x >= 2 ** 31 - 1:
        return 2 ** 31 - 1
    if x <= -(2 ** 31):
        return -(2 ** 31)
    return int(x)


def _jmin(a: np.float32, b: np.float32) -> np.float32:
    """java.lang.Math.min(float, float): NaN wins, -0 < +0."""
    if np.isnan(a) or np.isnan(b):
        return F32(np.nan)
    if a == b:
        return a if np.signbit(a) else b
    return a if a < b else b


def _jmax(a: np.float32, b: np.float32) -> np.float32:
    if np.isnan(a) or np.isnan(b):
        return F32(np.nan)
    if a == b:
        return b if np.signbit(a) else a
    return a if a > b else b


def draw_preprocess(ring: np.ndarray, read_index: int, peaks, frequency: int, sample_rate: int, width: int,
                    fft_height: int, viewport_frequency: int, viewport_sample_rate: int, min_db: float, max_db: float,
                    average_length: int, colormap: np.ndarray, dirty=None, colors=None):
    """AnalyzerSurface.kt:599-743.  Returns (colors [R][width] uint32 in ring storage
    order, path_y [width] float32 (NaN: no path point), peaks_y [width] or None,
    (autoscale_min, autoscale_max)).  With ``dirty`` (bool per ring row, updated in
    place) and ``colors`` (the persistent colour buffer, updated in place) only the
    rows the reference refreshes are processed (:678-684)."""
    R, fft_size = ring.shape
    ring = ring.astype(np.float32, copy=False)
    min_db, max_db = F32(min_db), F32(max_db)
    cmap_size = int(colormap.size)
    # :650-672
    samples_per_hz = F32(fft_size) / F32(sample_rate)
    frequency_diff = viewport_frequency - frequency
    sample_rate_diff = viewport_sample_rate - sample_rate
    start = kotlin_double_to_int((float(frequency_diff) - float(sample_rate_diff) / 2.0) * float(samples_per_hz))
    end = fft_size + kotlin_double_to_int((float(frequency_diff) + float(sample_rate_diff) / 2.0)
                                          * float(samples_per_hz))
    samples_per_px = F32(end - start) / F32(width)
    db_diff = max_db - min_db
    db_width = F32(fft_height) / db_diff
    scale = F32(cmap_size) / db_diff
    first_pixel = 0 if start >= 0 else kotlin_float_to_int(F32(start * -1) / samples_per_px)
    last_pixel = (kotlin_float_to_int(F32(fft_size - start) / samples_per_px) if end >= fft_size
                  else kotlin_float_to_int(F32(end - start) / samples_per_px))

    if colors is None:
        colors = np.zeros((R, width), np.uint32)
    time_avg = np.zeros(width, np.float32)
    path_y = np.full(width, np.nan, np.float32)
    peaks_y = np.zeros(width, np.float32) if peaks is not None else None
    mn, mx = VERTICAL_SCALE_UPPER_BOUNDARY, VERTICAL_SCALE_LOWER_BOUNDARY
    rows_processed = 0
    for row_number in range(R):
        buffer_index = (read_index + row_number) % R
        if dirty is not None:
            if not dirty[buffer_index] and row_number > average_length:
                continue  # already up to date
            if rows_processed > average_length + 5:
                break     # at most 5 dirty rows beyond the averaged ones per draw
        row = ring[buffer_index]
        for i in range(width):
            if first_pixel + 1 <= i < last_pixel - 1:
                avg, peak_avg, counter = F32(0.0), F32(0.0), 0
                j = kotlin_float_to_int(F32(i) * samples_per_px)
                hi = F32(i + 1) * samples_per_px
                if j + start < 0:  # the reference would throw here; the device skips such bins
                    j = -start
                while F32(j) < hi and j + start < fft_size:
                    avg = F32(avg + row[j + start])
                    if row_number == 0 and peaks is not None:
                        peak_avg = F32(peak_avg + F32(peaks[j + start]))
                    counter += 1
                    j += 1
                with np.errstate(invalid="ignore", divide="ignore"):
                    avg = F32(avg / F32(counter))
                    if row_number == 0 and peaks is not None:
                        peaks_y[i] = F32(fft_height) - (F32(peak_avg / F32(counter)) - min_db) * db_width
                if row_number <= average_length:
                    time_avg[i] = F32(time_avg[i] + avg)
                if row_number == average_length:
                    ta = F32(time_avg[i] / F32(average_length + 1))
                    path_y[i] = F32(fft_height) - (ta - min_db) * db_width
                    mn = _jmin(ta, mn)
                    mx = _jmax(ta, mx)
                with np.errstate(invalid="ignore"):
                    idx = kotlin_float_to_int(F32((avg - min_db) * scale))
                colors[buffer_index, i] = colormap[0 if idx < 0 else (cmap_size - 1 if idx >= cmap_size else idx)]
            else:
                colors[buffer_index, i] = BLACK
                if peaks is not None:
                    peaks_y[i] = F32(-1.0)
        rows_processed += 1
        if dirty is not None:
            dirty[buffer_index] = False
    return colors, path_y, peaks_y, (float(mn), float(mx))


class Surface:
    """The draw thread's persistent state: colour buffer, dirty map, last viewport."""

    def __init__(self, ring_rows: int):
        self.dirty = np.ones(ring_rows, bool)
        self.colors = None
        self.last = None

    def mark_row(self, buffer_index: int) -> None:  # FftProcessor.kt:223 (the row just written)
        self.dirty[buffer_index] = True

    def mark_all(self, ring_rows: int | None = None) -> None:  # :181,193,215,219 (new size, resize, retune)
        if ring_rows is not None and ring_rows != self.dirty.size:
            self.dirty = np.ones(ring_rows, bool)
        self.dirty[:] = True

    def draw(self, ring, read_index, peaks, frequency, sample_rate, width, fft_height, viewport_frequency,
             viewport_sample_rate, min_db, max_db, average_length, colormap):
        R = ring.shape[0]
        if self.dirty.size != R:
            self.mark_all(R)
        if self.colors is None or self.colors.shape != (R, width):  # :619-626 new bitmap / colour buffer
            self.colors = np.zeros((R, width), np.uint32)
            self.dirty[:] = True
        key = (viewport_frequency, viewport_sample_rate, F32(min_db), F32(max_db))
        if key != self.last:  # :634-640
            self.dirty[:] = True
            self.last = key
        c, p, k, mm = draw_preprocess(ring, read_index, peaks, frequency, sample_rate, width, fft_height,
                                      viewport_frequency, viewport_sample_rate, min_db, max_db, average_length,
                                      colormap, dirty=self.dirty, colors=self.colors)
        return c.copy(), p, k, mm
