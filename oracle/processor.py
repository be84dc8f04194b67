"""TEST INFRASTRUCTURE ONLY -- numpy restatement of the FftProcessor state machine.

Restates, line by line, what the reference does with each log-mag row after
the FFT (paths relative to app/src/main/java/com/mantz_it/rfanalyzer/):

* ring of R rows initialised to -9999f, written in reverse order
  (analyzer/FftProcessor.kt:103,178-195,222-227);
* retune history shift / clear (FftProcessor.kt:197-220);
* peak-hold (FftProcessor.kt:229-245);
* boxcar time average of the newest L+1 rows in dB, at bin resolution
  (ui/AnalyzerSurface.kt:657,683-686,710-714);
* exponential average -- a north-star extension with the reference's only EMA
  idiom (database/GlobalPerformanceData.kt:44-50): first frame initialises,
  then avg += alpha*(x-avg); a -inf average is re-seeded by the next frame;
* channel mean dB for the squelch (analyzer/FftProcessor.kt:143-157);
* Scheduler framing of source packets into FFT frames
  (analyzer/Scheduler.kt:252-279, source/FileIQSource.java:318-369).
"""
from __future__ import annotations

import numpy as np

RING_FILL = np.float32(-9999.0)
PEAK_FILL = np.float32(-999999.0)
WATERFALL_ROWS = {"SLOW": 500, "NORMAL": 400, "FAST": 300}  # FftProcessor.kt:103


def kotlin_float_to_int(x: np.float32) -> int:
    """Kotlin Float.toInt(): truncation toward zero, NaN -> 0, saturating."""
    if np.isnan(x):
        return 0
    if x >= 2 ** 31 - 1:
        return 2 ** 31 - 1
    if x <= -(2 ** 31):
        return -(2 ** 31)
    return int(x)


def retune_shift_offset(frequency_diff: int, n: int, sample_rate: int) -> int:
    """FftProcessor.kt:143,199: ((lastF - f) * (N / sampleRate.toFloat())).toInt() in float32."""
    samples_per_hz = np.float32(n) / np.float32(sample_rate)
    return kotlin_float_to_int(np.float32(np.float32(frequency_diff) * samples_per_hz))


class FftProcessorRef:
    def __init__(self, n: int, ring_rows: int = 400, peak_hold: bool = False, ema_alpha: float | None = None):
        self.n = n
        self.ring = np.full((ring_rows, n), RING_FILL, np.float32)
        self.write_index = 0
        self.read_index = 0
        self.last_frequency = None
        self.last_sample_rate = None
        self.peak_hold = peak_hold
        self.peaks = None
        self.ema_alpha = None if ema_alpha is None else np.float32(ema_alpha)
        self.ema = None
        self.freq_or_sr_changed = True

    def set_waterfall_rows(self, rows: int) -> None:
        """waterfallSpeed change: takes effect in the next push (FftProcessor.kt:185-195)."""
        self.waterfall_rows = rows

    def push(self, row: np.ndarray, frequency: int, sample_rate: int) -> None:
        row = np.asarray(row, np.float32)
        target = getattr(self, "waterfall_rows", self.ring.shape[0])
        if row.size != self.ring.shape[1]:  # FftProcessor.kt:178-183: new FFT size -> fresh ring
            self.n = row.size
            self.ring = np.full((target, row.size), RING_FILL, np.float32)
            self.write_index = 0
        if self.ring.shape[0] != target:  # FftProcessor.kt:185-195: resize, history kept
            old = self.ring
            new_ring = np.full((target, self.n), RING_FILL, np.float32)
            for i in range(min(target, old.shape[0])):
                new_ring[i] = old[(self.write_index + i) % old.shape[0]]
            self.ring = new_ring
            self.write_index = 0
        n = self.n
        freq_changed = frequency != self.last_frequency
        sr_changed = sample_rate != self.last_sample_rate
        self.freq_or_sr_changed = freq_changed or sr_changed
        frequency_diff = (self.last_frequency - frequency) if self.last_frequency is not None else 0
        self.last_frequency = frequency
        self.last_sample_rate = sample_rate
        if frequency_diff != 0:
            off = retune_shift_offset(frequency_diff, n, sample_rate)
            if abs(off) < n:
                if off < 0:  # shift left, fill right side
                    self.ring[:, : n + off] = self.ring[:, -off:].copy()
                    self.ring[:, n + off:] = RING_FILL
                else:  # shift right, fill left side
                    self.ring[:, off:] = self.ring[:, : n - off].copy()
                    self.ring[:, :off] = RING_FILL
            else:
                self.ring[:] = RING_FILL
        elif sr_changed:
            self.ring[:] = RING_FILL
        self.ring[self.write_index] = row
        self.read_index = self.write_index
        self.write_index = self.ring.shape[0] - 1 if self.write_index == 0 else self.write_index - 1
        if self.peak_hold:
            if self.peaks is None or self.peaks.size != n or self.freq_or_sr_changed:
                self.peaks = np.full(n, PEAK_FILL, np.float32)
            self.peaks = np.maximum(self.peaks, self.ring[self.read_index])
        else:
            self.peaks = None
        if self.ema_alpha is not None:
            if self.ema is None or self.ema.size != n or self.freq_or_sr_changed:
                self.ema = row.copy()
            else:
                reseed = ~(self.ema > -np.inf)
                upd = (self.ema + self.ema_alpha * (row - self.ema)).astype(np.float32)
                self.ema = np.where(reseed, row, upd).astype(np.float32)

    def boxcar(self, length: int) -> np.ndarray:
        """AnalyzerSurface.kt:710-714 at bin resolution: float32 running sum of the
        newest length+1 rows (newest first), divided by (length+1)."""
        acc = np.zeros(self.n, np.float32)
        rows = self.ring.shape[0]
        for r in range(length + 1):
            acc = (acc + self.ring[(self.read_index + r) % rows]).astype(np.float32)
        return (acc / np.float32(length + 1)).astype(np.float32)


def ema_batch(rows: np.ndarray, alpha: float, init: np.ndarray | None = None) -> np.ndarray:
    """EMA over rows in order (extension semantics above)."""
    a = np.float32(alpha)
    ema = None if init is None else np.asarray(init, np.float32).copy()
    for row in rows:
        if ema is None:
            ema = row.astype(np.float32).copy()
            continue
        reseed = ~(ema > -np.inf)
        upd = (ema + a * (row - ema)).astype(np.float32)
        ema = np.where(reseed, row, upd).astype(np.float32)
    return ema


def file_frames(n_bytes: int, packet_size: int, bytes_per_sample: int, n: int) -> list[tuple[int, int]]:
    """Frames a headerless IQ file is cut into by FileIQSource + Scheduler.

    FileIQSource.getPacket (FileIQSource.java:326-346) yields only FULL packets
    of `packet_size` bytes (a short tail at EOF is dropped).  The Scheduler FFT
    branch (Scheduler.kt:252-279 with IQConverter.fill*, e.g.
    Signed8BitIQConverter.java:80-99) appends samples from consecutive packets
    into an N-sample buffer, dropping the remainder of the packet that
    completes it, then starts the next buffer at the next packet (lossless
    mode: the consumer never back-pressures).  Returns, per frame, the list of
    (byte_offset, n_samples) pieces, flattened to (offset of first piece,
    contiguous flag) only when N <= packet samples.
    """
    ps = packet_size // bytes_per_sample
    n_packets = n_bytes // packet_size
    frames = []
    p = 0
    if n <= ps:
        for p in range(n_packets):
            frames.append((p * packet_size, n))
        return frames
    per = -(-n // ps)  # ceil
    while p + per <= n_packets:
        frames.append((p * packet_size, n))  # contiguous: whole packets concatenated
        p += per
    return frames


def channel_mean(row: np.ndarray, n: int, frequency: int, sample_rate: int, start: int, end: int):
    """FftProcessor.kt:143-157: mean dB over the channel's bins (None if empty).
    Index math in float32 with Kotlin's truncating toInt(), coerceIn(0, N);
    sequential float32 sum like the reference loop."""
    samples_per_hz = np.float32(n) / np.float32(sample_rate)
    f0 = frequency - sample_rate // 2

    def idx(f):
        return min(max(kotlin_float_to_int(np.float32(np.float32(f - f0) * samples_per_hz)), 0), n)

    s, e = idx(start), idx(end)
    if e <= s:
        return None
    acc = np.float32(0)
    for v in np.asarray(row[s:e], np.float32):
        acc = np.float32(acc + v)
    return np.float32(acc / np.float32(e - s))


def scheduler_frames(packets, n: int, bytes_per_sample: int):
    """Scheduler.run's FFT branch restated literally (Scheduler.kt:252-273 with
    fillPacketIntoSamplePacket, Signed8BitIQConverter.java:80-98): one buffer of
    N samples filled packet after packet from each packet's start, delivered when
    full, the rest of the completing packet dropped; the buffer takes the
    frequency / sample rate of every packet that fills it (the last one wins).
    packets: iterable of (bytes, frequency, sample_rate).  Returns a list of
    (frame_bytes, frequency, sample_rate), one per delivered frame."""
    out = []
    buf = bytearray()
    size = 0
    freq = rate = None
    for data, f, r in packets:
        if size >= n:  # never: a full buffer is delivered at once
            continue
        count = 0
        i = 0
        while i + bytes_per_sample <= len(data):
            buf += data[i:i + bytes_per_sample]
            count += 1
            i += bytes_per_sample
            if size + count >= n:
                break
        size += count
        freq, rate = f, r
        if size == n:
            out.append((bytes(buf), freq, rate))
            buf = bytearray()
            size = 0
    return out
