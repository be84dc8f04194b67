"""Mirror of the reference's spectrum consumer loop on top of librfa.

Reference: analyzer/FftProcessor.kt (class ``FftProcessor``, the "Analyzer
Processing Loop", and ``FftProcessorData``) and the load metric of
database/GlobalPerformanceData.kt.  The per-frame work of ``FftProcessor.run``
(:125-245) -- window + FFT + log-mag, channel mean, ring write, retune shift,
peak-hold -- runs on the GPU in one ``rfa_process`` call per batch; this class
keeps the reference's bookkeeping surface (queue-driven thread, metadata,
channel average callback, load EMA).
"""
from __future__ import annotations

import queue
import threading
import time

import numpy as np

from .engine import SpectrumEngine

WATERFALL_SPEED_ROWS = {"SLOW": 500, "NORMAL": 400, "FAST": 300}  # FftProcessor.kt:103


class GlobalPerformanceData:
    """EMA of per-block load, alpha = 0.05, first sample initialises (GlobalPerformanceData.kt:30-51)."""

    alpha = 0.05

    def __init__(self):
        self._loads: dict[str, float] = {}
        self._lock = threading.Lock()

    def updateLoad(self, id_: str, sample: float) -> None:  # noqa: N802
        if not np.isfinite(sample):
            return
        with self._lock:
            if id_ in self._loads:
                self._loads[id_] += self.alpha * (sample - self._loads[id_])
            else:
                self._loads[id_] = float(sample)

    def getLoad(self, id_: str) -> float:  # noqa: N802
        with self._lock:
            return self._loads.get(id_, 0.0)


class FftProcessorData:
    """Read side of the shared waterfall state (FftProcessor.kt:43-61), device-backed."""

    def __init__(self, engine: SpectrumEngine):
        self.lock = threading.RLock()
        self._engine = engine
        self.frequency = None
        self.sampleRate = None  # noqa: N815
        self.frequencyOrSampleRateChanged = True  # noqa: N815

    def waterfall(self):
        """(ring rows, readIndex, writeIndex) copied from HBM."""
        with self.lock:
            return self._engine.ring()

    def peaks(self):
        with self.lock:
            return self._engine.peaks() if self._engine.cfg.peak_hold else None


class FftProcessor:
    def __init__(self, fft_size: int, input_format: str = "s8", waterfall_speed: str = "NORMAL",
                 fft_peak_hold: bool = False, window: str = "blackman", avg: str = "none", avg_length: int = 0,
                 ema_alpha: float = 0.1, device: int = 0, channel_range=None, on_average_signal_strength=None,
                 performance: GlobalPerformanceData | None = None):
        self.engine = SpectrumEngine(fft_size, window, input_format, avg, avg_length, ema_alpha, fft_peak_hold,
                                     WATERFALL_SPEED_ROWS[waterfall_speed], device)
        self.data = FftProcessorData(self.engine)
        self.n = fft_size
        self.channel_range = channel_range
        self.on_average_signal_strength = on_average_signal_strength
        self.perf = performance or GlobalPerformanceData()
        self.input_queue: queue.Queue = queue.Queue(maxsize=2)  # FFT_QUEUE_SIZE, Scheduler.kt:50
        self._stop = True
        self._thread = None

    def process(self, frames, frequency: int, sample_rate: int, frame_stride: int = 0):
        """One batch of raw frames with common tuning -> rows (n_frames, N)."""
        t0 = time.perf_counter_ns()
        rng = self.channel_range() if (self.channel_range and self.on_average_signal_strength) else None
        self.engine.set_channel(*(rng if rng else (0, 0)))
        with self.data.lock:
            changed = frequency != self.data.frequency or sample_rate != self.data.sampleRate
            self.engine.set_tuning(frequency, sample_rate)
            rows = self.engine.process(frames, frame_stride=frame_stride)
            self.data.frequency, self.data.sampleRate = frequency, sample_rate
            self.data.frequencyOrSampleRateChanged = changed
        if rows.shape[0] and rng:
            for mean in self.engine.channel_means():  # one value per frame, as the reference's per-frame callback
                self.on_average_signal_strength(float(mean))
        # Load metric on every frame, channel range or not (FftProcessor.kt:159-161): the
        # batch's processing time is shared equally by its frames, and the EMA advances
        # once per frame as the reference's per-frame call does.
        if rows.shape[0]:
            ns_per_frame = self.n * 1e9 / sample_rate
            sample = (time.perf_counter_ns() - t0) / (ns_per_frame * rows.shape[0])
            for _ in range(rows.shape[0]):
                self.perf.updateLoad("FftProcessor", sample)
        return rows

    def setWaterfallSpeed(self, speed: str) -> None:  # noqa: N802
        """waterfallSpeed (FftProcessor.kt:79,185-195): ring of 500/400/300 rows, history kept,
        applied with the next frame."""
        self.engine.set_ring_rows(WATERFALL_SPEED_ROWS[speed])

    def setFftSize(self, fft_size: int) -> None:  # noqa: N802
        """A source packet of another size (FftProcessor.kt:136-139,178-183): fresh ring, peaks, EMA."""
        with self.data.lock:
            self.engine.set_fft_size(fft_size)
            self.n = fft_size

    # -- thread form (FftProcessor.kt:84-96,106-123) --------------------------------
    def start(self) -> None:
        self._stop = False
        self._thread = threading.Thread(target=self.run, name=f"Thread-FftProcessor-{int(time.time() * 1000)}",
                                        daemon=True)
        self._thread.start()

    def stopLoop(self) -> None:  # noqa: N802
        self._stop = True

    def run(self) -> None:
        while not self._stop:
            try:
                item = self.input_queue.get(timeout=0.016)  # FftProcessor.kt:111
            except queue.Empty:
                continue
            if item is None or self._stop:
                break
            frames, frequency, sample_rate = item
            self.process(frames, frequency, sample_rate)
        self._stop = True

    def join(self, timeout=None) -> None:
        if self._thread:
            self._thread.join(timeout)

    def close(self) -> None:
        self.stopLoop()
        self.join(1.0)
        self.engine.close()
