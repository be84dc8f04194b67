"""Host mirror of the reference's packet fan-out (analyzer/Scheduler.kt:140-298).

Every raw packet from the source goes, in the reference's order, to

1. the recording branch (``recording.RecordingWriter``: split before 4 GB, writes
   gated by the squelch with the 50-packet debounce, Scheduler.kt:161-234);
2. the demodulation branch, only while the squelch is satisfied or the debounce
   counter is below 50 (Scheduler.kt:237-250): ``demod.FrontEnd`` mixes the packet
   down to the channel and filters it to the quadrature rate on the GPU;
3. the FFT branch (Scheduler.kt:252-279): each packet fills the current FFT
   buffer, the rest of a packet is dropped, a full buffer becomes one frame.  Frames
   are batched and handed to ``SpectrumEngine.process`` with the equivalent byte
   stride (``source.frame_stride``), so the rows equal the reference's.

The reference drops packets when its FFT or demod thread falls behind (queue
back-pressure, Scheduler.kt:245-249,270-276); the GPU keeps up, so nothing is
dropped here and the batching only changes when rows appear, not their values.
"""
from __future__ import annotations

from . import recording, source

SQUELCH_DEBOUNCE_COUNT = recording.SQUELCH_DEBOUNCE_COUNT


class Scheduler:
    """One source's packets to recording / demod / FFT.  Branches are optional.

    ``engine``: a ``SpectrumEngine`` (FFT branch, rows kept in its ring and state);
    ``recorder``: a ``RecordingWriter``; ``frontend``: a ``demod.FrontEnd``.
    ``squelch_satisfied`` is set by the caller between packets, as MainViewModel
    does from the channel level.
    """

    def __init__(self, packet_size: int, bytes_per_sample: int, frequency: int = 0, engine=None, fft_batch: int = 64,
                 recorder=None, frontend=None, channel_frequency: int = 0, on_rows=None, on_demod=None):
        self.packet_size, self.bps = packet_size, bytes_per_sample
        self.frequency, self.channel_frequency = frequency, channel_frequency
        self.engine, self.recorder, self.frontend = engine, recorder, frontend
        self.fft_batch = fft_batch
        self.on_rows, self.on_demod = on_rows, on_demod
        self.squelch_satisfied = True
        self.debounce = 0                                   # squelchDebounceCounter (Scheduler.kt:77)
        self.demod_active = frontend is not None
        self._pending = bytearray()                         # whole packets not yet turned into frames
        self.packets = 0
        self.frames = 0

    # -- per packet (Scheduler.run loop body)
    def on_packet(self, packet: bytes) -> None:
        if len(packet) != self.packet_size:
            raise ValueError(f"packet of {len(packet)} bytes, expected {self.packet_size}")
        if self.squelch_satisfied:                           # Scheduler.kt:155-158
            self.debounce = 0
        elif self.debounce < SQUELCH_DEBOUNCE_COUNT:
            self.debounce += 1
        if self.recorder is not None:                         # recording branch
            self.recorder.write_packet(packet, self.squelch_satisfied)
        if self.demod_active and (self.squelch_satisfied or self.debounce < SQUELCH_DEBOUNCE_COUNT):
            re, im = self.frontend.process(packet, self.frequency, self.channel_frequency)
            if self.on_demod is not None:
                self.on_demod(re, im)
        if self.engine is not None:                           # FFT branch
            self._pending += packet
            stride = source.frame_stride(self.engine.n, self.packet_size, self.bps)
            if len(self._pending) >= stride * self.fft_batch:
                self._run_fft(len(self._pending) // stride)
        self.packets += 1

    def flush(self) -> None:
        """Turn every complete frame still pending into rows (end of stream)."""
        if self.engine is not None:
            stride = source.frame_stride(self.engine.n, self.packet_size, self.bps)
            if len(self._pending) >= stride:
                self._run_fft(len(self._pending) // stride)

    def _run_fft(self, n_frames: int) -> None:
        stride = source.frame_stride(self.engine.n, self.packet_size, self.bps)
        rows = self.engine.process(bytes(self._pending[:n_frames * stride]), n_frames, frame_stride=stride,
                                   rows=self.on_rows is not None)
        del self._pending[:n_frames * stride]
        self.frames += n_frames
        if self.on_rows is not None:
            self.on_rows(rows)

    def run(self, src, max_packets: int | None = None) -> None:
        """Pull packets from an ``IQSourceInterface``-like source (``getPacket``) until it
        returns None or ``max_packets`` were handled, then flush."""
        while max_packets is None or self.packets < max_packets:
            p = src.getPacket(1000)
            if p is None:
                break
            self.on_packet(p)
        self.flush()
