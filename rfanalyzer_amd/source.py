"""Host-side IQ sources and framing, mirroring the reference's source layer.

* ``SamplePacket``      source/SamplePacket.java:28-168 (planar re/im + metadata)
* ``FileIQSource``      source/FileIQSource.java: headerless file replay in
                        fixed packets (init :64-91, getPacket :318-369); full
                        packets only, EOF -> error or rewind when ``repeat``.
                        Pacing to the sample rate (:349-360) is optional
                        (``paced=False`` replays as fast as possible).
* ``frame_stride``      Scheduler.kt:252-279: which bytes of the packet stream
                        become FFT frames (one frame per packet, rest dropped,
                        or ceil(N/P) packets concatenated for N > P).

No sample conversion happens here: raw bytes go to the GPU, where the
converter LUT (Signed8BitIQConverter.java:48-50 etc.) is fused into the FFT
kernel.
"""
from __future__ import annotations

import os
import time

import numpy as np

FILE_FORMAT_8BIT_SIGNED = 0    # HackRF  -> rfa s8
FILE_FORMAT_8BIT_UNSIGNED = 1  # RTL-SDR -> rfa u8
FILE_FORMAT_16BIT_SIGNED = 2   # Airspy / HydraSDR -> rfa s16
RFA_FORMAT = {FILE_FORMAT_8BIT_SIGNED: "s8", FILE_FORMAT_8BIT_UNSIGNED: "u8", FILE_FORMAT_16BIT_SIGNED: "s16"}


class SamplePacket:
    def __init__(self, size: int):
        self._re = np.zeros(size, np.float32)
        self._im = np.zeros(size, np.float32)
        self.frequency = 0
        self.sampleRate = 0  # noqa: N815 - reference field name
        self._size = 0

    def re(self) -> np.ndarray:
        return self._re

    def im(self) -> np.ndarray:
        return self._im

    def capacity(self) -> int:
        return self._re.size

    def size(self) -> int:
        return self._size

    def setSize(self, size: int) -> None:  # noqa: N802
        self._size = min(size, self._re.size)  # SamplePacket.java:135-137


class FileIQSource:
    """Headerless IQ file replay (FileIQSource.java)."""

    def __init__(self):
        self.path = None
        self.stream = None
        self.error = None

    def init(self, path: str, sample_rate: int, frequency: int, packet_size: int = 1024 * 256, repeat: bool = False,
             file_format: int = FILE_FORMAT_8BIT_SIGNED, paced: bool = False) -> bool:
        self.path, self.sampleRate, self.frequency = path, sample_rate, frequency
        self.packetSize, self.repeat, self.fileFormat, self.paced = packet_size, repeat, file_format, paced
        self.buffer = bytearray(packet_size)
        self.bytesRead = 0
        return True

    def getBytesPerSample(self) -> int:  # noqa: N802 - FileIQSource.java:305-316
        return 4 if self.fileFormat == FILE_FORMAT_16BIT_SIGNED else 2

    def getPacketSize(self) -> int:  # noqa: N802
        return self.packetSize

    def rfa_format(self) -> str:
        return RFA_FORMAT[self.fileFormat]

    def open(self) -> bool:
        if not os.path.exists(self.path):
            self.error = "file not found"
            return False
        self.stream = open(self.path, "rb")  # noqa: SIM115
        self.startTime = time.monotonic_ns()
        return True

    def close(self) -> None:
        if self.stream:
            self.stream.close()
        self.stream = None

    def getPacket(self, timeout_ms: int = 1000):  # noqa: N802 - FileIQSource.java:318-369
        if self.stream is None:
            return None
        n = self.stream.readinto(self.buffer)
        if n != len(self.buffer):
            if not self.repeat:
                self.error = "End of File"
                return None
            self.stream.close()
            self.stream = open(self.path, "rb")  # noqa: SIM115 - rewind
            if self.stream.readinto(self.buffer) != len(self.buffer):
                self.error = "End of File"
                return None
        self.bytesRead += len(self.buffer)
        if self.paced:
            expected = self.startTime + int(1e9 / self.sampleRate * self.bytesRead / self.getBytesPerSample())
            sleep = min(expected - time.monotonic_ns(), timeout_ms * 1_000_000)
            if sleep > 0:
                time.sleep(sleep / 1e9)
        return bytes(self.buffer)

    def returnPacket(self, packet) -> None:  # noqa: N802
        pass


def frame_stride(fft_size: int, packet_size: int, bytes_per_sample: int) -> int:
    """Byte distance between consecutive FFT frames in a replayed packet stream
    (Scheduler.kt:252-279 with IQConverter.fill*, lossless: no back-pressure drops)."""
    ps = packet_size // bytes_per_sample
    per = max(1, -(-fft_size // ps))
    return per * packet_size


def file_frames(n_bytes: int, fft_size: int, packet_size: int, bytes_per_sample: int) -> int:
    """Number of frames a file yields: only whole packets are read (FileIQSource.java:326)."""
    n_packets = n_bytes // packet_size
    per = frame_stride(fft_size, packet_size, bytes_per_sample) // packet_size
    return n_packets // per
