"""Seeded synthetic IQ captures (pure numpy, PCG64) shared by the golden
generator, the parity tests and bench.py.

Quantisation follows the reference converters in reverse so the bytes decode
to the intended float signal: s8 ``round(x*128)`` (Signed8BitIQConverter.java:48-50),
u8 ``round(x*128+127.4)`` (Unsigned8BitIQConverter.java:48-50), s16
``round(x*32768)`` (Signed16BitIQConverter.kt:52-55).
"""
from __future__ import annotations

import hashlib

import numpy as np

FORMATS = {"s8": 0, "u8": 1, "s16": 2, "f32": 3, "f32p": 4}


def _rng(seed: int) -> np.random.Generator:
    return np.random.Generator(np.random.PCG64(seed))


def complex_signal(n: int, seed: int, tones=((0.125, 0.5),), noise=0.05, drift=0.0) -> np.ndarray:
    """sum_k a_k exp(2j*pi*(f_k + drift*t) t) + complex AWGN(sigma=noise); f in cycles/sample."""
    rng = _rng(seed)
    t = np.arange(n, dtype=np.float64)
    x = np.zeros(n, np.complex128)
    for f, a in tones:
        phase = 2 * np.pi * (f * t + 0.5 * drift * t * t / max(n, 1))
        x += a * np.exp(1j * phase)
    if noise:
        x += noise * (rng.standard_normal(n) + 1j * rng.standard_normal(n)) / np.sqrt(2.0)
    return x


def quantize(x: np.ndarray, fmt: str) -> bytes:
    if fmt == "s8":
        iq = np.empty(2 * x.size, np.float64)
        iq[0::2], iq[1::2] = x.real, x.imag
        return np.clip(np.rint(iq * 128), -128, 127).astype(np.int8).tobytes()
    if fmt == "u8":
        iq = np.empty(2 * x.size, np.float64)
        iq[0::2], iq[1::2] = x.real, x.imag
        return np.clip(np.rint(iq * 128 + 127.4), 0, 255).astype(np.uint8).tobytes()
    if fmt == "s16":
        iq = np.empty(2 * x.size, np.float64)
        iq[0::2], iq[1::2] = x.real, x.imag
        return np.clip(np.rint(iq * 32768), -32768, 32767).astype("<i2").tobytes()
    if fmt == "f32":
        iq = np.empty(2 * x.size, np.float32)
        iq[0::2], iq[1::2] = x.real, x.imag
        return iq.tobytes()
    if fmt == "f32p":
        return np.concatenate([x.real.astype(np.float32), x.imag.astype(np.float32)]).tobytes()
    raise ValueError(fmt)


def frames_bytes(n: int, n_frames: int, fmt: str, seed: int, **kw) -> bytes:
    """n_frames consecutive frames of one continuous capture (f32p: planar per frame)."""
    x = complex_signal(n * n_frames, seed, **kw)
    if fmt == "f32p":
        return b"".join(quantize(x[f * n:(f + 1) * n], fmt) for f in range(n_frames))
    return quantize(x, fmt)


def kat_bytes(kind: str, n: int) -> bytes:
    """Known-answer frames (f32 interleaved)."""
    t = np.arange(n)
    if kind == "impulse":
        x = np.zeros(n, np.complex128); x[0] = 1.0
    elif kind == "dc":
        x = np.ones(n, np.complex128)
    elif kind == "nyquist":  # ApplicationTest.kt:292-321 (commented-out KAT): alternating sign
        x = np.where(t % 2 == 0, 1.0, -1.0).astype(np.complex128)
    elif kind == "tone_bin":
        x = 0.5 * np.exp(2j * np.pi * (n // 8 + 3) * t / n)
    elif kind == "tone_halfbin":
        x = 0.5 * np.exp(2j * np.pi * (n // 8 + 3.5) * t / n)
    elif kind == "zeros":
        return bytes(2 * n)  # s8 zeros
    else:
        raise ValueError(kind)
    return quantize(x, "f32")


def file_capture(n_bytes: int = 4_000_000, seed: int = 1, sample_rate: int = 2_000_000) -> bytes:
    """Config 1: 8-bit signed (HackRF) capture, tone at +250 kHz amp 0.5, AWGN 0.05."""
    ns = n_bytes // 2
    x = complex_signal(ns, seed, tones=((250_000 / sample_rate, 0.5),), noise=0.05)
    return quantize(x, "s8")[:n_bytes]


def sha256(b: bytes) -> str:
    return hashlib.sha256(b).hexdigest()
