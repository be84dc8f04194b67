"""Mirror of the reference's ``NativeDsp`` Kotlin class on top of librfa.

Reference: nativedsp/src/main/java/com/mantz_it/nativedsp/NativeDsp.kt.
Same method names, argument meaning and error behaviour:

* ``performWindowedFftAndReturnMag(re, im, magOut) -> bool`` (NativeDsp.kt:43-62):
  returns False on a length mismatch (:45-46), otherwise fills ``magOut`` with
  the Blackman-windowed, fft-shifted ``10*log10(|X|/N)`` row -- here computed
  in one fused HIP kernel instead of a JVM window loop + pffft + log loop.
* ``performFFTAndLogMag(input, output)`` / ``performFFT(input, output)``
  (the two ``external`` natives, NativeDsp.kt:27-28 -> nativedsp.cpp:19-81).

Every length the reference's pffft accepts works: powers of two from 64 to 2^20
run on a streaming handle's fused kernels, the rest (16, 32, 2^21 .. 2^26, mixed
2/3/5 lengths) on a mixed-radix plan (``engine.SeamPlan``).  A length pffft
rejects raises ``RfaError`` (RFA_ERR_UNSUPPORTED) where the reference asserts.

Like the reference (NativeDsp.kt:23-26) one instance is meant for one thread.
"""
from __future__ import annotations

import numpy as np

from .engine import SeamPlan, SpectrumEngine

# lengths rfa_create takes (include/rfa.h RFA_MIN_FFT_SIZE .. RFA_MAX_FFT_SIZE, powers of two)
_HANDLE_MIN, _HANDLE_MAX = 64, 1 << 20


class NativeDsp:
    def __init__(self, device: int = 0):
        self.device = device
        self._planar = None  # Blackman, f32 planar
        self._raw = None     # no window, f32 interleaved

    def _engine(self, kind: str, n: int) -> SpectrumEngine | SeamPlan:
        cur = self._planar if kind == "planar" else self._raw
        if cur is None or cur.n != n:  # nativedsp.cpp:56-64: new setup on a size change
            if cur is not None:
                cur.close()
            self._set(kind, None)
            if not (_HANDLE_MIN <= n <= _HANDLE_MAX and n & (n - 1) == 0):
                cur = SeamPlan(n, device=self.device)
            elif kind == "planar":
                cur = SpectrumEngine(n, "blackman", "f32p", ring_rows=0, device=self.device)
            else:
                cur = SpectrumEngine(n, "none", "f32", ring_rows=0, device=self.device)
            self._set(kind, cur)
        return cur

    def _set(self, kind: str, obj) -> None:
        if kind == "planar":
            self._planar = obj
        else:
            self._raw = obj

    def performWindowedFftAndReturnMag(self, re, im, magOut) -> bool:  # noqa: N802,N803 - reference name
        n = len(re)
        if len(im) != n or len(magOut) != n:
            return False
        out = np.empty(n, np.float32)
        ok = self._engine("planar", n).windowed_fft_mag(np.asarray(re, np.float32), np.asarray(im, np.float32), out)
        if ok:
            magOut[:] = out
        return ok

    def performFFTAndLogMag(self, input, output) -> None:  # noqa: A002,N802 - reference name
        x = np.asarray(input, np.float32)
        output[: x.size // 2] = self._engine("raw", x.size // 2).fft_logmag(x)

    def performFFT(self, input, output) -> None:  # noqa: A002,N802 - reference name
        x = np.asarray(input, np.float32)
        output[: x.size] = self._engine("raw", x.size // 2).fft_ordered(x)

    def close(self) -> None:
        for e in (self._planar, self._raw):
            if e is not None:
                e.close()
        self._planar = self._raw = None
