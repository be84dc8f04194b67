"""TEST INFRASTRUCTURE ONLY -- CPU parity oracle for the RFAnalyzer spectrum path.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import this package.  The product (``rfanalyzer_amd``) never does: it
runs on the HIP extension or fails loudly.

Two checkers live here:

* ``liborc.so`` (``rfa_oracle.c``): our C restatement -- LUT converters,
  Blackman/Hann window, float64 FFT, log-mag + fft-shift.
* ``_ref/libpffft_ref.so`` (``ref_harness.c`` + the reference's own
  ``pffft.c`` compiled from ``/root/reference``): the real reference FFT, used
  to pin the restatement and to generate ``tests/golden`` fixtures.  It may be
  absent on a machine without the reference tree or the prebuilt .so.

``processor.py`` restates the FftProcessor state machine (ring, retune shift,
peak-hold), the AnalyzerSurface boxcar and the EMA extension in numpy.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ORC_PATH = os.path.join(HERE, "liborc.so")
REF_PATH = os.path.join(HERE, "_ref", "libpffft_ref.so")
# diagnostic only: the same pffft.c with exact (double-angle) twiddle tables, exact_twiddle.c
EXACT_PATH = os.path.join(HERE, "_ref", "libpffft_exact.so")

IN_S8, IN_U8, IN_S16LE, IN_F32_INTERLEAVED, IN_F32_PLANAR = range(5)
WIN_BLACKMAN, WIN_HANN, WIN_NONE = range(3)
BYTES_PER_SAMPLE = {IN_S8: 2, IN_U8: 2, IN_S16LE: 4, IN_F32_INTERLEAVED: 8, IN_F32_PLANAR: 8}

_orc = None
_ref = None
_exact = None

_fp = ctypes.POINTER(ctypes.c_float)


def build() -> None:
    """Compile liborc.so (and _ref when the reference tree is present)."""
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def orc() -> ctypes.CDLL:
    global _orc
    if _orc is None:
        if not os.path.exists(ORC_PATH):
            build()
        lib = ctypes.CDLL(ORC_PATH)
        lib.orc_window.argtypes = [ctypes.c_int, ctypes.c_int, _fp]
        lib.orc_spectrum_rows.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t, ctypes.c_size_t,
                                          ctypes.c_size_t, _fp, _fp]
        lib.orc_convert.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t, _fp, _fp]
        lib.orc_ddc_process.restype = ctypes.c_size_t
        lib.orc_ddc_process.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t, _fp, _fp, ctypes.c_int, _fp,
                                        ctypes.c_int, ctypes.c_int, _fp, _fp, ctypes.POINTER(ctypes.c_int32), _fp, _fp]
        _orc = lib
    return _orc


def ref_available() -> bool:
    return os.path.exists(REF_PATH)


def ref() -> ctypes.CDLL:
    global _ref
    if _ref is None:
        if not os.path.exists(REF_PATH):
            raise FileNotFoundError(f"{REF_PATH} missing (reference pffft not built)")
        lib = ctypes.CDLL(REF_PATH)
        lib.ref_fft_ordered.argtypes = [_fp, ctypes.c_int, _fp]
        lib.ref_fft_logmag.argtypes = [_fp, ctypes.c_int, _fp]
        lib.ref_loop.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_long, _fp,
                                 _fp, ctypes.c_int, _fp]
        _ref = lib
    return _ref


def exact_available() -> bool:
    return os.path.exists(EXACT_PATH)


def exact() -> ctypes.CDLL:
    """The reference's pffft with its twiddle tables recomputed from exact angles (a diagnostic
    of pffft's own float-argument twiddles, pffft.c:1140,1156,1160-1161,1261; never the oracle)."""
    global _exact
    if _exact is None:
        if not os.path.exists(EXACT_PATH):
            raise FileNotFoundError(f"{EXACT_PATH} missing (reference pffft not built)")
        lib = ctypes.CDLL(EXACT_PATH)
        lib.exact_fft_ordered.argtypes = [_fp, ctypes.c_int, _fp]
        lib.exact_fft_logmag.argtypes = [_fp, ctypes.c_int, _fp]
        lib.exact_max_change.restype = ctypes.c_double
        _exact = lib
    return _exact


def _f32ptr(a: np.ndarray):
    assert a.dtype == np.float32 and a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(_fp)


def window(n: int, kind: int = WIN_BLACKMAN) -> np.ndarray:
    """NativeDsp.kt:14-21 (Blackman, double then cast to float)."""
    w = np.empty(n, np.float32)
    if orc().orc_window(n, kind, _f32ptr(w)) != 0:
        raise ValueError("bad window")
    return w


def convert(frame: np.ndarray, fmt: int, n: int):
    """IQ converter fill loops -> planar (re, im) float32."""
    buf = np.ascontiguousarray(frame)
    re = np.empty(n, np.float32)
    im = np.empty(n, np.float32)
    if orc().orc_convert(buf.ctypes.data, fmt, n, _f32ptr(re), _f32ptr(im)) != 0:
        raise ValueError("bad format")
    return re, im


def spectrum_rows(data, fmt: int, n: int, n_frames: int, frame_stride_bytes: int | None = None,
                  win: int | np.ndarray | None = WIN_BLACKMAN) -> np.ndarray:
    """float64-FFT oracle: convert -> window (fp32 mul) -> FFT -> log-mag + shift."""
    buf = np.ascontiguousarray(np.frombuffer(memoryview(data).cast("B"), dtype=np.uint8))
    if frame_stride_bytes is None:
        frame_stride_bytes = n * BYTES_PER_SAMPLE[fmt]
    need = (n_frames - 1) * frame_stride_bytes + n * BYTES_PER_SAMPLE[fmt] if n_frames else 0
    if buf.size < need:
        raise ValueError("input too small")
    if win is None:
        wptr = None
    else:
        w = window(n, win) if isinstance(win, int) else np.ascontiguousarray(win, np.float32)
        wptr = _f32ptr(w)
    out = np.empty((n_frames, n), np.float32)
    rc = orc().orc_spectrum_rows(buf.ctypes.data, fmt, n, n_frames, frame_stride_bytes, wptr, _f32ptr(out))
    if rc != 0:
        raise ValueError("oracle failed")
    return out


def windowed_interleaved(re: np.ndarray, im: np.ndarray, w: np.ndarray) -> np.ndarray:
    """NativeDsp.kt:55-58: inputBuf[2i]=re[i]*w[i], inputBuf[2i+1]=im[i]*w[i] (fp32)."""
    out = np.empty(2 * re.size, np.float32)
    out[0::2] = re.astype(np.float32) * w
    out[1::2] = im.astype(np.float32) * w
    return out


def ref_fft_logmag(interleaved: np.ndarray) -> np.ndarray:
    """Reference pffft + nativedsp.cpp:72-79 on one windowed interleaved frame."""
    x = np.ascontiguousarray(interleaved, np.float32)
    n = x.size // 2
    out = np.empty(n, np.float32)
    if ref().ref_fft_logmag(_f32ptr(x), n, _f32ptr(out)) != 0:
        raise ValueError("pffft setup failed")
    return out


def ref_fft_ordered(interleaved: np.ndarray) -> np.ndarray:
    x = np.ascontiguousarray(interleaved, np.float32)
    out = np.empty_like(x)
    if ref().ref_fft_ordered(_f32ptr(x), x.size // 2, _f32ptr(out)) != 0:
        raise ValueError("pffft setup failed")
    return out


def ref_spectrum_rows(data, fmt: int, n: int, n_frames: int, frame_stride_bytes: int | None = None,
                      win: int | np.ndarray | None = WIN_BLACKMAN, exact_twiddles: bool = False) -> np.ndarray:
    """Same as spectrum_rows but with the reference's own pffft as the FFT (exact_twiddles: the
    diagnostic build whose twiddle tables come from exact angles, exact_twiddle.c)."""
    buf = np.frombuffer(memoryview(data).cast("B"), dtype=np.uint8)
    bps = BYTES_PER_SAMPLE[fmt]
    if frame_stride_bytes is None:
        frame_stride_bytes = n * bps
    if win is None:
        w = np.ones(n, np.float32)
    else:
        w = window(n, win) if isinstance(win, int) else np.ascontiguousarray(win, np.float32)
    out = np.empty((n_frames, n), np.float32)
    for f in range(n_frames):
        frame = buf[f * frame_stride_bytes: f * frame_stride_bytes + n * bps]
        re, im = convert(frame, fmt, n)
        x = windowed_interleaved(re, im, w)
        if exact_twiddles:
            if exact().exact_fft_logmag(_f32ptr(x), n, _f32ptr(out[f])) != 0:
                raise ValueError("exact-twiddle pffft setup failed")
        else:
            out[f] = ref_fft_logmag(x)
    return out
