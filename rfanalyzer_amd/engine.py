"""SpectrumEngine: Python face of one librfa handle.

One engine = one reference ``FftProcessor`` + ``NativeDsp`` pair
(analyzer/FftProcessor.kt:64-257, nativedsp/.../NativeDsp.kt) living on one
GPU: raw IQ frames in, waterfall rows out, with the ring, peak-hold and
averaging state kept in HBM.  All compute runs in librfa's HIP kernels.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib
from ._lib import AVG_MODES, BYTES_PER_SAMPLE, FORMATS, WINDOWS, RfaConfig, check

_fp = ctypes.POINTER(ctypes.c_float)


def _fptr(a: np.ndarray):
    assert a.dtype == np.float32 and a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(_fp)


def _as_u8(data) -> np.ndarray:
    if isinstance(data, np.ndarray):
        return np.ascontiguousarray(data).reshape(-1).view(np.uint8)
    return np.frombuffer(memoryview(data).cast("B"), dtype=np.uint8)


class SpectrumEngine:
    def __init__(self, fft_size: int, window: str = "blackman", input_format: str = "s8", avg: str = "none",
                 avg_length: int = 0, ema_alpha: float = 0.1, peak_hold: bool = False, ring_rows: int = 400,
                 device: int = 0):
        cfg = RfaConfig()
        _lib.lib().rfa_default_config(ctypes.byref(cfg))
        cfg.fft_size = fft_size
        cfg.window = WINDOWS[window] if isinstance(window, str) else int(window)
        cfg.input_format = FORMATS[input_format] if isinstance(input_format, str) else int(input_format)
        cfg.avg_mode = AVG_MODES[avg] if isinstance(avg, str) else int(avg)
        cfg.avg_length = avg_length
        cfg.ema_alpha = ema_alpha
        cfg.peak_hold = 1 if peak_hold else 0
        cfg.ring_rows = ring_rows
        cfg.device_id = device
        self.cfg = cfg
        self.n = fft_size
        self.fmt = cfg.input_format
        self.bps = BYTES_PER_SAMPLE[self.fmt]
        h = ctypes.c_void_p()
        check(_lib.lib().rfa_create(ctypes.byref(cfg), ctypes.byref(h)), "rfa_create")
        self._h = h

    # -- lifetime ---------------------------------------------------------------
    def close(self) -> None:
        if getattr(self, "_h", None):
            _lib.lib().rfa_destroy(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001
            pass

    @property
    def handle(self):
        return self._h

    def _check(self, status: int, where: str) -> None:
        check(status, where, self._h)

    # -- processing -------------------------------------------------------------
    def frames_in(self, n_bytes: int, frame_stride: int = 0) -> int:
        fb = self.n * self.bps
        stride = frame_stride or fb
        return 0 if n_bytes < fb else (n_bytes - fb) // stride + 1

    def process(self, data, n_frames: int | None = None, frame_stride: int = 0, rows: bool = True):
        """Host bytes/ndarray in -> (n_frames, N) float32 rows (or None)."""
        buf = _as_u8(data)
        if n_frames is None:
            n_frames = self.frames_in(buf.size, frame_stride)
        stride = frame_stride or self.n * self.bps
        need = (n_frames - 1) * stride + self.n * self.bps if n_frames else 0
        if buf.size < need:
            raise ValueError(f"input has {buf.size} bytes, {need} needed for {n_frames} frames")
        out = np.empty((n_frames, self.n), np.float32) if rows else None
        self._check(_lib.lib().rfa_process_host(self._h, buf.ctypes.data, n_frames, frame_stride,
                                                out.ctypes.data if rows else None), "rfa_process_host")
        return out

    def process_batches(self, in_ptr: int, n_batches: int, batch_stride: int, frames_per_batch: int,
                        frame_stride: int = 0, rows_ptr: int | None = None) -> None:
        """rfa_process_batches: n_batches consecutive rfa_process calls in one enqueue
        (one kernel launch when the batches are packed).  Device pointers, async."""
        self._check(_lib.lib().rfa_process_batches(self._h, in_ptr, n_batches, batch_stride, frames_per_batch,
                                                   frame_stride, rows_ptr), "rfa_process_batches")

    def push_packet(self, packet, frequency: int, sample_rate: int, row: bool = False):
        """One raw packet through the reference's framing (rfa_push_packet,
        Scheduler.kt:252-273): fills the partial frame, processes it once complete.
        Returns the completed frame's row (row=True) / True, or None / False."""
        buf = _as_u8(packet)
        out = np.empty(self.n, np.float32) if row else None
        got = ctypes.c_int32(0)
        self._check(_lib.lib().rfa_push_packet(self._h, buf.ctypes.data if buf.size else None, buf.size,
                                               int(frequency), int(sample_rate),
                                               out.ctypes.data if row else None, ctypes.byref(got)),
                    "rfa_push_packet")
        if row:
            return out if got.value else None
        return bool(got.value)

    def pending_samples(self) -> int:
        v = ctypes.c_int64(0)
        self._check(_lib.lib().rfa_pending_samples(self._h, ctypes.byref(v)), "rfa_pending_samples")
        return v.value

    def state_generation(self) -> int:
        v = ctypes.c_int64(0)
        self._check(_lib.lib().rfa_get_state_generation(self._h, ctypes.byref(v)), "rfa_get_state_generation")
        return v.value

    def process_device(self, in_ptr: int, n_frames: int, frame_stride: int = 0, rows_ptr: int | None = None) -> None:
        """Device pointers (e.g. torch .data_ptr()); asynchronous on the engine stream."""
        self._check(_lib.lib().rfa_process(self._h, in_ptr, n_frames, frame_stride, rows_ptr), "rfa_process")

    def process_tensor(self, t, n_frames: int | None = None, frame_stride: int = 0, rows=None) -> None:
        """torch.cuda tensors (uint8/int8/float32 input, float32 rows).  Enqueued on torch's
        current stream: ordered after the op that produced ``t`` and before later torch ops
        that read ``rows``.  Import torch before this package when mixing the two: torch's
        wheel bundles its own libamdhip64.so; loaded first, librfa binds to that same
        runtime, loaded second it finds the system one already mapped and torch sees no GPU."""
        import torch

        cur = torch.cuda.current_stream(t.device).cuda_stream
        if cur != getattr(self, "_torch_stream", None):
            self.set_stream(cur)
        nbytes = t.numel() * t.element_size()
        if n_frames is None:
            n_frames = self.frames_in(nbytes, frame_stride)
        self.process_device(t.data_ptr(), n_frames, frame_stride, rows.data_ptr() if rows is not None else None)

    def set_stream(self, stream_ptr: int | None) -> None:
        """Enqueue on exactly this hipStream_t (0/None = HIP null stream)."""
        self._check(_lib.lib().rfa_set_stream(self._h, stream_ptr or None), "rfa_set_stream")
        self._torch_stream = stream_ptr or None

    def use_own_stream(self) -> None:
        self._check(_lib.lib().rfa_use_own_stream(self._h), "rfa_use_own_stream")
        self._torch_stream = None

    def synchronize(self) -> None:
        self._check(_lib.lib().rfa_synchronize(self._h), "rfa_synchronize")

    def set_pipelined(self, state_cus: int) -> None:
        """rfa_set_pipelined: the peak / EMA pass of call k on `state_cus` reserved CUs under
        call k + 1's FFT (0: off).  The handle stream is then ordered after a call only by
        join() (or synchronize() / any other entry point)."""
        self._check(_lib.lib().rfa_set_pipelined(self._h, int(state_cus)), "rfa_set_pipelined")

    def join(self) -> None:
        """rfa_join: order the handle stream after every pipelined call so far."""
        self._check(_lib.lib().rfa_join(self._h), "rfa_join")

    # -- FftProcessor state -----------------------------------------------------
    def set_tuning(self, frequency: int, sample_rate: int) -> None:
        self._check(_lib.lib().rfa_set_tuning(self._h, int(frequency), int(sample_rate)), "rfa_set_tuning")

    def peaks(self) -> np.ndarray:
        out = np.empty(self.n, np.float32)
        self._check(_lib.lib().rfa_get_peaks(self._h, _fptr(out)), "rfa_get_peaks")
        return out

    def ema(self) -> np.ndarray:
        out = np.empty(self.n, np.float32)
        self._check(_lib.lib().rfa_get_ema(self._h, _fptr(out)), "rfa_get_ema")
        return out

    def boxcar(self, length: int | None = None) -> np.ndarray:
        out = np.empty(self.n, np.float32)
        length = self.cfg.avg_length if length is None else length
        self._check(_lib.lib().rfa_get_boxcar(self._h, length, _fptr(out)), "rfa_get_boxcar")
        return out

    def ring(self):
        self._sync_config()  # a pending ring resize lands with the next batch
        out = np.empty((self.cfg.ring_rows, self.n), np.float32)
        ri, wi = ctypes.c_int32(), ctypes.c_int32()
        self._check(_lib.lib().rfa_get_ring(self._h, _fptr(out), ctypes.byref(ri), ctypes.byref(wi)),
                    "rfa_get_ring")
        return out, ri.value, wi.value

    @property
    def ring_order(self) -> int:
        """Residues RS of the device ring's storage order (rfa_get_ring_order); ``ring()``
        always returns natural rows."""
        rs = ctypes.c_int32()
        self._check(_lib.lib().rfa_get_ring_order(self._h, ctypes.byref(rs)), "rfa_get_ring_order")
        return rs.value

    def ring_positions(self) -> np.ndarray:
        """Storage position of every fft-shifted bin in a device ring row (rfa_get_ring_positions)."""
        out = np.empty(self.n, np.int32)
        self._check(_lib.lib().rfa_get_ring_positions(self._h, out.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)),
                                                      self.n), "rfa_get_ring_positions")
        return out

    def reset_state(self) -> None:
        self._check(_lib.lib().rfa_reset_state(self._h), "rfa_reset_state")

    def set_ring_rows(self, ring_rows: int) -> None:
        """Waterfall speed change (FftProcessor.kt:185-195): applied with the next frame, history kept."""
        self._check(_lib.lib().rfa_set_ring_rows(self._h, int(ring_rows)), "rfa_set_ring_rows")

    def set_fft_size(self, fft_size: int) -> None:
        """FFT size change (FftProcessor.kt:178-183): ring, peaks and EMA start over at the new N."""
        self._check(_lib.lib().rfa_set_fft_size(self._h, int(fft_size)), "rfa_set_fft_size")
        self._sync_config()

    def _sync_config(self) -> None:
        _lib.lib().rfa_get_config(self._h, ctypes.byref(self.cfg))
        self.n = self.cfg.fft_size

    # -- reference seams (host arrays) ------------------------------------------
    def windowed_fft_mag(self, re: np.ndarray, im: np.ndarray, mag_out: np.ndarray) -> bool:
        """NativeDsp.performWindowedFftAndReturnMag (NativeDsp.kt:43-62)."""
        re = np.ascontiguousarray(re, np.float32)
        im = np.ascontiguousarray(im, np.float32)
        if im.size != re.size or mag_out.size != re.size:
            return False
        rc = _lib.lib().rfa_windowed_fft_mag_planar(self._h, _fptr(re), _fptr(im), _fptr(mag_out), re.size)
        if rc == _lib.RFA_ERR_SIZE:
            return False
        self._check(rc, "rfa_windowed_fft_mag_planar")
        return True

    def fft_logmag(self, interleaved: np.ndarray) -> np.ndarray:
        """JNI performFFTAndLogMag (nativedsp.cpp:44-81)."""
        x = np.ascontiguousarray(interleaved, np.float32)
        out = np.empty(x.size // 2, np.float32)
        self._check(_lib.lib().rfa_fft_logmag_interleaved(self._h, _fptr(x), _fptr(out), out.size),
                    "rfa_fft_logmag_interleaved")
        return out

    def fft_ordered(self, interleaved: np.ndarray) -> np.ndarray:
        """JNI performFFT (nativedsp.cpp:19-42)."""
        x = np.ascontiguousarray(interleaved, np.float32)
        out = np.empty_like(x)
        self._check(_lib.lib().rfa_fft_ordered(self._h, _fptr(x), _fptr(out), x.size // 2), "rfa_fft_ordered")
        return out

    # -- profiling --------------------------------------------------------------
    def set_profiling(self, on: bool) -> None:
        self._check(_lib.lib().rfa_set_profiling(self._h, 1 if on else 0), "rfa_set_profiling")

    def set_channel(self, start_frequency: int, end_frequency: int) -> None:
        """Channel range for the per-frame mean dB (FftProcessor.kt:143-157); equal ends disable it."""
        self._check(_lib.lib().rfa_set_channel(self._h, int(start_frequency), int(end_frequency)), "rfa_set_channel")

    def channel_means(self) -> np.ndarray:
        """Per-frame channel mean dB of the last batch (empty when the channel range is empty)."""
        cap = 1 << 16
        out = np.empty(cap, np.float32)
        cnt = ctypes.c_size_t()
        self._check(_lib.lib().rfa_get_channel_means(self._h, out.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), cap,
                                                     ctypes.byref(cnt)), "rfa_get_channel_means")
        return out[:min(cnt.value, cap)].copy()

    def draw_preprocess(self, width: int, fft_height: int, viewport_frequency: int, viewport_sample_rate: int,
                        min_db: float, max_db: float, average_length: int, colormap, peaks: bool = False):
        """AnalyzerSurface.drawPreprocessing (AnalyzerSurface.kt:599-743) on the device, from the ring.

        Like the reference's draw thread it refreshes only dirty rows plus the
        averaged ones (at most average_length + 6 per call, :678-684) and keeps
        the colour buffer between calls.  Returns (colors [ring_rows][width] uint32 ARGB in ring storage order,
        fft_path_y [width] (NaN where no path point), peaks_y [width] or None,
        (autoscale_min, autoscale_max))."""
        self._sync_config()
        cmap = np.ascontiguousarray(colormap, dtype=np.uint32)
        p = _lib.RfaDrawParams(int(width), int(fft_height), int(viewport_frequency), int(viewport_sample_rate),
                               float(min_db), float(max_db), int(average_length), int(cmap.size),
                               cmap.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)))
        colors = np.empty((self.cfg.ring_rows, int(width)), np.uint32)
        path = np.empty(int(width), np.float32)
        pk = np.empty(int(width), np.float32) if peaks else None
        mm = np.empty(2, np.float32)
        self._check(_lib.lib().rfa_draw_preprocess(self._h, ctypes.byref(p), colors.ctypes.data, _fptr(path),
                                                   _fptr(pk) if pk is not None else None, _fptr(mm)),
                    "rfa_draw_preprocess")
        return colors, path, pk, (float(mm[0]), float(mm[1]))

    def row_window_stats(self, lo, hi):
        """(peak, avg) float32 arrays over inclusive bin windows [lo, hi] of the newest ring row
        (MainViewModel.kt scanner / squelch reductions)."""
        lo = np.ascontiguousarray(lo, dtype=np.int32)
        hi = np.ascontiguousarray(hi, dtype=np.int32)
        if lo.shape != hi.shape:
            raise ValueError("lo and hi differ in length")
        pk = np.empty(lo.size, np.float32)
        av = np.empty(lo.size, np.float32)
        i32 = ctypes.POINTER(ctypes.c_int32)
        self._check(_lib.lib().rfa_row_window_stats(self._h, lo.ctypes.data_as(i32), hi.ctypes.data_as(i32), lo.size,
                                                    _fptr(pk), _fptr(av)), "rfa_row_window_stats")
        return pk, av

    def main_kernel_name(self) -> str:
        """HIP kernel that rfa_process launches for this configuration (rocprofv3 name)."""
        return _lib.lib().rfa_main_kernel_name(self._h).decode()

    def kernel_time(self):
        ms, n = ctypes.c_double(), ctypes.c_int64()
        self._check(_lib.lib().rfa_get_kernel_time(self._h, ctypes.byref(ms), ctypes.byref(n)),
                    "rfa_get_kernel_time")
        return ms.value, n.value


def seam_supported(n: int) -> bool:
    """True when the reference's pffft accepts N (pffft.c:1231-1280): a multiple of 16,
    N / 4 a product of 2, 3, 4, 5, N <= 2^26."""
    return bool(_lib.lib().rfa_seam_supported(int(n)))


class SeamPlan:
    """The reference seams at one length the streaming handle does not take (16, 32,
    2^21 .. 2^26, mixed 2/3/5 lengths): librfa's mixed-radix Stockham FFT on the GPU
    (csrc/fft_seam.hip), one plan per N like nativedsp.cpp:12-17's cached setup."""

    def __init__(self, n: int, device: int = 0):
        h = ctypes.c_void_p()
        check(_lib.lib().rfa_seam_create(int(n), int(device), ctypes.byref(h)), "rfa_seam_create")
        self._h = h
        self.n = int(n)

    def close(self) -> None:
        if getattr(self, "_h", None):
            _lib.lib().rfa_seam_destroy(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001
            pass

    def _check(self, status: int, where: str) -> None:
        if status != _lib.RFA_OK:
            raise _lib.RfaError(status, where, (_lib.lib().rfa_seam_last_error(self._h) or b"").decode())

    def plan(self) -> list[int]:
        """Pass radices, first pass first."""
        radices = (ctypes.c_int32 * 32)()
        cnt = ctypes.c_int32()
        self._check(_lib.lib().rfa_seam_get_plan(self._h, radices, 32, ctypes.byref(cnt)), "rfa_seam_get_plan")
        return list(radices[: cnt.value])

    def windowed_fft_mag(self, re: np.ndarray, im: np.ndarray, mag_out: np.ndarray) -> bool:
        """NativeDsp.performWindowedFftAndReturnMag (NativeDsp.kt:43-62)."""
        re = np.ascontiguousarray(re, np.float32)
        im = np.ascontiguousarray(im, np.float32)
        if im.size != re.size or mag_out.size != re.size:
            return False
        rc = _lib.lib().rfa_seam_windowed_fft_mag_planar(self._h, _fptr(re), _fptr(im), _fptr(mag_out), re.size)
        if rc == _lib.RFA_ERR_SIZE:
            return False
        self._check(rc, "rfa_seam_windowed_fft_mag_planar")
        return True

    def fft_logmag(self, interleaved: np.ndarray) -> np.ndarray:
        """JNI performFFTAndLogMag (nativedsp.cpp:44-81)."""
        x = np.ascontiguousarray(interleaved, np.float32)
        out = np.empty(x.size // 2, np.float32)
        self._check(_lib.lib().rfa_seam_fft_logmag_interleaved(self._h, _fptr(x), _fptr(out), out.size),
                    "rfa_seam_fft_logmag_interleaved")
        return out

    def fft_ordered(self, interleaved: np.ndarray) -> np.ndarray:
        """JNI performFFT (nativedsp.cpp:19-42)."""
        x = np.ascontiguousarray(interleaved, np.float32)
        out = np.empty_like(x)
        self._check(_lib.lib().rfa_seam_fft_ordered(self._h, _fptr(x), _fptr(out), x.size // 2),
                    "rfa_seam_fft_ordered")
        return out
