"""ctypes binding of librfa.so (include/rfa.h).

The library is built in-tree (``python -m rfanalyzer_amd.build`` or
``__graft_entry__.build()``).  There is no CPU fallback anywhere in this
package: if the library is missing or no HIP device is visible, calls raise.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
# RFA_LIB: load an alternative build (A/B experiments, scripts/); default in-tree librfa.so
LIB_PATH = os.environ.get("RFA_LIB") or os.path.join(HERE, "librfa.so")
CSRC = os.path.join(HERE, "csrc")

RFA_OK = 0
RFA_ERR_INVALID = -1
RFA_ERR_SIZE = -2
RFA_ERR_UNSUPPORTED = -3
RFA_ERR_NODEVICE = -4
RFA_ERR_NOMEM = -5
RFA_ERR_HIP = -6
RFA_ERR_STATE = -7

WINDOWS = {"blackman": 0, "hann": 1, "none": 2}
FORMATS = {"s8": 0, "u8": 1, "s16": 2, "f32": 3, "f32p": 4}
BYTES_PER_SAMPLE = {0: 2, 1: 2, 2: 4, 3: 8, 4: 8}
AVG_MODES = {"none": 0, "boxcar": 1, "ema": 2}


class RfaError(RuntimeError):
    def __init__(self, status: int, where: str, detail: str = ""):
        self.status = status
        msg = f"{where}: {status_string(status)} ({status})"
        if detail:
            msg += f": {detail}"
        super().__init__(msg)


class RfaConfig(ctypes.Structure):
    _fields_ = [
        ("fft_size", ctypes.c_int32),
        ("window", ctypes.c_int32),
        ("input_format", ctypes.c_int32),
        ("avg_mode", ctypes.c_int32),
        ("avg_length", ctypes.c_int32),
        ("ema_alpha", ctypes.c_float),
        ("peak_hold", ctypes.c_int32),
        ("ring_rows", ctypes.c_int32),
        ("device_id", ctypes.c_int32),
    ]


_lib = None
_fp = ctypes.POINTER(ctypes.c_float)
_vp = ctypes.c_void_p
_h = ctypes.c_void_p


def build(force: bool = False) -> str:
    """Compile librfa.so for gfx950 with hipcc (csrc/Makefile, incremental)."""
    if force:
        subprocess.run(["make", "-s", "-C", CSRC, "clean"], check=True)
    subprocess.run(["make", "-s", "-C", CSRC, "-j4"], check=True)
    return LIB_PATH


class RfaDrawParams(ctypes.Structure):
    """rfa_draw_params (include/rfa.h): AnalyzerSurface.drawPreprocessing inputs."""
    _fields_ = [("width", ctypes.c_int32), ("fft_height", ctypes.c_int32),
                ("viewport_frequency", ctypes.c_int64), ("viewport_sample_rate", ctypes.c_int64),
                ("min_db", ctypes.c_float), ("max_db", ctypes.c_float), ("average_length", ctypes.c_int32),
                ("colormap_size", ctypes.c_int32), ("colormap", ctypes.POINTER(ctypes.c_uint32))]


def _declare(lib: ctypes.CDLL) -> None:
    sig = {
        "rfa_abi_version": (ctypes.c_int, []),
        "rfa_device_count": (ctypes.c_int, [ctypes.POINTER(ctypes.c_int)]),
        "rfa_status_string": (ctypes.c_char_p, [ctypes.c_int]),
        "rfa_default_config": (None, [ctypes.POINTER(RfaConfig)]),
        "rfa_create": (ctypes.c_int, [ctypes.POINTER(RfaConfig), ctypes.POINTER(_h)]),
        "rfa_destroy": (ctypes.c_int, [_h]),
        "rfa_get_config": (ctypes.c_int, [_h, ctypes.POINTER(RfaConfig)]),
        "rfa_last_error": (ctypes.c_char_p, [_h]),
        "rfa_set_stream": (ctypes.c_int, [_h, _vp]),
        "rfa_get_stream": (ctypes.c_int, [_h, ctypes.POINTER(_vp)]),
        "rfa_use_own_stream": (ctypes.c_int, [_h]),
        "rfa_synchronize": (ctypes.c_int, [_h]),
        "rfa_set_pipelined": (ctypes.c_int, [_h, ctypes.c_int32]),
        "rfa_join": (ctypes.c_int, [_h]),
        "rfa_process": (ctypes.c_int, [_h, _vp, ctypes.c_size_t, ctypes.c_size_t, _vp]),
        "rfa_process_host": (ctypes.c_int, [_h, _vp, ctypes.c_size_t, ctypes.c_size_t, _vp]),
        "rfa_process_batches": (ctypes.c_int, [_h, _vp, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_size_t,
                                               ctypes.c_size_t, _vp]),
        "rfa_set_tuning": (ctypes.c_int, [_h, ctypes.c_int64, ctypes.c_int64]),
        "rfa_push_packet": (ctypes.c_int, [_h, _vp, ctypes.c_size_t, ctypes.c_int64, ctypes.c_int64, _vp,
                                           ctypes.POINTER(ctypes.c_int32)]),
        "rfa_pending_samples": (ctypes.c_int, [_h, ctypes.POINTER(ctypes.c_int64)]),
        "rfa_get_state_generation": (ctypes.c_int, [_h, ctypes.POINTER(ctypes.c_int64)]),
        "rfa_get_peaks": (ctypes.c_int, [_h, _fp]),
        "rfa_get_ema": (ctypes.c_int, [_h, _fp]),
        "rfa_get_boxcar": (ctypes.c_int, [_h, ctypes.c_int32, _fp]),
        "rfa_get_ring": (ctypes.c_int, [_h, _fp, ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_int32)]),
        "rfa_reset_state": (ctypes.c_int, [_h]),
        "rfa_set_ring_rows": (ctypes.c_int, [_h, ctypes.c_int32]),
        "rfa_set_fft_size": (ctypes.c_int, [_h, ctypes.c_int32]),
        "rfa_get_device_state": (ctypes.c_int, [_h, ctypes.POINTER(_vp), ctypes.POINTER(_vp), ctypes.POINTER(_vp)]),
        "rfa_get_ring_order": (ctypes.c_int, [_h, ctypes.POINTER(ctypes.c_int32)]),
        "rfa_get_ring_positions": (ctypes.c_int, [_h, ctypes.POINTER(ctypes.c_int32), ctypes.c_size_t]),
        "rfa_stream_copy": (ctypes.c_int, [_vp, _vp, ctypes.c_size_t, _vp]),
        "rfa_ddc_get_format": (ctypes.c_int, [_h, ctypes.POINTER(ctypes.c_int32)]),
        "rfa_windowed_fft_mag_planar": (ctypes.c_int, [_h, _fp, _fp, _fp, ctypes.c_size_t]),
        "rfa_fft_logmag_interleaved": (ctypes.c_int, [_h, _fp, _fp, ctypes.c_size_t]),
        "rfa_fft_ordered": (ctypes.c_int, [_h, _fp, _fp, ctypes.c_size_t]),
        "rfa_seam_supported": (ctypes.c_int, [ctypes.c_int32]),
        "rfa_seam_create": (ctypes.c_int, [ctypes.c_int32, ctypes.c_int32, ctypes.POINTER(_h)]),
        "rfa_seam_destroy": (ctypes.c_int, [_h]),
        "rfa_seam_last_error": (ctypes.c_char_p, [_h]),
        "rfa_seam_get_plan": (ctypes.c_int, [_h, ctypes.POINTER(ctypes.c_int32), ctypes.c_int32,
                                             ctypes.POINTER(ctypes.c_int32)]),
        "rfa_seam_windowed_fft_mag_planar": (ctypes.c_int, [_h, _fp, _fp, _fp, ctypes.c_size_t]),
        "rfa_seam_fft_logmag_interleaved": (ctypes.c_int, [_h, _fp, _fp, ctypes.c_size_t]),
        "rfa_seam_fft_ordered": (ctypes.c_int, [_h, _fp, _fp, ctypes.c_size_t]),
        "rfa_set_profiling": (ctypes.c_int, [_h, ctypes.c_int]),
        "rfa_get_kernel_time": (ctypes.c_int, [_h, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_int64)]),
        "rfa_main_kernel_name": (ctypes.c_char_p, [_h]),
        "rfa_retune_offset": (ctypes.c_int64, [ctypes.c_int64, ctypes.c_int, ctypes.c_int64]),
        "rfa_set_channel": (ctypes.c_int, [_h, ctypes.c_int64, ctypes.c_int64]),
        "rfa_draw_preprocess": (ctypes.c_int, [_h, ctypes.POINTER(RfaDrawParams), _vp, _fp, _fp, _fp]),
        "rfa_row_window_stats": (ctypes.c_int, [_h, ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_int32),
                                                ctypes.c_size_t, _fp, _fp]),
        "rfa_get_channel_means": (ctypes.c_int, [_h, ctypes.POINTER(ctypes.c_float), ctypes.c_size_t,
                                                 ctypes.POINTER(ctypes.c_size_t)]),
        # demod front end (rfanalyzer_amd/demod.py)
        "rfa_ddc_create": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int32, ctypes.c_int32,
                                          ctypes.POINTER(_h)]),
        "rfa_ddc_create_resampler": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int32, ctypes.c_int32,
                                                    ctypes.POINTER(_h)]),
        "rfa_ddc_create_fir": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int32, _fp, ctypes.c_int32,
                                              ctypes.c_int32, ctypes.POINTER(_h)]),
        "rfa_ddc_set_stream": (ctypes.c_int, [_h, _vp]),
        "rfa_ddc_get_ratio": (ctypes.c_int, [_h, ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_int32),
                                             ctypes.POINTER(ctypes.c_int32)]),
        "rfa_resampler_design": (ctypes.c_int, [ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_float,
                                                ctypes.c_int32, ctypes.POINTER(ctypes.c_int32),
                                                ctypes.POINTER(ctypes.c_int32), _fp, ctypes.c_size_t,
                                                ctypes.POINTER(ctypes.c_int32)]),
        "rfa_ddc_destroy": (ctypes.c_int, [_h]),
        "rfa_ddc_last_error": (ctypes.c_char_p, [_h]),
        "rfa_ddc_set_sample_rate": (ctypes.c_int, [_h, ctypes.c_int32]),
        "rfa_ddc_set_frequencies": (ctypes.c_int, [_h, ctypes.c_int64, ctypes.c_int64]),
        "rfa_ddc_process": (ctypes.c_int, [_h, _vp, ctypes.c_size_t, _vp, _vp, ctypes.c_size_t,
                                           ctypes.POINTER(ctypes.c_size_t)]),
        "rfa_ddc_process_host": (ctypes.c_int, [_h, _vp, ctypes.c_size_t, _vp, _vp, ctypes.c_size_t,
                                                ctypes.POINTER(ctypes.c_size_t)]),
        "rfa_ddc_synchronize": (ctypes.c_int, [_h]),
        "rfa_ddc_get_stream": (ctypes.c_int, [_h, ctypes.POINTER(_vp)]),
        "rfa_ddc_get_taps": (ctypes.c_int, [_h, _fp, ctypes.c_size_t, ctypes.POINTER(ctypes.c_int32),
                                            ctypes.POINTER(ctypes.c_int32)]),
        "rfa_ddc_get_mixer": (ctypes.c_int, [_h, _fp, _fp, ctypes.c_size_t, ctypes.POINTER(ctypes.c_int32),
                                             ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_int32)]),
        "rfa_lowpass_taps": (ctypes.c_int, [ctypes.c_float, ctypes.c_float, ctypes.c_float, ctypes.c_float,
                                            ctypes.c_float, ctypes.c_int32, _fp, ctypes.c_size_t,
                                            ctypes.POINTER(ctypes.c_int32)]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args


def lib() -> ctypes.CDLL:
    """Load librfa.so (raises if it has not been built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} not built: run __graft_entry__.build() (no CPU fallback exists)")
        l = ctypes.CDLL(LIB_PATH)
        _declare(l)
        _lib = l
    return _lib


def status_string(status: int) -> str:
    try:
        return lib().rfa_status_string(status).decode()
    except Exception:  # noqa: BLE001 - library not loadable: plain text
        return str(status)


def check(status: int, where: str, handle=None) -> None:
    if status != RFA_OK:
        detail = ""
        if handle is not None:
            detail = (lib().rfa_last_error(handle) or b"").decode()
        raise RfaError(status, where, detail)


def device_count() -> int:
    c = ctypes.c_int(0)
    check(lib().rfa_device_count(ctypes.byref(c)), "rfa_device_count")
    return c.value
