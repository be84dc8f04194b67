"""GPU: the JNI drop-in symbols (include/rfa_jni.h) driven through a mock JNIEnv,
compared with the reference pffft path they replace (nativedsp.cpp:19-81)."""
import ctypes

import numpy as np
import pytest

import golden_util as gu
import oracle
import signals
from jni_mock import MockJNIEnv

pytestmark = pytest.mark.gpu


def _sym(rfa, name, restype, nargs):
    fn = getattr(rfa.lib(), name)
    fn.restype = restype
    fn.argtypes = [ctypes.c_void_p] * nargs
    return fn


def test_perform_fft_and_log_mag(rfa):
    if not oracle.ref_available():
        pytest.skip("reference pffft build absent")
    n = 16384
    jenv = MockJNIEnv()
    rng = np.random.default_rng(7)
    inter = oracle.windowed_interleaved(rng.standard_normal(n).astype(np.float32),
                                        rng.standard_normal(n).astype(np.float32), oracle.window(n))
    out = np.zeros(n, np.float32)
    fn = _sym(rfa, "Java_com_mantz_1it_nativedsp_NativeDsp_performFFTAndLogMag", None, 4)
    fn(jenv.env, None, jenv.new_array(inter), jenv.new_array(out))
    assert gu.pffft_diff(out, oracle.ref_fft_logmag(inter)) <= gu.DB_TOL
    assert "SetFloatArrayRegion" in jenv.calls


def test_perform_fft(rfa):
    if not oracle.ref_available():
        pytest.skip("reference pffft build absent")
    n = 1024
    jenv = MockJNIEnv()
    x = np.random.default_rng(8).standard_normal(2 * n).astype(np.float32)
    out = np.zeros(2 * n, np.float32)
    fn = _sym(rfa, "Java_com_mantz_1it_nativedsp_NativeDsp_performFFT", None, 4)
    fn(jenv.env, None, jenv.new_array(x), jenv.new_array(out))
    ref = oracle.ref_fft_ordered(x)
    assert np.abs(out - ref).max() / np.abs(ref).max() < 1e-5


def test_windowed_planar_native_and_size_mismatch(rfa):
    n = 4096
    jenv = MockJNIEnv()
    rng = np.random.default_rng(9)
    re = rng.standard_normal(n).astype(np.float32)
    im = rng.standard_normal(n).astype(np.float32)
    out = np.zeros(n, np.float32)
    fn = _sym(rfa, "Java_com_mantz_1it_nativedsp_NativeDsp_performWindowedFftAndReturnMagNative", ctypes.c_uint8, 5)
    assert fn(jenv.env, None, jenv.new_array(re), jenv.new_array(im), jenv.new_array(out)) == 1
    planar = np.concatenate([re, im]).tobytes()
    ref = oracle.spectrum_rows(planar, oracle.IN_F32_PLANAR, n, 1, None, oracle.WIN_BLACKMAN)[0]
    assert gu.db_diff(out, ref) <= gu.DB_TOL
    short = np.zeros(n - 1, np.float32)
    assert fn(jenv.env, None, jenv.new_array(re), jenv.new_array(short), jenv.new_array(out)) == 0


def test_process_iq_bytes_native(rfa):
    n = 1024
    data = np.frombuffer(signals.file_capture(262_144 * 3), np.int8).copy()
    jenv = MockJNIEnv()
    out = np.zeros(3 * n, np.float32)
    fn = _sym(rfa, "Java_com_mantz_1it_nativedsp_NativeDsp_processIqBytesNative", ctypes.c_int32, 6)
    fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                   ctypes.c_void_p]
    got = fn(jenv.env, None, jenv.new_array(data), 0, n, 262_144, jenv.new_array(out))
    assert got == 3
    ref = oracle.spectrum_rows(data.tobytes(), oracle.IN_S8, n, 3, 262_144, oracle.WIN_BLACKMAN)
    assert gu.db_diff(out.reshape(3, n), ref) <= gu.DB_TOL
