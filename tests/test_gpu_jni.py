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


# ---------------------------------------------------------------- stateful natives (rfa_jni.h)
_P = "Java_com_mantz_1it_nativedsp_NativeDsp_"
_V, _I32, _I64, _F, _U8 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_float, ctypes.c_uint8


def _native(rfa, name, restype, argtypes):
    fn = getattr(rfa.lib(), _P + name)
    fn.restype = restype
    fn.argtypes = [_V, _V] + argtypes
    return fn


def _analyzer(rfa, jenv, n, rows, frames, seed):
    """createAnalyzerNative + processPacketNative (FftProcessor on the device) and the
    same frames through the C-ABI engine, for comparison."""
    create = _native(rfa, "createAnalyzerNative", _I64, [_I32, _I32, _I32, _I32, _I32, _F, _U8, _I32, _I32])
    process = _native(rfa, "processPacketNative", _I32, [_I64, _V, _I32, _I64, _I64])
    h = create(jenv.env, None, n, 0, 0, 0, 0, 0.1, 1, rows, 0)
    assert h != 0
    data = np.frombuffer(signals.frames_bytes(n, frames, "s8", seed, tones=((0.13, 0.4), (0.31, 0.02)), noise=0.03),
                         np.int8).copy()
    assert process(jenv.env, None, h, jenv.new_array(data), 2 * n, 100_000_000, 2_000_000) == frames
    e = rfa.SpectrumEngine(n, "blackman", "s8", peak_hold=True, ring_rows=rows)
    e.set_tuning(100_000_000, 2_000_000)
    e.process(data.tobytes(), frames, rows=False)
    return h, e


def test_draw_preprocess_native_matches_c_abi(rfa):
    """drawPreprocessNative (AnalyzerSurface.kt:599-743 seam) returns exactly what
    rfa_draw_preprocess returns for the same ring: colours in colorBuffer layout,
    path y, peaks y, autoscale."""
    n, rows, w = 2048, 10, 333
    jenv = MockJNIEnv()
    h, e = _analyzer(rfa, jenv, n, rows, 14, 21)
    from oracle import display as od
    cmap = od.gqrx_colormap().astype(np.int32)
    colors = np.zeros(rows * w, np.int32)
    path, pk, mm = np.zeros(w, np.float32), np.zeros(w, np.float32), np.zeros(2, np.float32)
    draw = _native(rfa, "drawPreprocessNative", _I32,
                   [_I64, _I32, _I32, _I64, _I64, _F, _F, _I32, _V, _V, _V, _V, _V])
    rc = draw(jenv.env, None, h, w, 480, 100_000_000, 2_000_000, -110.0, -20.0, 3, jenv.new_array(cmap),
              jenv.new_array(colors), jenv.new_array(path), jenv.new_array(pk), jenv.new_array(mm))
    assert rc == 0
    c2, p2, k2, mm2 = e.draw_preprocess(w, 480, 100_000_000, 2_000_000, -110.0, -20.0, 3, cmap.view(np.uint32),
                                        peaks=True)
    np.testing.assert_array_equal(colors.view(np.uint32).reshape(rows, w), c2)
    assert np.array_equal(np.isnan(path), np.isnan(p2))
    np.testing.assert_array_equal(path[~np.isnan(path)], p2[~np.isnan(p2)])
    np.testing.assert_array_equal(pk, k2)
    assert (float(mm[0]), float(mm[1])) == mm2
    # peaks y is optional (null array), a short colour buffer is RFA_ERR_SIZE
    assert draw(jenv.env, None, h, w, 480, 100_000_000, 2_000_000, -110.0, -20.0, 3, jenv.new_array(cmap),
                jenv.new_array(colors), jenv.new_array(path), None, jenv.new_array(mm)) == 0
    short = np.zeros(rows * w - 1, np.int32)
    assert draw(jenv.env, None, h, w, 480, 100_000_000, 2_000_000, -110.0, -20.0, 3, jenv.new_array(cmap),
                jenv.new_array(short), jenv.new_array(path), None, jenv.new_array(mm)) == -2
    _native(rfa, "destroyAnalyzerNative", None, [_I64])(jenv.env, None, h)
    e.close()


def test_row_window_stats_native(rfa):
    """rowWindowStatsNative (MainViewModel.kt scanner / squelch reductions) on the
    analyzer's newest row equals the C-ABI call."""
    n, rows = 4096, 4
    jenv = MockJNIEnv()
    h, e = _analyzer(rfa, jenv, n, rows, 6, 33)
    rng = np.random.default_rng(4)
    lo = rng.integers(0, n - 1, 50).astype(np.int32)
    hi = np.minimum(n - 1, lo + rng.integers(0, 300, 50)).astype(np.int32)
    pk, av = np.zeros(50, np.float32), np.zeros(50, np.float32)
    stats = _native(rfa, "rowWindowStatsNative", _I32, [_I64, _V, _V, _V, _V])
    assert stats(jenv.env, None, h, jenv.new_array(lo), jenv.new_array(hi), jenv.new_array(pk),
                 jenv.new_array(av)) == 0
    epk, eav = e.row_window_stats(lo, hi)
    np.testing.assert_array_equal(pk, epk)
    np.testing.assert_array_equal(av, eav)
    _native(rfa, "destroyAnalyzerNative", None, [_I64])(jenv.env, None, h)
    e.close()


@pytest.mark.parametrize("resampler", [False, True])
def test_ddc_natives_match_front_end(rfa, resampler):
    """ddcCreate / ddcSetFrequencies / ddcProcess (Scheduler.kt:237-250 demod branch)
    give the samples the C-ABI front end gives, packet after packet."""
    from rfanalyzer_amd import demod
    jenv = MockJNIEnv()
    create = _native(rfa, "ddcCreate", _I64, [_I32, _I32, _I32, _U8, _I32])
    setf = _native(rfa, "ddcSetFrequencies", _I32, [_I64, _I64, _I64])
    proc = _native(rfa, "ddcProcess", _I32, [_I64, _V, _V, _V])
    h = create(jenv.env, None, 0, 2_400_000, 96_000, 1 if resampler else 0, 0)
    assert h != 0
    assert setf(jenv.env, None, h, 100_000_000, 100_130_000) == 0
    fe = demod.FrontEnd("s8", 2_400_000, 96_000, resampler=resampler)
    fe.set_frequencies(100_000_000, 100_130_000)
    rng = np.random.default_rng(12)
    for size in (262_144, 70_001 * 2, 262_144):
        packet = rng.integers(-128, 128, size, dtype=np.int8)
        re, im = np.zeros(20_000, np.float32), np.zeros(20_000, np.float32)
        got = proc(jenv.env, None, h, jenv.new_array(packet), jenv.new_array(re), jenv.new_array(im))
        w_re, w_im = fe.process(packet.tobytes())
        assert got == w_re.size
        np.testing.assert_array_equal(re[:got], w_re)
        np.testing.assert_array_equal(im[:got], w_im)
    tiny = np.zeros(3, np.float32)
    assert proc(jenv.env, None, h, jenv.new_array(rng.integers(-128, 128, 262_144, dtype=np.int8)),
                jenv.new_array(tiny), jenv.new_array(tiny)) == -2  # RFA_ERR_SIZE
    _native(rfa, "ddcDestroy", None, [_I64])(jenv.env, None, h)
    fe.close()
