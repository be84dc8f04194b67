"""GPU: the legacy seam at every length the reference's pffft accepts
(pffft.c:1231-1280: N a multiple of 16, N / 4 a product of 2, 3, 4, 5, N <= 2^26).
Powers of two from 64 to 2^20 run on the streaming handle (test_gpu_parity.py);
the rest -- 16, 32, 2^21 .. 2^26 and mixed 2/3/5 lengths -- on librfa's
mixed-radix plan (csrc/fft_seam.hip, rfa_seam_*), checked here against the
reference's own pffft (oracle/_ref, compiled from its pffft.c) and a float64 FFT."""
import ctypes

import numpy as np
import pytest

import golden_util as gu
import oracle
from jni_mock import MockJNIEnv

pytestmark = pytest.mark.gpu

_P = "Java_com_mantz_1it_nativedsp_NativeDsp_"
# 16, 32: below the handle's 64; 48 .. 48000: mixed 2/3/5 lengths, every radix as the
# first and the last pass; 2^21 and 3 * 2^20: above the handle's 2^20
SIZES = [16, 32, 48, 80, 144, 240, 720, 1200, 3888, 10000, 48000, 1 << 21, 3 << 20]


def _noise(n, seed):
    rng = np.random.default_rng(seed)
    return rng.standard_normal(2 * n).astype(np.float32)


def _rel_err(got, ref):
    g = got[0::2].astype(np.float64) + 1j * got[1::2]
    r = ref[0::2].astype(np.float64) + 1j * ref[1::2]
    return np.abs(g - r).max() / np.abs(r).max()


@pytest.mark.parametrize("n", SIZES)
def test_seam_plan_matches_pffft_and_float64(rfa, n):
    from rfanalyzer_amd.engine import SeamPlan
    x = _noise(n, n)
    exact = np.fft.fft(x[0::2].astype(np.float64) + 1j * x[1::2])
    with SeamPlan(n) as p:
        plan = p.plan()
        assert int(np.prod(plan)) == n and set(plan) <= {2, 3, 4, 5, 8}
        cx = p.fft_ordered(x)
        mag = p.fft_logmag(x)
        re, im = x[0::2].copy(), x[1::2].copy()
        wmag = np.empty(n, np.float32)
        assert p.windowed_fft_mag(re, im, wmag)
    g = cx[0::2].astype(np.float64) + 1j * cx[1::2]
    assert np.abs(g - exact).max() / np.abs(exact).max() < 2e-6
    ref_db = np.fft.fftshift(10 * np.log10(np.abs(exact) / n)).astype(np.float32)
    assert gu.db_diff(mag, ref_db) <= gu.DB_TOL
    if oracle.ref_available():
        assert _rel_err(cx, oracle.ref_fft_ordered(x)) < 2e-6
        assert gu.pffft_diff(mag, oracle.ref_fft_logmag(x)) <= gu.DB_TOL
        w = oracle.window(n, oracle.WIN_BLACKMAN)
        assert gu.pffft_diff(wmag, oracle.ref_fft_logmag(oracle.windowed_interleaved(re, im, w))) <= gu.DB_TOL


def test_seam_plan_at_the_pffft_maximum(rfa):
    """N = 2^26, the largest length pffft_new_setup takes (pffft.c:1236)."""
    from rfanalyzer_amd.engine import SeamPlan
    n = 1 << 26
    x = _noise(n, 26)
    with SeamPlan(n) as p:
        assert p.plan() == [8] * 8 + [4]
        cx = p.fft_ordered(x)
    if oracle.ref_available():
        assert _rel_err(cx, oracle.ref_fft_ordered(x)) < 2e-6
    else:
        exact = np.fft.fft(x[0::2].astype(np.float64) + 1j * x[1::2])
        g = cx[0::2].astype(np.float64) + 1j * cx[1::2]
        assert np.abs(g - exact).max() / np.abs(exact).max() < 2e-6


@pytest.mark.parametrize("n", [1024, 65536])
def test_seam_plan_agrees_with_the_streaming_handle(rfa, n):
    """Where both take N, the mixed-radix plan and the fused kernel give the same row."""
    from rfanalyzer_amd.engine import SeamPlan
    x = _noise(n, 3 * n)
    with SeamPlan(n) as p, rfa.SpectrumEngine(n, "none", "f32", ring_rows=0) as e:
        assert gu.db_diff(p.fft_logmag(x), e.fft_logmag(x)) <= gu.DB_TOL


def test_seam_zero_input_and_tone_bin(rfa):
    """Zeros give -inf (log10(0), nativedsp.cpp:78); a bin-centred tone lands on its
    fft-shifted bin at 10 log10(1) = 0 dB (|X| / N = 1)."""
    from rfanalyzer_amd.engine import SeamPlan
    n, k = 240, 37
    with SeamPlan(n) as p:
        assert np.all(np.isneginf(p.fft_logmag(np.zeros(2 * n, np.float32))))
        t = np.exp(2j * np.pi * k * np.arange(n) / n)
        x = np.empty(2 * n, np.float32)
        x[0::2], x[1::2] = t.real, t.imag
        row = p.fft_logmag(x)
    assert int(np.argmax(row)) == (k + n // 2) % n
    assert abs(row[(k + n // 2) % n]) < 1e-5


def test_seam_sizes_and_errors(rfa):
    from rfanalyzer_amd import RfaError
    from rfanalyzer_amd.engine import SeamPlan
    for bad in (0, 8, 40, 112, 1000, (1 << 26) + 16 * 3):
        with pytest.raises(RfaError) as e:
            SeamPlan(bad)
        assert e.value.status == -3  # RFA_ERR_UNSUPPORTED, pffft rejects it
    with SeamPlan(48) as p:
        out = np.empty(48, np.float32)
        assert not p.windowed_fft_mag(np.zeros(48, np.float32), np.zeros(47, np.float32), out)
        with pytest.raises(RfaError):
            p.fft_ordered(np.zeros(2 * 64, np.float32))  # RFA_ERR_SIZE: not the plan's N


def test_native_dsp_mirror_takes_every_pffft_length(rfa):
    """NativeDsp (the Kotlin class's mirror) switches between the streaming handle and a
    plan as the length changes, like the reference's per-size setup (nativedsp.cpp:56-64)."""
    from rfanalyzer_amd.nativedsp import NativeDsp
    dsp = NativeDsp()
    for n in (48, 1024, 3888, 16, 4096):
        x = _noise(n, n + 1)
        out = np.empty(n, np.float32)
        dsp.performFFTAndLogMag(x, out)
        exact = np.fft.fft(x[0::2].astype(np.float64) + 1j * x[1::2])
        assert gu.db_diff(out, np.fft.fftshift(10 * np.log10(np.abs(exact) / n)).astype(np.float32)) <= gu.DB_TOL
        cx = np.empty(2 * n, np.float32)
        dsp.performFFT(x, cx)
        g = cx[0::2].astype(np.float64) + 1j * cx[1::2]
        assert np.abs(g - exact).max() / np.abs(exact).max() < 2e-6
    dsp.close()


@pytest.mark.parametrize("m", [48, 480, 16, 32, 1 << 21])
def test_jni_legacy_symbols_at_pffft_only_lengths(rfa, m):
    """performFFT / performFFTAndLogMag / performWindowedFftAndReturnMagNative through a
    mock JNIEnv at lengths the handle does not take: the shim's cached plan serves them,
    rfa_jni_last_status() is RFA_OK, and the rows equal the reference pffft's."""
    jenv = MockJNIEnv()
    lib = rfa.lib()
    status = lib.rfa_jni_last_status
    status.restype = ctypes.c_int32
    fft = getattr(lib, _P + "performFFT")
    logmag = getattr(lib, _P + "performFFTAndLogMag")
    planar = getattr(lib, _P + "performWindowedFftAndReturnMagNative")
    for fn in (fft, logmag):
        fn.restype = None
        fn.argtypes = [ctypes.c_void_p] * 4
    planar.restype = ctypes.c_uint8
    planar.argtypes = [ctypes.c_void_p] * 5
    x = _noise(m, m + 7)
    cx = np.zeros(2 * m, np.float32)
    fft(jenv.env, None, jenv.new_array(x), jenv.new_array(cx))
    assert status() == 0
    mag = np.zeros(m, np.float32)
    logmag(jenv.env, None, jenv.new_array(x), jenv.new_array(mag))
    assert status() == 0
    re, im = x[0::2].copy(), x[1::2].copy()
    wmag = np.zeros(m, np.float32)
    assert planar(jenv.env, None, jenv.new_array(re), jenv.new_array(im), jenv.new_array(wmag)) == 1
    assert status() == 0
    exact = np.fft.fft(x[0::2].astype(np.float64) + 1j * x[1::2])
    g = cx[0::2].astype(np.float64) + 1j * cx[1::2]
    assert np.abs(g - exact).max() / np.abs(exact).max() < 2e-6
    if oracle.ref_available():
        assert _rel_err(cx, oracle.ref_fft_ordered(x)) < 2e-6
        assert gu.pffft_diff(mag, oracle.ref_fft_logmag(x)) <= gu.DB_TOL
        w = oracle.window(m, oracle.WIN_BLACKMAN)
        assert gu.pffft_diff(wmag, oracle.ref_fft_logmag(oracle.windowed_interleaved(re, im, w))) <= gu.DB_TOL


def test_seam_and_refused_lengths_keep_the_framing_setup(rfa):
    """A legacy call at a length the handle does not take (a seam plan's 48 or 2^21, or
    1000, which pffft rejects too) evicts no cached handle: with the shim's four slots
    full and the framing-mode setup the least recently used, processIqBytesNative's
    partial frame survives them, and every row of the reference framing arrives."""
    from oracle import processor
    import signals
    n, pkt = 8192, 1500
    jenv = MockJNIEnv()
    lib = rfa.lib()
    status = lib.rfa_jni_last_status
    status.restype = ctypes.c_int32
    frame_fn = getattr(lib, _P + "processIqBytesNative")
    frame_fn.restype = ctypes.c_int32
    frame_fn.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_int32] * 3 + [ctypes.c_void_p]
    fft = getattr(lib, _P + "performFFT")
    logmag = getattr(lib, _P + "performFFTAndLogMag")
    for fn in (fft, logmag):
        fn.restype = None
        fn.argtypes = [ctypes.c_void_p] * 4

    def legacy(fn, m):
        fn(jenv.env, None, jenv.new_array(np.ones(2 * m, np.float32)), jenv.new_array(np.zeros(2 * m, np.float32)))
        return status()

    for m in (64, 128, 256, 512):  # fill the four slots: no framing setup of an earlier test survives
        assert legacy(fft, m) == 0
    raw = signals.frames_bytes(n, 4, "u8", 23, tones=((0.17, 0.5),), noise=0.04)
    packets = [raw[i:i + pkt] for i in range(0, len(raw) - pkt + 1, pkt)]
    frames = processor.scheduler_frames([(b, 0, 1) for b in packets], n, 2)
    rows = []
    for b in packets:
        out = np.zeros(n, np.float32)
        got = frame_fn(jenv.env, None, jenv.new_array(np.frombuffer(b, np.int8).copy()), 1, n, 0,
                       jenv.new_array(out))  # format 1 = u8
        assert got in (0, 1) and status() == 0
        if got:
            rows.append(out)
        for m in (128, 256, 512):  # the framing setup is now the least recently used slot
            assert legacy(fft, m) == 0
        assert legacy(fft, 48) == 0
        assert legacy(logmag, 1 << 21) == 0
        assert legacy(fft, 1000) == -3
    assert len(rows) == len(frames) > 0
    exp = np.stack([oracle.spectrum_rows(f[0], oracle.IN_U8, n, 1, None, oracle.WIN_BLACKMAN)[0] for f in frames])
    assert gu.db_diff(np.stack(rows), exp) <= gu.DB_TOL
