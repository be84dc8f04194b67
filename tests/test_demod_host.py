"""CPU: demod front end restatement (oracle/demod.py) and the library's host-side
filter design (rfa_lowpass_taps).

Parity with the JVM is pinned by the reference's own FIR golden vectors
(ApplicationTest.kt:20-176, testFirFilter / testFirFilter2: JVM outputs of
createLowPass + FirFilter.filter at a 1e-9 tolerance, tests/golden/
fir_application_test.json), by the restated per-sample loop of FirFilter.filter,
and by the property ResamplerTest.kt:20-116 checks (a 100 Hz tone through
Decimator 48 kHz -> 12 kHz).  The mixer tables and the polyphase resampler have
no JVM vectors in the reference: parity unpinned beyond the restatement."""
import numpy as np
import pytest

from oracle import demod as od

F32 = np.float32


def test_vectorised_filter_equals_literal_loop_across_packets():
    rng = np.random.default_rng(5)
    d, taps = od.decimator_taps(240_000, 24_000)            # D = 10
    assert d == 10 and len(taps) % 2 == 1
    a, b = od.FirDecimator(taps, d), od.FirDecimator(taps, d)
    x = rng.standard_normal((2, 3000)).astype(F32)
    got_re, got_im, lit_re, lit_im = [], [], [], []
    pos = 0
    for n in [1, 7, 0, 130, 999, 3, 1860]:                 # ragged packets, some shorter than the filter
        r, i = a.filter(x[0, pos:pos + n], x[1, pos:pos + n])
        lr, li = b.filter_literal(x[0, pos:pos + n], x[1, pos:pos + n])
        got_re.append(r), got_im.append(i), lit_re.append(lr), lit_im.append(li)
        pos += n
    assert pos == 3000
    np.testing.assert_array_equal(np.concatenate(got_re), np.concatenate(lit_re))
    np.testing.assert_array_equal(np.concatenate(got_im), np.concatenate(lit_im))
    assert len(np.concatenate(got_re)) == 300                # outputs at inputs 9, 19, ... (counter starts at 1)


def test_decimator_taps_shape_and_gain():
    d, taps = od.decimator_taps(48_000, 12_000)
    assert d == 4
    assert len(taps) == 43                                   # (60*48000/(22*3000)).toInt() = 43, odd
    assert abs(float(taps.astype(np.float64).sum()) - 1.0) < 1e-5
    np.testing.assert_array_equal(taps, taps[::-1])          # symmetric
    assert od.low_pass_taps(1, 48_000, 30_000, 1000, 60) is None   # cutoff above fs/2 -> null


def test_resampler_test_tone_passes_the_decimator():
    """ResamplerTest.kt:20-116 drives Decimator(12000) with a 100 Hz IQ tone at 48 kHz."""
    n = 48_000
    t = np.arange(n) / 48_000.0
    iq = np.empty(2 * n, F32)
    iq[0::2] = np.cos(2 * np.pi * 100.0 * t).astype(F32)
    iq[1::2] = np.sin(2 * np.pi * 100.0 * t).astype(F32)
    fe = od.FrontEnd(od.IN_F32_INTERLEAVED, 48_000, 12_000)
    outs = [fe.process(iq[k:k + 2048]) for k in range(0, 2 * n, 2048)]   # 1024-sample packets
    re = np.concatenate([o[0] for o in outs])
    im = np.concatenate([o[1] for o in outs])
    assert len(re) == n // 4
    z = (re + 1j * im)[100:]                                  # past the filter's transient
    assert np.abs(np.abs(z) - 1).max() < 2e-3                 # pass-band gain 1
    ang = np.angle(z[1:] * np.conj(z[:-1]))
    assert np.allclose(ang, 2 * np.pi * 100 / 12_000, atol=1e-3)


def test_mixer_fold_and_cosine_length():
    sr = 2_400_000
    assert od.mix_frequency(100_000_000, 100_000_000, sr) == sr          # 0 -> +sampleRate
    assert od.mix_frequency(100_000_000, 100_001_000, sr) == -1000 + sr  # sr/1000 > 500 -> folded
    assert od.mix_frequency(100_000_000, 99_900_000, sr) == 100_000
    assert od.optimal_cosine_length(sr, 100_000) == 24
    assert od.optimal_cosine_length(sr, sr) == 1
    n = od.optimal_cosine_length(sr, 7_001)                              # best multiple below 500 samples
    assert 0 < n < 500
    assert od.mix_frequency(2 ** 40 + 5, 0, sr) == 5 + sr                # (int) keeps the low 32 bits


def test_mix_brings_the_channel_to_dc():
    sr, f, ch = 1_000_000, 100_000_000, 100_125_000
    n = 4000
    k = np.arange(n)
    tone = np.exp(2j * np.pi * (ch - f) / sr * k) * 0.9
    raw = np.empty(2 * n, np.int8)
    raw[0::2] = np.round(tone.real * 127).astype(np.int8)
    raw[1::2] = np.round(tone.imag * 127).astype(np.int8)
    mf = od.mix_frequency(f, ch, sr)
    c, s = od.mixer_table(od.IN_S8, sr, mf)
    re, im = od.mix(od.IN_S8, raw.view(np.uint8), c, s, 0)
    z = re + 1j * im
    assert abs(np.mean(z)) > 0.85                              # energy at DC
    assert np.std(np.angle(z)) < 0.05


@pytest.fixture(scope="module")
def lib():
    import rfanalyzer_amd
    rfanalyzer_amd.build()
    return rfanalyzer_amd.lib()


@pytest.mark.parametrize("args", [
    (1, 48_000, 9_000, 3_000, 60, 0),
    (1, 2_400_000, 72_000, 24_000, 60, 0),
    (1, 20_000_000, 288_000, 96_000, 60, 0),
    (1, 10_000_000, 36_000, 12_000, 60, 500),                 # maxTaps clamp (RationalResampler's use)
    (2.5, 1_000_000, 10_000, 777, 40, 0),
])
def test_library_taps_bit_exact_with_restatement(lib, args):
    from rfanalyzer_amd import demod
    got = demod.create_low_pass_taps(*args)
    want = od.low_pass_taps(*args)
    assert got.dtype == np.float32 and got.shape == want.shape
    np.testing.assert_array_equal(got.view(np.int32), want.view(np.int32))


def test_library_taps_null_cases(lib):
    from rfanalyzer_amd import demod
    assert demod.create_low_pass_taps(1, 0, 100, 10, 60) is None
    assert demod.create_low_pass_taps(1, 1000, 600, 10, 60) is None
    assert demod.create_low_pass_taps(1, 1000, 100, 0, 60) is None


@pytest.mark.parametrize("fmt,sr,out", [(od.IN_S8, 2_400_000, 96_000), (od.IN_U8, 1_000_000, 48_000),
                                        (od.IN_S16LE, 10_000_000, 384_000), (od.IN_F32_INTERLEAVED, 48_000, 12_000)])
def test_c_loop_equals_vectorised_restatement(fmt, sr, out):
    """orc_ddc_process (the reference's per-sample loop in C) == FrontEnd (numpy form)."""
    rng = np.random.default_rng(sr)
    sb = {od.IN_S8: 2, od.IN_U8: 2, od.IN_S16LE: 4, od.IN_F32_INTERLEAVED: 8}[fmt]
    n = 40_000
    raw = (rng.standard_normal(2 * n).astype(F32).view(np.uint8) if fmt == od.IN_F32_INTERLEAVED
           else rng.integers(0, 256, n * sb, dtype=np.uint8))
    a, b = od.FrontEnd(fmt, sr, out), od.CFrontEnd(fmt, sr, out)
    pos = 0
    for n_s, ch in [(5, 100_050_000), (9000, 100_050_000), (1, 99_990_000), (30_994, 99_990_000)]:
        a.set_frequencies(100_000_000, ch)
        b.set_frequencies(100_000_000, ch)
        chunk = raw[pos * sb:(pos + n_s) * sb]
        ra, rb = a.process(chunk), b.process(chunk)
        np.testing.assert_array_equal(ra[0].view(np.int32), rb[0].view(np.int32))
        np.testing.assert_array_equal(ra[1].view(np.int32), rb[1].view(np.int32))
        pos += n_s
    assert pos == n


@pytest.mark.parametrize("out,inp", [(96_000, 2_400_000), (384_000, 20_000_000), (12_000, 48_000),
                                     (44_100, 1_000_000)])
def test_resampler_closed_form_equals_literal_loop(out, inp):
    """RationalResampler.resample per call (RationalResampler.kt:62-127) == the
    closed form the kernel uses, across ragged calls."""
    i, d = od.limit_denominator(out, inp, 10000)
    a, b = od.RationalResampler(i, d, max_taps=40), od.RationalResampler(i, d, max_taps=40)
    rng = np.random.default_rng(out)
    x = rng.standard_normal((2, 4000)).astype(F32)
    pos, ga, gb = 0, [], []
    for n in [1, 2, 3, 500, 0, 77, 3417]:
        ga.append(a.resample(x[0, pos:pos + n], x[1, pos:pos + n]))
        gb.append(b.resample_literal(x[0, pos:pos + n], x[1, pos:pos + n]))
        pos += n
    for k in (0, 1):
        np.testing.assert_array_equal(np.concatenate([g[k] for g in ga]), np.concatenate([g[k] for g in gb]))
    assert a.n_done == len(np.concatenate([g[0] for g in gb]))


def test_limit_denominator_and_resampler_design():
    assert od.limit_denominator(96_000, 2_400_000) == (1, 25)
    assert od.limit_denominator(384_000, 20_000_000) == (12, 625)
    i, d = od.limit_denominator(1, 10_007 * 3, 10000)               # denominator beyond the limit
    assert d <= 10000 and i >= 0
    t = od.design_resampler_taps(1, 25, 0.4, 500)
    assert len(t) == 501 and abs(float(t.astype(np.float64).sum()) - 1.0) < 1e-4   # gain I at DC


def test_library_resampler_design_bit_exact(lib):
    import ctypes
    L = lib
    for out, inp in [(96_000, 2_400_000), (384_000, 20_000_000), (12_000, 48_000)]:
        i, d, n = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int32()
        assert L.rfa_resampler_design(out, inp, 10000, ctypes.c_float(0.4), 500, ctypes.byref(i), ctypes.byref(d),
                                      None, 0, ctypes.byref(n)) == 0
        got = np.empty(n.value, np.float32)
        assert L.rfa_resampler_design(out, inp, 10000, ctypes.c_float(0.4), 500, ctypes.byref(i), ctypes.byref(d),
                                      got.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), got.size,
                                      ctypes.byref(n)) == 0
        wi, wd = od.limit_denominator(out, inp, 10000)
        assert (i.value, d.value) == (wi, wd)
        np.testing.assert_array_equal(got.view(np.int32), od.design_resampler_taps(wi, wd, 0.4, 500).view(np.int32))


# ---------------------------------------------------------------- the reference's FIR golden vectors
import fir_vectors  # noqa: E402


@pytest.mark.parametrize("case", fir_vectors.cases(), ids=lambda c: c["name"])
def test_restatement_matches_reference_fir_vectors(case):
    """ApplicationTest.kt testFirFilter / testFirFilter2: createLowPass + FirFilter.filter,
    JVM outputs at the test's 1e-9 tolerance -- the numpy form, the literal loop and
    the C loop (orc_ddc_process) of the restatement."""
    re, im = fir_vectors.inputs(case)
    taps = od.low_pass_taps(case["gain"], case["sample_rate"], case["cutoff"], case["transition"],
                            case["attenuation"])
    d = case["decimation"]
    fir_vectors.check(case, *od.FirDecimator(taps, d).filter(re, im))
    fir_vectors.check(case, *od.FirDecimator(taps, d).filter_literal(re, im))
    # the same samples split into ragged packets: state carries over
    f = od.FirDecimator(taps, d)
    parts = [f.filter(re[a:b], im[a:b]) for a, b in ((0, 3), (3, 4), (4, 40), (40, len(re)))]
    fir_vectors.check(case, np.concatenate([p[0] for p in parts]), np.concatenate([p[1] for p in parts]))
    iq = np.empty(2 * re.size, F32)
    iq[0::2], iq[1::2] = re, im
    fe = od.CFrontEnd(od.IN_F32_INTERLEAVED, int(case["sample_rate"]), int(case["sample_rate"]) // d, taps, d)
    fir_vectors.check(case, *fe.process(iq.view(np.uint8)))


@pytest.mark.parametrize("case", fir_vectors.cases(), ids=lambda c: c["name"])
def test_library_taps_match_reference_fir_vectors(lib, case):
    """rfa_lowpass_taps (host C) designs the taps behind those vectors bit for bit."""
    from rfanalyzer_amd import demod
    args = (case["gain"], case["sample_rate"], case["cutoff"], case["transition"], case["attenuation"])
    got, want = demod.create_low_pass_taps(*args), od.low_pass_taps(*args)
    np.testing.assert_array_equal(got.view(np.int32), want.view(np.int32))


@pytest.mark.parametrize("offset,sr", [(25_000, 20_000_000), (4_000, 2_400_000), (1_000, 2_000_000),
                                       (-1_000, 2_000_000), (39_999, 20_000_000), (0, 2_400_000)])
def test_mixer_table_length_bound(offset, sr):
    """calcOptimalCosineLength after generateMixerLookupTable's fold (IQConverter.java:64-76,
    Signed8BitIQConverter.java:53-57) stays <= MAX_COSINE_LENGTH (500) + 1: an unfolded
    cycle is < 501 samples and the search stops below 500."""
    mf = od.mix_frequency(100_000_000 + offset, 100_000_000, sr)
    n = od.optimal_cosine_length(sr, mf)
    assert 1 <= n <= 501
