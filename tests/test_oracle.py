"""CPU: pin the oracle against the reference's own pffft (golden fixtures) and
check the restated state machine against the stored sequences."""
import numpy as np
import pytest

import golden_util as gu
import oracle
import signals
from oracle import processor

MANIFEST = gu.manifest()
FIXTURES = MANIFEST["fixtures"]


@pytest.mark.parametrize("spec", FIXTURES, ids=[s["name"] for s in FIXTURES])
def test_oracle_matches_reference_pffft(spec):
    data = gu.fixture_input(spec)
    rows = oracle.spectrum_rows(data, signals.FORMATS[spec["fmt"]], spec["n"], spec["n_frames"],
                                spec.get("packet_size"), gu.WINDOW_IDS[spec["window"]])
    exp = gu.expected(spec)
    assert gu.db_diff(rows[:, ::spec["subset_stride"]], exp) <= gu.DB_TOL
    assert [int(a) for a in np.argmax(rows, axis=1)] == spec["argmax"]


@pytest.mark.skipif(not oracle.ref_available(), reason="reference pffft build absent")
def test_ref_harness_matches_fixture_exactly():
    """The committed fixture IS the reference pffft output (bit-exact regeneration)."""
    spec = next(s for s in FIXTURES if s["name"] == "s8_n8192_x4")
    data = gu.fixture_input(spec)
    rows = oracle.ref_spectrum_rows(data, 0, spec["n"], spec["n_frames"], None, oracle.WIN_BLACKMAN)
    np.testing.assert_array_equal(rows, gu.expected(spec))


@pytest.mark.skipif(not oracle.ref_available(), reason="reference pffft build absent")
@pytest.mark.parametrize("n", [64, 1024, 65536])
def test_reference_pffft_ordered_vs_numpy(n):
    rng = np.random.default_rng(n)
    x = rng.standard_normal(2 * n).astype(np.float32)
    got = oracle.ref_fft_ordered(x)
    ref = np.fft.fft(x[0::2].astype(np.float64) + 1j * x[1::2])
    err = np.abs((got[0::2] + 1j * got[1::2]) - ref).max() / np.abs(ref).max()
    assert err < 1e-5


@pytest.mark.skipif(not oracle.exact_available(), reason="exact-twiddle pffft build absent")
@pytest.mark.parametrize("n", [1024, 48000, 65536, 1 << 20])
def test_exact_twiddle_pffft_build(n):
    """oracle/exact_twiddle.c (diagnostic): the reference's pffft with its two
    twiddle tables recomputed from exact angles.  Every table entry moved by <= 1e-6 (the restated
    setup layout is the reference's), the transform stays within 1e-6 of max |X| of the unmodified
    pffft, and its RMS error against float64 is below pffft's (the float-argument twiddles of
    pffft.c:1140,1156,1160-1161,1261 are a third of pffft's rounding error)."""
    x = np.random.default_rng(n).standard_normal(2 * n).astype(np.float32)
    a = oracle.ref_fft_ordered(x)
    b = np.empty_like(x)
    assert oracle.exact().exact_fft_ordered(oracle._f32ptr(x), n, oracle._f32ptr(b)) == 0
    assert 0 < oracle.exact().exact_max_change() <= 1e-6
    f = np.fft.fft(x[0::2].astype(np.float64) + 1j * x[1::2])
    ca, cb = a[0::2] + 1j * a[1::2].astype(np.float64), b[0::2] + 1j * b[1::2].astype(np.float64)
    m = np.abs(f).max()
    assert np.abs(ca - cb).max() <= 1e-6 * m
    assert np.sqrt(np.mean(np.abs(cb - f) ** 2)) < np.sqrt(np.mean(np.abs(ca - f) ** 2))


def test_kat_values():
    n = 1024
    imp = oracle.spectrum_rows(signals.kat_bytes("impulse", n), oracle.IN_F32_INTERLEAVED, n, 1, None, None)[0]
    np.testing.assert_allclose(imp, 10 * np.log10(1 / n), atol=1e-5)  # flat |X|/N = 1/N
    tone = oracle.spectrum_rows(signals.kat_bytes("tone_bin", n), oracle.IN_F32_INTERLEAVED, n, 1, None, None)[0]
    assert int(np.argmax(tone)) == (n // 8 + 3 + n // 2) % n  # fft-shift: bin k -> k + N/2
    assert abs(tone.max() - 10 * np.log10(0.5)) < 1e-5
    ny = oracle.spectrum_rows(signals.kat_bytes("nyquist", n), oracle.IN_F32_INTERLEAVED, n, 1, None, None)[0]
    assert int(np.argmax(ny)) == 0 and abs(ny[0]) < 1e-5  # bin N/2 -> out[0]
    z = oracle.spectrum_rows(signals.kat_bytes("zeros", n), oracle.IN_S8, n, 1, None, oracle.WIN_BLACKMAN)[0]
    assert np.all(np.isneginf(z))


def test_converters_bit_exact_against_reference_luts():
    b = np.arange(256, dtype=np.uint8)
    iq = np.stack([b, b[::-1]], 1).reshape(-1)
    re, im = oracle.convert(iq, oracle.IN_S8, 256)
    np.testing.assert_array_equal(re, (b.view(np.int8).astype(np.float32)) / np.float32(128))
    re, im = oracle.convert(iq, oracle.IN_U8, 256)  # Unsigned8BitIQConverter.java:48-50
    np.testing.assert_array_equal(re, (b.astype(np.float32) - np.float32(127.4)) / np.float32(128))
    s = np.array([-32768, -1, 0, 1, 32767, 1234], "<i2")
    re, im = oracle.convert(np.stack([s, s], 1).reshape(-1).view(np.uint8), oracle.IN_S16LE, s.size)
    np.testing.assert_array_equal(re, s.astype(np.float32) / np.float32(32768))


def test_blackman_window_matches_reference_formula():
    n = 1000
    w = oracle.window(n, oracle.WIN_BLACKMAN)
    i = np.arange(n)
    ref = (0.42 - 0.5 * np.cos(2 * np.pi * i / (n - 1)) + 0.08 * np.cos(4 * np.pi * i / (n - 1))).astype(np.float32)
    np.testing.assert_array_equal(w, ref)


def test_state_sequence_matches_fixture():
    spec = MANIFEST["state"]
    data = gu.fixture_input(spec)
    rows = oracle.ref_spectrum_rows(data, 0, spec["n"], spec["n_frames"]) if oracle.ref_available() else None
    if rows is None:
        pytest.skip("reference pffft build absent")
    p = processor.FftProcessorRef(spec["n"], spec["ring_rows"], peak_hold=True, ema_alpha=spec["ema_alpha"])
    for f in range(spec["n_frames"]):
        freq, sr = [t for t in spec["tuning"] if t[0] <= f][-1][1:]
        p.push(rows[f], freq, sr)
    exp = gu.expected(spec)
    np.testing.assert_array_equal(p.peaks, exp["peaks"])
    np.testing.assert_array_equal(p.ema, exp["ema"])
    np.testing.assert_array_equal(p.boxcar(spec["boxcar_length"]), exp["boxcar"])


def test_retune_shift_semantics():
    p = processor.FftProcessorRef(16, ring_rows=4)
    row = np.arange(16, dtype=np.float32)
    p.push(row, 1000, 16)  # samplesPerHz = 1
    p.push(row, 1003, 16)  # frequencyDiff = -3 -> shift left by 3, fill right
    older = p.ring[(p.read_index + 1) % 4]
    np.testing.assert_array_equal(older[:13], row[3:])
    assert np.all(older[13:] == -9999)
    p.push(row, 1003, 32)  # sample-rate change clears history
    assert np.all(p.ring[(p.read_index + 1) % 4] == -9999)
    assert processor.retune_shift_offset(-3, 16, 16) == -3
    assert processor.retune_shift_offset(7, 1024, 2_000_000) == 0  # truncation toward zero


def test_file_framing_config1():
    """Config 1: 4,000,000 B s8 file, 262,144 B packets -> 15 frames, 67,840 B tail dropped."""
    frames = processor.file_frames(4_000_000, 262_144, 2, 1024)
    assert len(frames) == 15 and frames[1][0] - frames[0][0] == 262_144
    assert 4_000_000 - 15 * 262_144 == 67_840
    big = processor.file_frames(4_000_000, 262_144, 2, 262_144)  # N > packet samples: 2 packets/frame
    assert len(big) == 7 and big[1][0] == 2 * 262_144


def test_config1_fixture_full_row_bar():
    """Config 1 replay fixture: the float64 restatement is within 0.01 dB of the
    reference's pffft rows on EVERY bin (no Parseval floor), so the GPU test can hold
    the product to the full-row bar too (tests/test_gpu_parity.py)."""
    spec = next(s for s in MANIFEST["fixtures"] if s["name"] == "file_s8_2msps_n1024")
    data = gu.fixture_input(spec)
    ref64 = oracle.spectrum_rows(data, oracle.IN_S8, 1024, 15, spec["packet_size"], oracle.WIN_BLACKMAN)
    st = gu.db_stats(ref64, gu.expected(spec), gu.FLOOR_PFFFT_DB)
    assert st["excluded"] < 0.001  # 2 of 15 360 bins fall below the 45 dB floor
    assert gu.full_row_diff(ref64, gu.expected(spec)) <= gu.DB_TOL
