"""GPU: the packet seam -- Scheduler.run's FFT branch fills one N-sample frame
across as many packets as it takes (Scheduler.kt:252-273 with
fillPacketIntoSamplePacket, Signed8BitIQConverter.java:80-98).  rfa_push_packet
and the JNI processPacketNative / processIqBytesNative (frame_stride 0) against
the literal restatement oracle.processor.scheduler_frames + FftProcessorRef."""
import ctypes

import numpy as np
import pytest

import golden_util as gu
import oracle
import signals
from jni_mock import MockJNIEnv
from oracle import processor

pytestmark = pytest.mark.gpu

_P = "Java_com_mantz_1it_nativedsp_NativeDsp_"
_V, _I32, _I64, _F, _U8 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_float, ctypes.c_uint8
_FMT_ID = {"s8": oracle.IN_S8, "u8": oracle.IN_U8, "s16": oracle.IN_S16LE}
_BPS = {"s8": 2, "u8": 2, "s16": 4}


def _native(rfa, name, restype, argtypes):
    fn = getattr(rfa.lib(), _P + name)
    fn.restype = restype
    fn.argtypes = [_V, _V] + argtypes
    return fn


def _expected(frames, n, fmt, rows_r):
    """Rows of the delivered frames (float64 oracle) pushed through the FftProcessor restatement."""
    p = processor.FftProcessorRef(n, rows_r, peak_hold=True)
    rows = []
    for data, f, r in frames:
        row = oracle.spectrum_rows(data, _FMT_ID[fmt], n, 1, None, oracle.WIN_BLACKMAN)[0]
        rows.append(row)
        p.push(row, f, r)
    return p, np.array(rows, np.float32).reshape(-1, n)


def _check_state(e, p):
    ring, ri, wi = e.ring()
    assert (ri, wi) == (p.read_index, p.write_index)
    for r in range(ring.shape[0]):
        fill = p.ring[r] == -9999
        np.testing.assert_array_equal(ring[r][fill], p.ring[r][fill])
        if (~fill).any():
            assert gu.db_diff(ring[r][~fill], p.ring[r][~fill]) <= gu.DB_TOL
    assert gu.db_diff(e.peaks(), p.peaks) <= gu.DB_TOL


@pytest.mark.parametrize("n", [16384, 65536])
def test_rtlsdr_packets_through_process_packet_native(rfa, n):
    """RTL-SDR: 16 KiB u8 packets = 8192 samples (RtlsdrSource.java:112) at N = 16384
    (the default, AppStateRepository.kt:196) and 65536: one row every N / 8192 packets,
    equal to rfa_process on the contiguous frames and to the oracle."""
    pkt, rows_r = 16384, 6
    per = n * 2 // pkt
    n_packets = per * 5 + per // 2  # 5 frames and a partial one left pending
    data = np.frombuffer(signals.frames_bytes(n, n_packets // per + 1, "u8", 5 + n // 1024,
                                              tones=((0.11, 0.3), (0.37, 0.05)), noise=0.04),
                         np.uint8)[: n_packets * pkt].copy()
    jenv = MockJNIEnv()
    create = _native(rfa, "createAnalyzerNative", _I64, [_I32, _I32, _I32, _I32, _I32, _F, _U8, _I32, _I32])
    process = _native(rfa, "processPacketNative", _I32, [_I64, _V, _I32, _I64, _I64])
    h = create(jenv.env, None, n, 1, 0, 0, 0, 0.1, 1, rows_r, 0)
    assert h != 0
    got = [process(jenv.env, None, h, jenv.new_array(data[i * pkt:(i + 1) * pkt].view(np.int8)), 0,
                   28_800_000, 2_400_000) for i in range(n_packets)]
    assert got == [1 if (i + 1) % per == 0 else 0 for i in range(n_packets)]
    # the same frames through the batch entry point (contiguous stride) and the oracle
    frames = processor.scheduler_frames([(data[i * pkt:(i + 1) * pkt].tobytes(), 28_800_000, 2_400_000)
                                         for i in range(n_packets)], n, 2)
    assert len(frames) == 5
    p, exp_rows = _expected(frames, n, "u8", rows_r)
    with rfa.SpectrumEngine(n, "blackman", "u8", peak_hold=True, ring_rows=rows_r) as e:
        e.set_tuning(28_800_000, 2_400_000)
        rows = e.process(data[: 5 * n * 2].tobytes(), 5)
        assert gu.db_diff(rows, exp_rows) <= gu.DB_TOL
        assert gu.full_row_diff(rows, exp_rows) <= gu.DB_TOL
        _check_state(e, p)
        ring_b, _, _ = e.ring()
        peaks_b = e.peaks()
    # the JNI handle's ring and peaks equal the batch handle's (same kernels, same frames)
    read = _native(rfa, "destroyAnalyzerNative", None, [_I64])
    eng = ctypes.c_void_p(h)
    lib = rfa.lib()
    ring = np.empty((rows_r, n), np.float32)
    ri, wi = ctypes.c_int32(), ctypes.c_int32()
    assert lib.rfa_get_ring(eng, ring.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), ctypes.byref(ri),
                            ctypes.byref(wi)) == 0
    np.testing.assert_array_equal(ring, ring_b)
    pk = np.empty(n, np.float32)
    assert lib.rfa_get_peaks(eng, pk.ctypes.data_as(ctypes.POINTER(ctypes.c_float))) == 0
    np.testing.assert_array_equal(pk, peaks_b)
    pend = ctypes.c_int64()
    assert lib.rfa_pending_samples(eng, ctypes.byref(pend)) == 0
    assert pend.value == (n_packets % per) * pkt // 2
    read(jenv.env, None, h)


@pytest.mark.parametrize("fmt", ["s8", "u8", "s16"])
def test_ragged_packets_retunes_and_long_packets(rfa, fmt):
    """Ragged packet sizes (odd byte counts, empty packets, packets longer than a frame
    whose rest is dropped) with retunes inside a partially filled frame: every frame
    takes the tuning of the packet that completes it."""
    n, rows_r = 4096, 5
    bps = _BPS[fmt]
    raw = signals.frames_bytes(n, 12, fmt, 91, tones=((0.21, 0.5),), noise=0.05)
    sizes = [3000, 0, 5001, 1, 9000, 2 * n * bps + 100, 777, 8190, 4 * n * bps, 10000, 12345, 333, 20000]
    packets, off = [], 0
    tunes = [(100_000_000, 2_000_000), (100_000_000, 2_000_000), (100_000_500, 2_000_000), (99_999_000, 2_000_000),
             (99_999_000, 4_000_000)]
    for i, s in enumerate(sizes):
        s = min(s, len(raw) - off)
        f, r = tunes[min(i // 3, len(tunes) - 1)]
        packets.append((raw[off:off + s], f, r))
        off += s
    frames = processor.scheduler_frames(packets, n, bps)
    assert len(frames) >= 5
    p, exp_rows = _expected(frames, n, fmt, rows_r)
    with rfa.SpectrumEngine(n, "blackman", fmt, peak_hold=True, ring_rows=rows_r) as e:
        got = []
        for data, f, r in packets:
            row = e.push_packet(data, f, r, row=True)
            if row is not None:
                got.append(row)
        assert len(got) == len(frames)
        got = np.array(got)
        assert gu.db_diff(got, exp_rows) <= gu.DB_TOL
        _check_state(e, p)
        assert 0 <= e.pending_samples() < n


def test_process_iq_bytes_native_fills_across_calls(rfa):
    """The stateless symbol in framing mode (frame_stride 0): rows appear every
    ceil(N / P) calls and equal the oracle row of the assembled frame."""
    n, pkt = 8192, 6000
    raw = signals.frames_bytes(n, 6, "s8", 5, tones=((0.3, 0.4),), noise=0.02)
    jenv = MockJNIEnv()
    fn = getattr(rfa.lib(), _P + "processIqBytesNative")
    fn.restype = _I32
    fn.argtypes = [_V, _V, _V, _I32, _I32, _I32, _V]
    packets = [raw[i:i + pkt] for i in range(0, len(raw) - pkt + 1, pkt)]
    frames = processor.scheduler_frames([(b, 0, 1) for b in packets], n, 2)
    rows = []
    for b in packets:
        out = np.zeros(n, np.float32)
        got = fn(jenv.env, None, jenv.new_array(np.frombuffer(b, np.int8).copy()), 0, n, 0, jenv.new_array(out))
        assert got in (0, 1)
        if got:
            rows.append(out)
    assert len(rows) == len(frames)
    exp = np.stack([oracle.spectrum_rows(f[0], oracle.IN_S8, n, 1, None, oracle.WIN_BLACKMAN)[0] for f in frames])
    assert gu.db_diff(np.stack(rows), exp) <= gu.DB_TOL
    # a mag_out shorter than one row is an error, not a silent partial copy
    assert fn(jenv.env, None, jenv.new_array(np.frombuffer(packets[0], np.int8).copy()), 0, n, 0,
              jenv.new_array(np.zeros(n - 1, np.float32))) == -1


def test_legacy_calls_alternate_without_losing_the_partial_frame(rfa):
    """The legacy symbols share an LRU cache of setups keyed by (N, format, window)
    (jni_shim.cpp handle_for): performFFT (f32, no window) between the packets of
    processIqBytesNative's framing mode (s8, Blackman) neither rebuilds that setup nor
    drops its partial frame -- every row of the reference framing arrives, and every
    performFFT result equals the reference's pffft.  (The cache is process-wide and keeps
    a setup's partial frame by design, so this test uses a setup key -- s8, N = 2048,
    Blackman -- that no other framing-mode test leaves half filled.)"""
    n, pkt = 2048, 1500
    raw = signals.frames_bytes(n, 6, "s8", 11, tones=((0.21, 0.5),), noise=0.03)
    jenv = MockJNIEnv()
    fn = getattr(rfa.lib(), _P + "processIqBytesNative")
    fn.restype = _I32
    fn.argtypes = [_V, _V, _V, _I32, _I32, _I32, _V]
    fft = getattr(rfa.lib(), _P + "performFFT")
    fft.restype = None
    fft.argtypes = [_V, _V, _V, _V]
    status = rfa.lib().rfa_jni_last_status
    status.restype = _I32
    packets = [raw[i:i + pkt] for i in range(0, len(raw) - pkt + 1, pkt)]
    frames = processor.scheduler_frames([(b, 0, 1) for b in packets], n, 2)
    rng = np.random.default_rng(5)
    rows = []
    for k, b in enumerate(packets):
        out = np.zeros(n, np.float32)
        got = fn(jenv.env, None, jenv.new_array(np.frombuffer(b, np.int8).copy()), 0, n, 0, jenv.new_array(out))
        assert got in (0, 1) and status() == 0
        if got:
            rows.append(out)
        m = (1024, 2048)[k % 2]  # two more setups in the cache between the packets
        x = rng.standard_normal(2 * m).astype(np.float32)
        y = np.zeros(2 * m, np.float32)
        fft(jenv.env, None, jenv.new_array(x), jenv.new_array(y))
        assert status() == 0
        if oracle.ref_available():
            ref = oracle.ref_fft_ordered(x)
            assert np.abs(y - ref).max() / np.abs(ref).max() < 1e-5
    assert len(rows) == len(frames)
    exp = np.stack([oracle.spectrum_rows(f[0], oracle.IN_S8, n, 1, None, oracle.WIN_BLACKMAN)[0] for f in frames])
    assert gu.db_diff(np.stack(rows), exp) <= gu.DB_TOL


@pytest.mark.parametrize("m", [8, 40, 112, 1000])
def test_legacy_unsupported_length_reports_status(rfa, m):
    """Lengths the reference's pffft rejects (not a multiple of 16, or a factor other
    than 2, 3, 5: pffft.c:1236-1277, where the reference asserts or gets a null setup):
    the void legacy symbol leaves its output untouched and rfa_jni_last_status() says
    RFA_ERR_UNSUPPORTED; the next supported call resets it to RFA_OK.  (Every length
    pffft takes is served: tests/test_gpu_seam.py.)"""
    jenv = MockJNIEnv()
    status = rfa.lib().rfa_jni_last_status
    status.restype = _I32
    for name in ("performFFT", "performFFTAndLogMag"):
        fn = getattr(rfa.lib(), _P + name)
        fn.restype = None
        fn.argtypes = [_V, _V, _V, _V]
        x = np.ones(2 * m, np.float32)
        out = np.full(2 * m, 7.0, np.float32)
        arr = jenv.new_array(out)
        fn(jenv.env, None, jenv.new_array(x), arr)
        assert status() == -3  # RFA_ERR_UNSUPPORTED
        assert np.all(out == 7.0)
        good = np.zeros(2 * 64, np.float32)
        fn(jenv.env, None, jenv.new_array(np.ones(2 * 64, np.float32)), jenv.new_array(good))
        assert status() == 0


def test_push_packet_checks_only_the_completing_packets_rate(rfa):
    """Only the packet that completes a frame supplies the tuning
    (Signed8BitIQConverter.java:95-97), so a partial packet with sample rate 0 is
    accepted and buffered; a completing packet with rate 0 is an error that drops
    the frame."""
    n = 4096
    raw = signals.frames_bytes(n, 3, "s8", 21, tones=((0.1, 0.5),), noise=0.02)
    half = n  # bytes = n / 2 samples of s8 IQ
    with rfa.SpectrumEngine(n, "blackman", "s8", ring_rows=4) as e:
        assert e.push_packet(raw[:half], 0, 0) is False
        assert e.pending_samples() == n // 2
        row = e.push_packet(raw[half:2 * half], 100_000_000, 2_000_000, row=True)
        assert row is not None
        exp = oracle.spectrum_rows(raw[:2 * half], oracle.IN_S8, n, 1, None, oracle.WIN_BLACKMAN)[0]
        assert gu.db_diff(row, exp) <= gu.DB_TOL
        assert e.push_packet(raw[2 * half:3 * half], 0, 0) is False
        with pytest.raises(Exception):
            e.push_packet(raw[3 * half:4 * half], 100_000_000, 0)
        assert e.pending_samples() == 0
