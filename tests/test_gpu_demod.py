"""GPU: demod front end (rfa_ddc_*) bit-exact against the
restatement (oracle/demod.py) -- NCO mix of raw s8/u8/s16 bytes + decimating FIR
with state carried across ragged packets, retunes and rate changes."""
import numpy as np
import pytest

from oracle import demod as od
from rfanalyzer_amd import _lib
from rfanalyzer_amd import demod

pytestmark = pytest.mark.gpu

FMT = {"s8": od.IN_S8, "u8": od.IN_U8, "s16": od.IN_S16LE, "f32": od.IN_F32_INTERLEAVED}
SB = {"s8": 2, "u8": 2, "s16": 4, "f32": 8}


def _raw(fmt, n, seed):
    rng = np.random.default_rng(seed)
    if fmt == "s16":
        return rng.integers(-32768, 32768, 2 * n, dtype=np.int16).view(np.uint8)
    if fmt == "f32":
        return rng.standard_normal(2 * n).astype(np.float32).view(np.uint8)
    return rng.integers(0, 256, 2 * n, dtype=np.uint8)


def _same(a, b):
    assert a.shape == b.shape, (a.shape, b.shape)
    np.testing.assert_array_equal(a.view(np.int32), b.view(np.int32))


def _run_both(fmt, sr, out, sizes, seed, freqs=(100_000_000, 100_130_000)):
    raw = _raw(fmt, sum(sizes), seed)
    ref = od.FrontEnd(FMT[fmt], sr, out)
    fe = demod.FrontEnd(fmt, sr, out)
    ref.set_frequencies(*freqs)
    fe.set_frequencies(*freqs)
    pos = 0
    for n in sizes:
        chunk = raw[pos * SB[fmt]:(pos + n) * SB[fmt]]
        r_re, r_im = ref.process(chunk)
        g_re, g_im = fe.process(chunk)
        _same(g_re, r_re)
        _same(g_im, r_im)
        pos += n
    return fe, ref


@pytest.mark.parametrize("fmt", ["s8", "u8", "s16"])
@pytest.mark.parametrize("sr,out", [(2_400_000, 96_000), (1_000_000, 48_000), (10_000_000, 384_000)])
def test_mix_and_decimate_bit_exact(rfa, fmt, sr, out):
    fe, ref = _run_both(fmt, sr, out, [16384, 7, 1, 0, 5000, 123457], seed=sr + len(fmt))
    c, s, mf, ci = fe.mixer()
    _same(c, ref.cos_t)
    _same(s, ref.sin_t)
    assert mf == ref.cos_freq and ci == ref.cosine_index
    _same(fe.taps, ref.fir.taps)
    fe.close()


def test_filter_only_resampler_test_rates(rfa):
    """ResamplerTest.kt's Decimator case: float IQ at 48 kHz -> 12 kHz in 1024-sample packets."""
    fe, _ = _run_both("f32", 48_000, 12_000, [1024] * 46 + [896], seed=3)
    fe.close()


def test_long_filter_uses_several_lds_chunks(rfa):
    # 20 MHz -> 10 kHz: D = 2000, 21 819 taps, longer than one LDS chunk
    fe, ref = _run_both("s8", 20_000_000, 10_000, [150_000, 80_001], seed=8)
    assert len(fe.taps) > 8192 and fe.decimation == 2000
    fe.close()


def test_whole_buffer_equals_packets(rfa):
    raw = _raw("s8", 200_000, 11)
    a = demod.FrontEnd("s8", 2_400_000, 48_000)
    b = demod.FrontEnd("s8", 2_400_000, 48_000)
    for fe in (a, b):
        fe.set_frequencies(433_000_000, 433_250_000)
    whole = a.process(raw)
    parts = [b.process(raw[k:k + 2 * 4096]) for k in range(0, raw.size, 2 * 4096)]
    _same(whole[0], np.concatenate([p[0] for p in parts]))
    _same(whole[1], np.concatenate([p[1] for p in parts]))
    a.close(), b.close()


def test_retune_and_rate_change(rfa):
    raw = _raw("u8", 60_000, 12)
    ref = od.FrontEnd(od.IN_U8, 2_400_000, 48_000)
    fe = demod.FrontEnd("u8", 2_400_000, 48_000)
    steps = [(100_000_000, 100_200_000), (100_000_000, 100_200_000), (100_000_000, 99_700_000),
             (100_000_000, 100_000_000)]
    pos = 0
    for f, ch in steps:                    # an unchanged frequency keeps the cosine index
        ref.set_frequencies(f, ch)
        fe.set_frequencies(f, ch)
        chunk = raw[2 * pos:2 * (pos + 15_000)]
        r = ref.process(chunk)
        g = fe.process(chunk)
        _same(g[0], r[0]), _same(g[1], r[1])
        pos += 15_000
    # same decimation after a rate change: filter (and its delay line) kept, mixer regenerated
    fe.set_sample_rate(2_410_000)
    assert fe.decimation == 50
    fe.set_frequencies(100_000_000, 100_200_000)
    c, _, mf, ci = fe.mixer()
    assert mf == od.mix_frequency(100_000_000, 100_200_000, 2_410_000) and ci == 0
    # new decimation: rebuilt from scratch
    fe.set_sample_rate(1_200_000)
    assert fe.decimation == 25
    _, taps = od.decimator_taps(1_200_000, 48_000)
    _same(fe.taps, taps)
    fe.close()


class _Dev:
    """Device buffer from the same HIP runtime librfa links (/opt/rocm), via ctypes."""
    hip = None

    def __init__(self, nbytes):
        import ctypes
        if _Dev.hip is None:
            _Dev.hip = ctypes.CDLL("libamdhip64.so.7")
        self.ptr = ctypes.c_void_p()
        assert _Dev.hip.hipMalloc(ctypes.byref(self.ptr), ctypes.c_size_t(max(nbytes, 4))) == 0
        self.nbytes = nbytes

    def put(self, a):
        import ctypes
        a = np.ascontiguousarray(a)
        assert _Dev.hip.hipMemcpy(self.ptr, a.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(a.nbytes), 1) == 0

    def get(self, n, dtype=np.float32):
        import ctypes
        out = np.empty(n, dtype)
        assert _Dev.hip.hipMemcpy(out.ctypes.data_as(ctypes.c_void_p), self.ptr, ctypes.c_size_t(out.nbytes), 2) == 0
        return out

    def free(self):
        _Dev.hip.hipFree(self.ptr)


def test_device_pointers_and_capacity(rfa):
    raw_h = _raw("s16", 50_000, 4)
    raw = _Dev(raw_h.nbytes)
    raw.put(raw_h)
    fe = demod.FrontEnd("s16", 2_000_000, 50_000)
    fe.set_frequencies(7_000_000, 7_100_000)
    cap = fe.max_outputs(50_000)
    re, im = _Dev(4 * cap), _Dev(4 * cap)
    with pytest.raises(_lib.RfaError) as e:
        fe.process_device(raw.ptr.value, 50_000, re.ptr.value, im.ptr.value, 5)
    assert e.value.status == _lib.RFA_ERR_SIZE          # nothing consumed: the next call starts fresh
    n = fe.process_device(raw.ptr.value, 50_000, re.ptr.value, im.ptr.value, cap)
    fe.synchronize()
    ref = od.FrontEnd(od.IN_S16LE, 2_000_000, 50_000)
    ref.set_frequencies(7_000_000, 7_100_000)
    r = ref.process(raw_h)
    assert n == len(r[0]) == 50_000 // 40
    _same(re.get(n), r[0])
    _same(im.get(n), r[1])
    for b in (raw, re, im):
        b.free()
    fe.close()


def test_errors(rfa):
    with pytest.raises(_lib.RfaError):
        demod.FrontEnd("s8", 48_000, 40_000)            # cutoff 30 kHz > fs/2: createLowPassTaps -> null
    fe = demod.FrontEnd("s8", 1_000_000, 50_000)
    with pytest.raises(_lib.RfaError) as e:             # mixing before any channel is set
        fe.process(b"\x00" * 64)
    assert e.value.status == _lib.RFA_ERR_STATE
    fe.close()


def _run_resampler(fmt, sr, out, sizes, seed, freqs=(433_000_000, 433_120_000)):
    raw = _raw(fmt, sum(sizes), seed)
    ref = od.ResamplerFrontEnd(FMT[fmt], sr, out)
    fe = demod.FrontEnd(fmt, sr, out, resampler=True)
    ref.set_frequencies(*freqs)
    fe.set_frequencies(*freqs)
    i, d, t = fe.ratio()
    assert (i, d, t) == (ref.rs.I, ref.rs.D, ref.rs.nt)
    _same(fe.taps, ref.rs.proto)
    pos = 0
    for n in sizes:
        chunk = raw[pos * SB[fmt]:(pos + n) * SB[fmt]]
        r = ref.process(chunk)
        g = fe.process(chunk)
        _same(g[0], r[0])
        _same(g[1], r[1])
        pos += n
    return fe


@pytest.mark.parametrize("fmt,sr,out", [("u8", 2_400_000, 96_000),      # 1/25: one phase
                                        ("s8", 20_000_000, 384_000),    # 12/625: polyphase
                                        ("s16", 10_000_000, 96_000),    # 12/1250 -> 6/625
                                        ("f32", 48_000, 12_000)])       # ResamplerTest.kt rates
def test_resampler_bit_exact(rfa, fmt, sr, out):
    _run_resampler(fmt, sr, out, [16384, 3, 1, 0, 9000, 40_001], seed=len(fmt) + out).close()


def test_resampler_rate_change_rebuilds(rfa):
    fe = _run_resampler("s8", 2_000_000, 96_000, [5000], seed=1)
    fe.set_sample_rate(2_400_000)                  # Resampler.kt:102 recreates on any input-rate change
    assert fe.ratio()[:2] == (1, 25)
    fe.close()


def test_misaligned_device_input_takes_the_per_sample_loads(rfa):
    """A raw pointer not aligned to 4 samples uses the per-sample staging loop; same bits."""
    raw_h = _raw("s8", 30_001, 6)
    raw = _Dev(raw_h.nbytes)
    raw.put(raw_h)
    fe = demod.FrontEnd("s8", 2_400_000, 48_000)
    fe.set_frequencies(100_000_000, 100_070_000)
    cap = fe.max_outputs(30_000)
    re, im = _Dev(4 * cap), _Dev(4 * cap)
    n = fe.process_device(raw.ptr.value + 2, 30_000, re.ptr.value, im.ptr.value, cap)   # one sample in
    fe.synchronize()
    ref = od.FrontEnd(od.IN_S8, 2_400_000, 48_000)
    ref.set_frequencies(100_000_000, 100_070_000)
    r = ref.process(raw_h[2:])
    _same(re.get(n), r[0])
    _same(im.get(n), r[1])
    for b in (raw, re, im):
        b.free()
    fe.close()


def test_resampler_rejects_upsampling_and_keeps_state_on_bad_rate(rfa):
    with pytest.raises(_lib.RfaError) as e:
        demod.FrontEnd("s8", 48_000, 96_000, resampler=True)     # the reference only guarantees downsampling
    assert e.value.status == _lib.RFA_ERR_UNSUPPORTED
    fe = demod.FrontEnd("u8", 2_400_000, 96_000)
    with pytest.raises(_lib.RfaError):
        fe.set_sample_rate(100_000)                                # 0.75*96k > fs/2: design fails
    assert fe.decimation == 25                                     # the old filter is still in place
    fe.set_frequencies(100_000_000, 100_100_000)
    raw = _raw("u8", 10_000, 2)
    ref = od.FrontEnd(od.IN_U8, 2_400_000, 96_000)
    ref.set_frequencies(100_000_000, 100_100_000)
    g, r = fe.process(raw), ref.process(raw)
    _same(g[0], r[0]), _same(g[1], r[1])
    fe.close()


# ---------------------------------------------------------------- the reference's FIR golden vectors on the device
import fir_vectors  # noqa: E402


@pytest.mark.parametrize("case", fir_vectors.cases(), ids=lambda c: c["name"])
@pytest.mark.parametrize("split", [None, (1, 3, 7, 40)])
def test_fir_filter_matches_reference_vectors(rfa, case, split):
    """ApplicationTest.kt:20-176: FirFilter.createLowPass(...).filter(in, out) on the GPU
    (rfa_ddc_create_fir, pre-mixed f32 input) equals the JVM's outputs within the test's
    1e-9, whole or in ragged packets (delay line and decimation counter carried over;
    testFirFilter2 has D = 1: first output at input 1)."""
    re, im = fir_vectors.inputs(case)
    f = demod.FirFilter.createLowPass(case["decimation"], case["gain"], case["sample_rate"], case["cutoff"],
                                      case["transition"], case["attenuation"])
    assert f is not None and f.numberOfTaps == len(od.low_pass_taps(case["gain"], case["sample_rate"],
                                                                     case["cutoff"], case["transition"],
                                                                     case["attenuation"]))
    if split is None:
        got = f.filter(re, im)
    else:
        bounds = [0, *split, re.size]
        parts = [f.filter(re[a:b], im[a:b]) for a, b in zip(bounds, bounds[1:])]
        got = (np.concatenate([p[0] for p in parts]), np.concatenate([p[1] for p in parts]))
    fir_vectors.check(case, *got)
    f.close()


@pytest.mark.parametrize("offset,sr", [(25_000, 20_000_000), (4_000, 2_400_000), (1_000, 2_000_000),
                                       (-1_000, 2_000_000), (39_999, 20_000_000)])
def test_mixer_tables_near_the_centre_frequency(rfa, offset, sr):
    """Channels within sr/500 of the centre (the fold case of generateMixerLookupTable)
    demodulate bit-exact against the restatement (table sizes)."""
    out = 96_000 if sr < 10_000_000 else 384_000
    _run_both("s8", sr, out, [50_000, 3, 70_001], seed=offset & 0xffff,
              freqs=(100_000_000 + offset, 100_000_000))


def test_process_tensor_is_ordered_on_torch_stream(rfa):
    """process_tensor runs on torch's current stream: a torch op producing the input just
    before, and one reading the outputs just after, see the right data."""
    import torch
    raw = _raw("s8", 200_000, 77)
    want = od.FrontEnd(od.IN_S8, 2_400_000, 96_000)
    want.set_frequencies(100_000_000, 100_130_000)
    w_re, w_im = want.process(raw)
    fe = demod.FrontEnd("s8", 2_400_000, 96_000)
    fe.set_frequencies(100_000_000, 100_130_000)
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        src = torch.from_numpy(raw.copy()).to("cuda", non_blocking=False)
        big = torch.empty(64 << 20, dtype=torch.uint8, device="cuda")
        big.fill_(1)                                    # keeps the stream busy ahead of the copy
        t = torch.empty_like(src)
        t.copy_(src)                                    # producer on the current (side) stream
        cap = fe.max_outputs(200_000)
        o_re = torch.empty(cap, dtype=torch.float32, device="cuda")
        o_im = torch.empty(cap, dtype=torch.float32, device="cuda")
        n = fe.process_tensor(t, o_re, o_im)
        r_re, r_im = o_re[:n].clone(), o_im[:n].clone()  # consumer on the same stream
    s.synchronize()
    _same(r_re.cpu().numpy(), w_re)
    _same(r_im.cpu().numpy(), w_im)
    fe.close()
