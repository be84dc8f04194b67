"""TEST INFRASTRUCTURE ONLY -- restatement of the reference's demod-branch front end.

SURVEY.md §8(f) row 4: the NCO down-mix of raw IQ bytes
(``IQConverter.mixPacketIntoSamplePacket``) followed by the decimating low-pass
FIR (``Decimator.downsampling`` -> ``FirFilter.filter``).  Paths relative to
app/src/main/java/com/mantz_it/rfanalyzer/:

* mixer fold and table: source/Signed8BitIQConverter.java:53-77 (u8 identical,
  Unsigned8BitIQConverter.java:53-77 with the (i-127.4f)/128 LUT),
  source/Signed16BitIQConverter.kt:59-87 (different angle rounding);
* table length: source/IQConverter.java:64-76 (calcOptimalCosineLength);
* mix loop: Signed8BitIQConverter.java:101-130, Signed16BitIQConverter.kt:126-181;
* filter design: dsp/FirFilter.kt:134-195 (createLowPassTaps, Blackman window of
  dsp/WindowFunctions.kt:44-52) with the arguments of analyzer/Decimator.java:177-181;
* filter loop: dsp/FirFilter.kt:63-107 (circular delay line, decimationCounter
  starting at 1, sequential float sum newest sample first).

Float32 semantics are kept per operation (numpy float32 scalars and arrays round
every product and sum; no fused multiply-add).  ``math.sin``/``math.cos`` are the
platform libm; the JVM's Math.sin/cos may differ from it by one double ulp, which
after the cast to float almost never shows -- the device library computes its
tables with the same libm, so GPU parity with this file is exact, and parity with
the JVM is pinned only through the reference's own test (ResamplerTest.kt:20-116:
a 100 Hz tone through Decimator 48 kHz -> 12 kHz) as a property, not by vectors.
"""
from __future__ import annotations

import math

import numpy as np

F32 = np.float32
MAX_COSINE_LENGTH = 500                      # IQConverter.java:39
IN_S8, IN_U8, IN_S16LE, IN_F32_INTERLEAVED = 0, 1, 2, 3


def _i32(v: int) -> int:
    return (v + 2 ** 31) % 2 ** 32 - 2 ** 31


def _jtoint(x: float) -> int:
    """Java/Kotlin (int) of a double: truncate, saturate, NaN -> 0."""
    if math.isnan(x):
        return 0
    if x >= 2 ** 31 - 1:
        return 2 ** 31 - 1
    if x <= -2 ** 31:
        return -2 ** 31
    return int(x)


def mix_frequency(frequency: int, channel_frequency: int, sample_rate: int) -> int:
    """(int)(frequency - channelFrequency) then the fold of generateMixerLookupTable:
    += sampleRate when 0 or when sampleRate / |mix| > MAX_COSINE_LENGTH (int math)."""
    mix = _i32(frequency - channel_frequency)
    a = abs(mix) if mix != -2 ** 31 else mix          # Math.abs(Integer.MIN_VALUE) stays negative
    q = (abs(sample_rate) // abs(a)) * (1 if (sample_rate < 0) == (a < 0) else -1) if a != 0 else 0  # truncating
    if mix == 0 or q > MAX_COSINE_LENGTH:
        mix = _i32(mix + sample_rate)
    return mix


def optimal_cosine_length(sample_rate: int, cosine_frequency: int) -> int:
    """IQConverter.calcOptimalCosineLength (IQConverter.java:64-76)."""
    cycle = sample_rate / abs(float(cosine_frequency))
    best = _jtoint(cycle)
    err = abs(best - cycle)
    i = 1
    while i * cycle < MAX_COSINE_LENGTH:
        if abs(i * cycle - _jtoint(i * cycle)) < err:
            best = _jtoint(i * cycle)
            err = abs(best - i * cycle)
        i += 1
    return best


def mixer_table(fmt: int, sample_rate: int, cosine_frequency: int):
    """Per-time-step cos/sin (float) of the mixer table.  The 8-bit converters store
    lut[b] * cos_t; that product is formed per sample in ``mix`` with the same rounding."""
    n = optimal_cosine_length(sample_rate, cosine_frequency)
    c = np.empty(n, F32)
    s = np.empty(n, F32)
    if fmt == IN_S16LE:   # Signed16BitIQConverter.kt:73-81
        w = (2.0 * math.pi * cosine_frequency) / float(sample_rate)
        for t in range(n):
            c[t] = F32(math.cos(w * t))
            s[t] = F32(math.sin(w * t))
    else:                 # Signed8BitIQConverter.java:68-70: 2*PI*f*t / (float)sampleRate in double
        fsr = float(F32(sample_rate))
        for t in range(n):
            x = 2 * math.pi * cosine_frequency * t / fsr
            c[t] = F32(math.cos(x))
            s[t] = F32(math.sin(x))
    return c, s


def lut(fmt: int, raw: bytes | np.ndarray):
    """Byte -> float lookup of the three converters: (I, Q) float32 arrays."""
    raw = np.frombuffer(bytes(raw), np.uint8) if not isinstance(raw, np.ndarray) else raw
    if fmt == IN_S8:
        v = raw.view(np.int8).astype(F32) / F32(128.0)
    elif fmt == IN_U8:
        v = (raw.astype(F32) - F32(127.4)) / F32(128.0)
    elif fmt == IN_S16LE:
        v = raw.view("<i2").astype(F32) / F32(32768.0)
    else:
        raise ValueError(fmt)
    return v[0::2], v[1::2]


def mix(fmt: int, raw, cos_t, sin_t, cosine_index: int):
    """mixPacketIntoSamplePacket body: re = I*c - Q*s, im = Q*c + I*s, index wraps."""
    i, q = lut(fmt, raw)
    t = (cosine_index + np.arange(len(i))) % len(cos_t)
    c, s = cos_t[t], sin_t[t]
    return (i * c - q * s).astype(F32), (q * c + i * s).astype(F32)


def blackman(n: int, N: int) -> np.float32:
    """BlackmanWindow.value (WindowFunctions.kt:44-49)."""
    c1 = F32(math.cos(2.0 * math.pi * n / (N - 1)))
    c2 = F32(math.cos(4.0 * math.pi * n / (N - 1)))
    return F32(F32(F32(0.42) - F32(0.5) * c1) + F32(0.08) * c2)


def low_pass_taps(gain: float, sample_rate: float, cutoff: float, transition: float, attenuation: float,
                  max_taps: int = 0):
    """FirFilter.createLowPassTaps (FirFilter.kt:134-195); None where it returns null."""
    g, fs, fc, tw, att = (F32(v) for v in (gain, sample_rate, cutoff, transition, attenuation))
    if fs <= 0.0 or fc <= 0.0 or fc > fs / F32(2) or tw <= 0:
        return None
    ntaps = _jtoint(float(att * fs) / (22.0 * float(tw)))
    if max_taps > 0:
        ntaps = min(ntaps, max_taps)
    if ntaps & 1 == 0:
        ntaps += 1
    pi = F32(math.pi)
    taps = np.empty(ntaps, F32)
    M = (ntaps - 1) // 2
    fwt0 = F32(F32(F32(2) * pi) * fc) / fs
    for n in range(-M, M + 1):
        w = blackman(n + M, ntaps)
        if n == 0:
            taps[n + M] = F32(fwt0 / pi) * w
        else:
            taps[n + M] = F32(F32(math.sin(float(F32(n) * fwt0))) / F32(F32(n) * pi)) * w
    fmax = taps[M]
    for n in range(1, M + 1):
        fmax = F32(fmax + F32(2) * taps[n + M])
    gain_n = F32(g / fmax)
    return (taps * gain_n).astype(F32)


def decimator_taps(sample_rate: int, output_rate: int):
    """Decimator.downsampling's filter (Decimator.java:177-181)."""
    d = sample_rate // output_rate
    taps = low_pass_taps(1, float(F32(sample_rate)), F32(output_rate) * F32(0.75), F32(output_rate) * F32(0.25), 60)
    return d, taps


class FirDecimator:
    """FirFilter.filter state machine (FirFilter.kt:42-46,63-107): delay line of
    len(taps) zeros, tapCounter 0, decimationCounter 1.  ``filter`` is the
    vectorised form (outputs at once, taps in the reference's order);
    ``filter_literal`` is the per-sample loop for small cases."""

    def __init__(self, taps, decimation: int):
        self.taps = np.asarray(taps, F32)
        self.d = decimation
        T = len(self.taps)
        self.hist_re = np.zeros(T - 1, F32)   # the T-1 newest samples before the next input
        self.hist_im = np.zeros(T - 1, F32)
        self.counter = 1
        # literal-form state
        self._dre = np.zeros(T, F32)
        self._dim = np.zeros(T, F32)
        self._tap = 0

    def filter(self, re, im):
        re, im = np.asarray(re, F32), np.asarray(im, F32)
        T, S, D = len(self.taps), len(re), self.d
        xre = np.concatenate([self.hist_re, re])
        xim = np.concatenate([self.hist_im, im])
        # decimationCounter starts at 1 and wraps to 0 when it reaches D (FirFilter.kt:46,101-103):
        # outputs at inputs with counter == 0, i.e. (counter + j) % D == 0 -- except D = 1,
        # where the initial 1 is checked once before it becomes 0 (first output at input 1)
        first = 1 if (D == 1 and self.counter == 1) else ((D - self.counter) % D if D > 0 else 0)
        js = np.arange(first, S, max(D, 1))
        ore = np.zeros(len(js), F32)
        oim = np.zeros(len(js), F32)
        for k in range(T):
            ore = ore + self.taps[k] * xre[T - 1 + js - k]
            oim = oim + self.taps[k] * xim[T - 1 + js - k]
        self.hist_re = xre[len(xre) - (T - 1):].copy() if T > 1 else xre[:0]
        self.hist_im = xim[len(xim) - (T - 1):].copy() if T > 1 else xim[:0]
        self.counter = (self.counter + S) % D if D > 0 else 0
        return ore.astype(F32), oim.astype(F32)

    def filter_literal(self, re, im):
        taps, T = self.taps, len(self.taps)
        out_re, out_im = [], []
        for x, y in zip(np.asarray(re, F32), np.asarray(im, F32)):
            self._dre[self._tap] = x
            self._dim[self._tap] = y
            if self.counter == 0:
                a, b = F32(0), F32(0)
                idx = self._tap
                for t in taps:
                    a = F32(a + F32(t * self._dre[idx]))
                    b = F32(b + F32(t * self._dim[idx]))
                    idx = idx - 1 if idx > 0 else T - 1
                out_re.append(a)
                out_im.append(b)
            self.counter += 1
            if self.counter >= self.d:
                self.counter = 0
            self._tap = self._tap + 1 if self._tap + 1 < T else 0
        return np.array(out_re, F32), np.array(out_im, F32)


class FrontEnd:
    """Scheduler demod branch + Decimator for one channel: mix the raw packet, then
    filter-decimate it.  ``fmt`` IN_F32_INTERLEAVED feeds already-mixed float samples
    straight to the filter (Decimator on a SamplePacket, ResamplerTest.kt:56-62)."""

    def __init__(self, fmt: int, sample_rate: int, output_rate: int, taps=None, decimation=None):
        self.fmt, self.sample_rate = fmt, sample_rate
        if taps is not None:  # a FirFilter(taps, decimation) of the caller's (FirFilter.kt:34-46)
            self.d = int(decimation)
        else:
            self.d, taps = decimator_taps(sample_rate, output_rate)
        if taps is None:
            raise ValueError("filter design rejected the rates")
        self.fir = FirDecimator(taps, self.d)
        self.cos_freq = None
        self.cos_t = self.sin_t = None
        self.cosine_index = 0

    def set_frequencies(self, frequency: int, channel_frequency: int):
        mf = mix_frequency(frequency, channel_frequency, self.sample_rate)
        if self.cos_t is None or mf != self.cos_freq:
            self.cos_freq = mf
            self.cos_t, self.sin_t = mixer_table(self.fmt, self.sample_rate, mf)
            self.cosine_index = 0

    def process(self, raw):
        if self.fmt == IN_F32_INTERLEAVED:
            v = np.frombuffer(bytes(raw), F32) if not isinstance(raw, np.ndarray) else raw.view(F32)
            return self.fir.filter(v[0::2], v[1::2])
        if len(self.cos_t) == 0:
            return np.zeros(0, F32), np.zeros(0, F32)
        re, im = mix(self.fmt, raw, self.cos_t, self.sin_t, self.cosine_index)
        self.cosine_index = (self.cosine_index + len(re)) % len(self.cos_t)
        return self.fir.filter(re, im)


class CFrontEnd(FrontEnd):
    """The same front end through the literal per-sample C loop (rfa_oracle.c
    orc_ddc_process): second restatement for the tests, scalar CPU baseline for
    scripts/ddc_bench.py."""

    def __init__(self, fmt: int, sample_rate: int, output_rate: int, taps=None, decimation=None):
        super().__init__(fmt, sample_rate, output_rate, taps, decimation)
        T = len(self.fir.taps)
        self._dre = np.zeros(T, F32)
        self._dim = np.zeros(T, F32)
        self._ctr = np.array([0, 1, 0], np.int32)      # tapCounter, decimationCounter, cosineIndex

    def set_frequencies(self, frequency: int, channel_frequency: int):
        old = self.cos_freq
        super().set_frequencies(frequency, channel_frequency)
        if self.cos_freq != old:
            self._ctr[2] = 0

    def process(self, raw):
        import ctypes
        from . import orc
        buf = np.ascontiguousarray(np.frombuffer(bytes(raw), np.uint8) if not isinstance(raw, np.ndarray)
                                   else raw.view(np.uint8).reshape(-1))
        sb = {IN_S8: 2, IN_U8: 2, IN_S16LE: 4, IN_F32_INTERLEAVED: 8}[self.fmt]
        n = buf.size // sb
        mixed = self.fmt != IN_F32_INTERLEAVED
        if mixed and len(self.cos_t) == 0:
            return np.zeros(0, F32), np.zeros(0, F32)
        cap = n // self.d + 1
        ore = np.empty(cap, F32)
        oim = np.empty(cap, F32)
        fp = ctypes.POINTER(ctypes.c_float)
        ptr = (lambda a: a.ctypes.data_as(fp))
        k = orc().orc_ddc_process(self.fmt, buf.ctypes.data, n, ptr(self.cos_t) if mixed else None,
                                  ptr(self.sin_t) if mixed else None, len(self.cos_t) if mixed else 0,
                                  ptr(self.fir.taps), len(self.fir.taps), self.d, ptr(self._dre), ptr(self._dim),
                                  self._ctr.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), ptr(ore), ptr(oim))
        return ore[:k], oim[:k]


# ---------------------------------------------------------------- RationalResampler
# dsp/RationalResampler.kt (the resampler the live app's Demodulator uses through
# analyzer/Resampler.kt:102-110: limitDenominator(out, in, 10000), maxTaps 500).

def gcd(a: int, b: int) -> int:
    x, y = abs(a), abs(b)
    while y != 0:
        x, y = y, x % y
    return x


def limit_denominator(num: int, den: int, max_den: int = 10000):
    """RationalResampler.limitDenominator (RationalResampler.kt:165-203)."""
    target = num / den
    g0 = gcd(num, den)
    if den // g0 <= max_den:
        return num // g0, den // g0
    ln, ld, un, ud = 0, 1, 1, 0
    while True:
        mn, md = ln + un, ld + ud
        if md > max_den:
            break
        if mn / md < target:
            ln, ld = mn, md
        else:
            un, ud = mn, md
    return (ln, ld) if abs(target - ln / ld) < abs(target - un / ud) else (un, ud)


def _izero(x: float) -> float:
    s, term, half, k = 1.0, 1.0, x / 2.0, 1
    while True:
        tmp = half / k
        term *= tmp * tmp
        s += term
        if term < 1e-12:
            break
        k += 1
    return s


def kaiser(n: int, N: int, beta: float = 7.0) -> np.float32:
    """KaiserWindow.value (WindowFunctions.kt:63-80)."""
    ibeta = 1.0 / _izero(beta)
    if n == 0 or n == N - 1:
        return F32(ibeta)
    inm1 = 1.0 / float(N - 1)
    temp = 2.0 * n * inm1 - 1.0
    return F32(_izero(beta * math.sqrt(1.0 - temp * temp)) * ibeta)


def low_pass_taps_window(gain, sample_rate, cutoff, transition, attenuation, max_taps, window):
    """createLowPassTaps with an explicit window function (FirFilter.kt:134-195)."""
    g, fs, fc, tw, att = (F32(v) for v in (gain, sample_rate, cutoff, transition, attenuation))
    if fs <= 0.0 or fc <= 0.0 or fc > fs / F32(2) or tw <= 0:
        return None
    ntaps = _jtoint(float(att * fs) / (22.0 * float(tw)))
    if max_taps > 0:
        ntaps = min(ntaps, max_taps)
    if ntaps & 1 == 0:
        ntaps += 1
    pi = F32(math.pi)
    taps = np.empty(ntaps, F32)
    M = (ntaps - 1) // 2
    fwt0 = F32(F32(F32(2) * pi) * fc) / fs
    for n in range(-M, M + 1):
        w = window(n + M, ntaps)
        if n == 0:
            taps[n + M] = F32(fwt0 / pi) * w
        else:
            taps[n + M] = F32(F32(math.sin(float(F32(n) * fwt0))) / F32(F32(n) * pi)) * w
    fmax = taps[M]
    for n in range(1, M + 1):
        fmax = F32(fmax + F32(2) * taps[n + M])
    return (taps * F32(g / fmax)).astype(F32)


def design_resampler_taps(I: int, D: int, fractional_bw: float = 0.4, max_taps: int = 0):
    """RationalResampler.designResamplerTaps (RationalResampler.kt:210-235)."""
    halfband = 0.5
    fbw = float(F32(fractional_bw))
    rate = F32(F32(I) / F32(D))
    if rate >= F32(1.0):
        tw = F32(halfband - fbw)
        mid = F32(halfband - float(tw) / 2.0)
    else:
        tw = F32(float(rate) * (halfband - fbw))
        mid = F32(float(rate) * halfband - float(tw) / 2.0)
    t = low_pass_taps_window(I, I, mid, tw, F32(72.22087), max_taps * I, kaiser)
    return np.zeros(0, F32) if t is None else t


class RationalResampler:
    """RationalResampler state machine (RationalResampler.kt:27-127).  ``resample``
    is the closed form used for parity (output n: newest input (n*D)//I, phase
    (n*D) % I, taps summed in the reference's order); ``resample_literal`` the
    reference's per-call loop, for small cases."""

    def __init__(self, interpolation: int, decimation: int, max_taps: int = 0, fractional_bw: float = 0.4):
        if not (0 < fractional_bw < 0.5):
            fractional_bw = 0.4
        g = gcd(interpolation, decimation)
        self.I, self.D = interpolation // g, decimation // g
        proto = list(design_resampler_taps(self.I, self.D, fractional_bw, max_taps))
        while len(proto) % self.I:
            proto.append(F32(0))
        self.proto = np.array(proto, F32)
        self.nt = len(proto) // self.I
        self.bank = np.stack([self.proto[p::self.I] for p in range(self.I)]).astype(F32)   # firTaps[phase][i]
        self.hist_re = np.zeros(self.nt - 1, F32)
        self.hist_im = np.zeros(self.nt - 1, F32)
        self.n_done = self.in_done = 0
        # literal state
        self._dre = np.zeros(self.nt, F32)
        self._dim = np.zeros(self.nt, F32)
        self._di = 0
        self._ctr = 0

    def _n_total(self, in_total):
        lim = in_total * self.I
        return (lim + self.D - 1) // self.D if lim > 0 else 0

    def resample(self, re, im):
        re, im = np.asarray(re, F32), np.asarray(im, F32)
        S, T = len(re), self.nt
        xre = np.concatenate([self.hist_re, re])
        xim = np.concatenate([self.hist_im, im])
        ns = np.arange(self.n_done, self._n_total(self.in_done + S), dtype=np.int64)
        c = (ns * self.D) // self.I - self.in_done + (T - 1)
        ph = (ns * self.D) % self.I
        ore = np.zeros(len(ns), F32)
        oim = np.zeros(len(ns), F32)
        for t in range(T):
            w = self.bank[ph, t]
            ore = ore + w * xre[c - t]
            oim = oim + w * xim[c - t]
        self.hist_re = xre[len(xre) - (T - 1):].copy() if T > 1 else xre[:0]
        self.hist_im = xim[len(xim) - (T - 1):].copy() if T > 1 else xim[:0]
        self.n_done += len(ns)
        self.in_done += S
        return ore.astype(F32), oim.astype(F32)

    def resample_literal(self, re, im):
        re, im = np.asarray(re, F32), np.asarray(im, F32)
        length, nt = len(re), self.nt
        out_re, out_im = [], []
        if length == 0:
            return np.zeros(0, F32), np.zeros(0, F32)
        consumed, idx = 0, 0
        self._dre[self._di], self._dim[self._di] = re[0], im[0]

        def advance():
            nonlocal consumed, idx
            while self._ctr >= self.I:
                self._ctr -= self.I
                idx += 1
                self._di = self._di + 1 if self._di + 1 < nt else 0
                consumed += 1
                if consumed >= length:
                    break
                self._dre[self._di], self._dim[self._di] = re[idx], im[idx]

        advance()
        while consumed < length:
            a, b = F32(0), F32(0)
            di = self._di
            for t in self.bank[self._ctr]:
                a = F32(a + F32(t * self._dre[di]))
                b = F32(b + F32(t * self._dim[di]))
                di = di - 1 if di > 0 else nt - 1
            out_re.append(a)
            out_im.append(b)
            self._ctr += self.D
            advance()
        return np.array(out_re, F32), np.array(out_im, F32)


class ResamplerFrontEnd(FrontEnd):
    """Scheduler mix + Resampler (Resampler.kt:102-110) for one channel."""

    def __init__(self, fmt: int, sample_rate: int, output_rate: int):
        self.fmt, self.sample_rate = fmt, sample_rate
        i, d = limit_denominator(output_rate, sample_rate, 10000)
        self.rs = RationalResampler(i, d, max_taps=500)
        self.cos_freq = None
        self.cos_t = self.sin_t = None
        self.cosine_index = 0

    def process(self, raw):
        if self.fmt == IN_F32_INTERLEAVED:
            v = np.frombuffer(bytes(raw), F32) if not isinstance(raw, np.ndarray) else raw.view(F32)
            return self.rs.resample(v[0::2], v[1::2])
        if len(self.cos_t) == 0:
            return np.zeros(0, F32), np.zeros(0, F32)
        re, im = mix(self.fmt, raw, self.cos_t, self.sin_t, self.cosine_index)
        self.cosine_index = (self.cosine_index + len(re)) % len(self.cos_t)
        return self.rs.resample(re, im)
