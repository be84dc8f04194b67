"""Demod-branch front end on the GPU.

Host mirror of what the reference's demodulation branch does before the
demodulator proper (paths relative to app/src/main/java/com/mantz_it/rfanalyzer/):

* ``Scheduler.run`` hands every raw packet to ``source.mixPacketIntoSamplePacket(
  packet, demodBuffer, channelFrequency)`` (analyzer/Scheduler.kt:237-245), i.e.
  ``IQConverter.mixPacketIntoSamplePacket`` (source/Signed8BitIQConverter.java:101-130,
  Unsigned8BitIQConverter.java:101-130, Signed16BitIQConverter.kt:126-181): LUT
  conversion and an NCO down-mix by ``(int)(frequency - channelFrequency)``;
* ``Decimator.downsampling`` (analyzer/Decimator.java:175-191) filters the mixed
  packet with ``FirFilter.createLowPass(decimation, 1, inRate, 0.75*out, 0.25*out, 60)``
  and keeps every decimation-th output (dsp/FirFilter.kt:63-107).

``FrontEnd`` runs both in one HIP kernel (``rfanalyzer_amd/csrc/ddc.hip``) through
the C-ABI ``rfa_ddc_*`` (include/rfa.h).  Filter and mixer state carry over between
calls exactly as in the reference, so feeding packets one by one or a whole buffer
at once gives the same samples.  There is no CPU fallback: without librfa.so or a
HIP device every call raises.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib

FORMATS = {"s8": 0, "u8": 1, "s16": 2, "f32": 3}     # f32: already-mixed interleaved I,Q (filter only)
BYTES_PER_SAMPLE = {0: 2, 1: 2, 2: 4, 3: 8}


def create_low_pass_taps(gain: float, sample_rate: float, cutoff_frequency: float, transition_width: float,
                         attenuation_db: float, max_taps: int = 0) -> np.ndarray | None:
    """FirFilter.createLowPassTaps (dsp/FirFilter.kt:134-195), Blackman window; None where
    the reference returns null.  Host-only (no device work)."""
    L = _lib.lib()
    n = ctypes.c_int32(0)
    st = L.rfa_lowpass_taps(gain, sample_rate, cutoff_frequency, transition_width, attenuation_db, max_taps,
                            None, 0, ctypes.byref(n))
    if st == _lib.RFA_ERR_INVALID:
        return None
    _lib.check(st, "rfa_lowpass_taps")
    taps = np.empty(n.value, np.float32)
    _lib.check(L.rfa_lowpass_taps(gain, sample_rate, cutoff_frequency, transition_width, attenuation_db, max_taps,
                                  taps.ctypes.data_as(_lib._fp), taps.size, ctypes.byref(n)), "rfa_lowpass_taps")
    return taps


class FrontEnd:
    """One demodulated channel: mix + decimate raw IQ on ``device``.

    ``resampler=True`` filters with the live app's Resampler (analyzer/Resampler.kt:
    RationalResampler of limitDenominator(out, in, 10000), Kaiser taps) instead of the
    Decimator.
    ``input_format`` "s8" (HackRF), "u8" (RTL-SDR), "s16" (Airspy/HydraSDR) or "f32"
    (already-mixed interleaved floats: the Decimator alone, as ResamplerTest drives it).
    """

    def __init__(self, input_format: str, sample_rate: int, output_sample_rate: int, device: int = 0,
                 resampler: bool = False, _fir=None):
        if input_format not in FORMATS:
            raise ValueError(f"input_format must be one of {sorted(FORMATS)}")
        self.fmt = FORMATS[input_format]
        self.output_sample_rate = output_sample_rate
        self.resampler = resampler
        self._stream = None
        h = _lib._h()
        if _fir is not None:  # FirFilter(taps, decimation): see FirFilter below
            taps, decimation = _fir
            taps = np.ascontiguousarray(taps, np.float32)
            _lib.check(_lib.lib().rfa_ddc_create_fir(device, self.fmt, sample_rate, taps.ctypes.data_as(_lib._fp),
                                                     taps.size, decimation, ctypes.byref(h)), "rfa_ddc_create_fir")
        else:
            create = _lib.lib().rfa_ddc_create_resampler if resampler else _lib.lib().rfa_ddc_create
            _lib.check(create(device, self.fmt, sample_rate, output_sample_rate, ctypes.byref(h)),
                       "rfa_ddc_create_resampler" if resampler else "rfa_ddc_create")
        self._h = h

    # -- lifetime
    def close(self) -> None:
        if getattr(self, "_h", None):
            _lib.lib().rfa_ddc_destroy(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001 - interpreter shutdown
            pass

    def _check(self, status: int, where: str) -> None:
        if status != _lib.RFA_OK:
            detail = (_lib.lib().rfa_ddc_last_error(self._h) or b"").decode()
            raise _lib.RfaError(status, where, detail)

    # -- configuration (IQConverter.setSampleRate / mixPacketIntoSamplePacket's table check)
    def set_sample_rate(self, sample_rate: int) -> None:
        self._check(_lib.lib().rfa_ddc_set_sample_rate(self._h, sample_rate), "rfa_ddc_set_sample_rate")

    def set_frequencies(self, frequency: int, channel_frequency: int) -> None:
        self._check(_lib.lib().rfa_ddc_set_frequencies(self._h, frequency, channel_frequency),
                    "rfa_ddc_set_frequencies")

    @property
    def taps(self) -> np.ndarray:
        n, d = ctypes.c_int32(0), ctypes.c_int32(0)
        self._check(_lib.lib().rfa_ddc_get_taps(self._h, None, 0, ctypes.byref(n), ctypes.byref(d)), "get_taps")
        out = np.empty(n.value, np.float32)
        self._check(_lib.lib().rfa_ddc_get_taps(self._h, out.ctypes.data_as(_lib._fp), out.size, ctypes.byref(n),
                                                ctypes.byref(d)), "get_taps")
        return out

    @property
    def decimation(self) -> int:
        n, d = ctypes.c_int32(0), ctypes.c_int32(0)
        self._check(_lib.lib().rfa_ddc_get_taps(self._h, None, 0, ctypes.byref(n), ctypes.byref(d)), "get_taps")
        return d.value

    def mixer(self):
        """(cos_t, sin_t, mix_frequency, cosine_index) of the current mixer table."""
        n, mf, ci = ctypes.c_int32(0), ctypes.c_int32(0), ctypes.c_int32(0)
        L = _lib.lib()
        self._check(L.rfa_ddc_get_mixer(self._h, None, None, 0, ctypes.byref(n), ctypes.byref(mf), ctypes.byref(ci)),
                    "get_mixer")
        c = np.empty(n.value, np.float32)
        s = np.empty(n.value, np.float32)
        self._check(L.rfa_ddc_get_mixer(self._h, c.ctypes.data_as(_lib._fp), s.ctypes.data_as(_lib._fp), c.size,
                                        ctypes.byref(n), ctypes.byref(mf), ctypes.byref(ci)), "get_mixer")
        return c, s, mf.value, ci.value

    def ratio(self):
        """(interpolation, decimation, taps per output) of the filter."""
        i, d, t = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int32()
        self._check(_lib.lib().rfa_ddc_get_ratio(self._h, ctypes.byref(i), ctypes.byref(d), ctypes.byref(t)),
                    "rfa_ddc_get_ratio")
        return i.value, d.value, t.value

    def max_outputs(self, n_samples: int) -> int:
        i, d, _ = self.ratio()
        return n_samples * i // max(d, 1) + 2

    # -- processing
    def process(self, data, frequency: int | None = None, channel_frequency: int | None = None):
        """Host bytes / numpy in -> (re, im) float32 numpy arrays of decimated samples."""
        if frequency is not None:
            self.set_frequencies(frequency, channel_frequency)
        buf = np.ascontiguousarray(np.frombuffer(data, np.uint8) if isinstance(data, (bytes, bytearray, memoryview))
                                   else np.asarray(data).view(np.uint8).reshape(-1))
        n = buf.size // BYTES_PER_SAMPLE[self.fmt]
        cap = self.max_outputs(n)
        re = np.empty(cap, np.float32)
        im = np.empty(cap, np.float32)
        got = ctypes.c_size_t(0)
        self._check(_lib.lib().rfa_ddc_process_host(self._h, buf.ctypes.data, n, re.ctypes.data, im.ctypes.data, cap,
                                                    ctypes.byref(got)), "rfa_ddc_process_host")
        return re[:got.value], im[:got.value]

    def process_device(self, in_ptr: int, n_samples: int, re_ptr: int, im_ptr: int, capacity: int) -> int:
        """Device pointers; asynchronous on the handle's stream; returns the output count."""
        got = ctypes.c_size_t(0)
        self._check(_lib.lib().rfa_ddc_process(self._h, in_ptr, n_samples, re_ptr, im_ptr, capacity,
                                               ctypes.byref(got)), "rfa_ddc_process")
        return got.value

    def set_stream(self, stream_ptr: int | None) -> None:
        """Enqueue on exactly this hipStream_t (None: the handle's own stream)."""
        self._check(_lib.lib().rfa_ddc_set_stream(self._h, stream_ptr or None), "rfa_ddc_set_stream")
        self._stream = stream_ptr or None

    def process_tensor(self, raw, out_re, out_im) -> int:
        """torch.cuda tensors: raw bytes (uint8/int8/int16/float32, contiguous) -> planar float32 outputs.
        Runs on torch's current stream, so it is ordered after the op that produced ``raw``
        and before any later torch op that reads the outputs."""
        import torch

        cur = torch.cuda.current_stream(raw.device).cuda_stream
        if cur != self._stream:
            self.set_stream(cur)
        n = raw.numel() * raw.element_size() // BYTES_PER_SAMPLE[self.fmt]
        if out_re.numel() != out_im.numel():
            raise ValueError("out_re and out_im must have the same length")
        return self.process_device(raw.data_ptr(), n, out_re.data_ptr(), out_im.data_ptr(), out_re.numel())

    def synchronize(self) -> None:
        self._check(_lib.lib().rfa_ddc_synchronize(self._h), "rfa_ddc_synchronize")

    @property
    def stream(self) -> int:
        s = _lib._vp()
        self._check(_lib.lib().rfa_ddc_get_stream(self._h, ctypes.byref(s)), "rfa_ddc_get_stream")
        return s.value or 0


class FirFilter(FrontEnd):
    """dsp/FirFilter.kt on the device: ``FirFilter.createLowPass(decimation, gain, sampleRate,
    cutoff, transition, attenuation)`` (FirFilter.kt:243-263) or explicit taps, then
    ``filter(re, im)`` with the reference's delay line and decimation counter
    (FirFilter.kt:63-110) carried across calls.  Already-mixed float samples in."""

    def __init__(self, taps, decimation: int, sample_rate: int = 1, device: int = 0):
        super().__init__("f32", int(sample_rate), max(1, int(sample_rate) // max(1, int(decimation))), device,
                         _fir=(taps, int(decimation)))

    @classmethod
    def createLowPass(cls, decimation: int, gain: float, sample_rate: float, cutoff_frequency: float,  # noqa: N802
                      transition_width: float, attenuation_db: float, device: int = 0):
        taps = create_low_pass_taps(gain, sample_rate, cutoff_frequency, transition_width, attenuation_db)
        if taps is None:
            return None
        return cls(taps, decimation, max(1, int(sample_rate)), device)

    @property
    def numberOfTaps(self) -> int:  # noqa: N802
        return int(self.taps.size)

    def filter(self, re, im):
        """Planar float32 in -> (re, im) outputs (FirFilter.filter over a whole packet)."""
        re = np.asarray(re, np.float32)
        im = np.asarray(im, np.float32)
        iq = np.empty(2 * re.size, np.float32)
        iq[0::2], iq[1::2] = re, im
        return self.process(iq)
