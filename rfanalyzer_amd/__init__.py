"""rfanalyzer_amd -- MI355X-native drop-in for RFAnalyzer's spectrum hot path.

Raw IQ bytes -> convert -> window -> FFT -> 10*log10(|X|/N) + fft-shift ->
waterfall ring / peak-hold / averaging, as hand-written gfx950 HIP kernels
behind the C-ABI in include/rfa.h (librfa.so).  The Python modules mirror the
reference's interfaces for this path:

    nativedsp.NativeDsp        nativedsp/.../NativeDsp.kt
    processor.FftProcessor     analyzer/FftProcessor.kt
    source.FileIQSource        source/FileIQSource.java (+ Scheduler framing)
    engine.SpectrumEngine      one librfa handle
    engine.SeamPlan            the legacy seams at pffft-only lengths (mixed 2/3/5, 16, 32, > 2^20)
    SpectrumEngine.draw_preprocess, scanner   AnalyzerSurface.drawPreprocessing, MainViewModel scanner
    recording                  Scheduler recording branch, file names, replay metadata
    demod.FrontEnd             IQConverter.mixPacketIntoSamplePacket + Decimator / Resampler
    scheduler.Scheduler        analyzer/Scheduler.kt packet fan-out

There is no CPU fallback: without librfa.so or a HIP device, calls raise.
"""
from ._lib import RfaError, build, device_count, lib  # noqa: F401
from .engine import SeamPlan, SpectrumEngine  # noqa: F401

__all__ = ["SpectrumEngine", "SeamPlan", "RfaError", "build", "device_count", "lib"]
