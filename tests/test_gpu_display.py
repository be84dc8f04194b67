"""GPU: display preprocessing on the device (rfa_draw_preprocess, SURVEY.md §8(f)
row 1) vs the restatement of AnalyzerSurface.drawPreprocessing
(oracle/display.py) on the ring the device holds -- bit-exact: colours, path y,
peak-hold y and autoscale min / max."""
import numpy as np
import pytest

import signals
from oracle import display as od

pytestmark = pytest.mark.gpu

N, R, F0, SR = 2048, 12, 100_000_000, 2_000_000


def _engine(rfa, frames, n=N):
    e = rfa.SpectrumEngine(n, "blackman", "s8", avg="none", peak_hold=True, ring_rows=R)
    e.set_tuning(F0, SR)
    data = signals.frames_bytes(n, frames, "s8", seed=21, tones=((0.13, 0.4), (0.31, 0.02)), noise=0.03)
    e.process(data, frames, rows=False)
    return e


def _both(e, surf=None, tuning=(F0, SR), **kw):
    """One draw on the device and on the restated draw thread (od.Surface: the
    persistent colour buffer and dirty map, AnalyzerSurface.kt:619-640,678-684)."""
    ring, ri, _ = e.ring()
    args = dict(width=333, fft_height=480, viewport_frequency=F0, viewport_sample_rate=SR, min_db=-110.0,
                max_db=-20.0, average_length=3, colormap=od.gqrx_colormap())
    args.update(kw)
    got = e.draw_preprocess(peaks=True, **args)
    surf = surf or od.Surface(ring.shape[0])
    exp = surf.draw(ring, ri, e.peaks(), *tuning, **args)
    return got, exp


def _assert_same(got, exp):
    colors, path, pk, mm = got
    c2, p2, k2, mm2 = exp
    np.testing.assert_array_equal(colors, c2)
    assert np.array_equal(np.isnan(path), np.isnan(p2))
    np.testing.assert_array_equal(path[~np.isnan(path)], p2[~np.isnan(p2)])
    np.testing.assert_array_equal(pk, k2)
    assert mm == mm2


@pytest.mark.parametrize("vf,vsr", [(F0, SR), (F0 + 150_000, SR // 3), (F0, 2 * SR), (F0 - 700_000, SR),
                                    (F0 + 333_333, 5 * SR // 4)])
def test_viewports_bit_exact(rfa, vf, vsr):
    e = _engine(rfa, 20)  # more frames than rows: the ring wrapped
    try:
        _assert_same(*_both(e, viewport_frequency=vf, viewport_sample_rate=vsr))
    finally:
        e.close()


def test_partial_ring_and_no_average(rfa):
    e = _engine(rfa, 5)  # rows 5..11 still hold the -9999 fill
    surf = od.Surface(R)
    try:
        _assert_same(*_both(e, surf, average_length=0, width=1000))  # 6 of 12 rows refreshed
        _assert_same(*_both(e, surf, average_length=R - 1, min_db=-150.0, max_db=0.0))
    finally:
        e.close()


@pytest.mark.parametrize("n", [65536, 131072])
def test_residue_major_ring_bit_exact(rfa, n):
    """At 64 K / 128 K the device ring is stored residue-major (rfa_get_ring_order);
    the draw kernel gathers each pixel's bins in bin order, so the result is still
    bit-identical to the restatement on the natural rows."""
    e = _engine(rfa, 14, n)
    try:
        assert e.ring_order == {65536: 2, 131072: 4}[n]
        _assert_same(*_both(e, width=1111, viewport_frequency=F0 + 150_000, viewport_sample_rate=SR // 3))
    finally:
        e.close()


def test_dirty_rows_across_draws(rfa):
    """The reference refreshes only dirty rows plus the L + 1 averaged ones, at most
    L + 6 rows per draw (AnalyzerSurface.kt:678-684); FftProcessor marks the rows it
    writes (FftProcessor.kt:223) and everything on a resize / retune (:181,193,215,219).
    The device keeps the same colour buffer and dirty map: a sequence of draws
    interleaved with new frames, a retune shift, a clear and a viewport change stays
    bit-identical to the restated draw thread, including the rows still pending."""
    n = 2048
    e = rfa.SpectrumEngine(n, "blackman", "s8", avg="none", peak_hold=True, ring_rows=R)
    e.set_tuning(F0, SR)
    surf = od.Surface(R)
    seed = [30]

    def feed(k):
        seed[0] += 1
        e.process(signals.frames_bytes(n, k, "s8", seed=seed[0], tones=((0.13, 0.4),), noise=0.05), k, rows=False)
        ri = e.ring()[1]
        for j in range(min(k, R)):
            surf.mark_row((ri + j) % R)

    try:
        feed(20)
        for step in range(4):  # R = 12 > L + 6 = 9: the first draws converge over two calls
            _assert_same(*_both(e, surf))
            feed(step + 1)
        _assert_same(*_both(e, surf))
        _assert_same(*_both(e, surf))  # nothing new: only the averaged rows are redrawn
        e.set_tuning(F0 + 10_000, SR)  # shift by a few bins: every row dirty
        surf.mark_all()
        t = (F0 + 10_000, SR)
        _assert_same(*_both(e, surf, t))
        feed(2)
        _assert_same(*_both(e, surf, t, viewport_frequency=F0 + 50_000))  # new viewport: all dirty
        _assert_same(*_both(e, surf, t, viewport_frequency=F0 + 50_000))
        e.set_tuning(F0, 2 * SR)  # sample-rate change clears the ring
        surf.mark_all()
        _assert_same(*_both(e, surf, (F0, 2 * SR), width=500))  # new width: new colour buffer
    finally:
        e.close()


def test_argument_checks(rfa):
    e = _engine(rfa, 3)
    try:
        with pytest.raises(rfa.RfaError):
            e.draw_preprocess(100, 100, F0, SR, -100, 0, R, od.gqrx_colormap())  # average_length >= ring rows
    finally:
        e.close()
