"""CPU: the display-preprocessing restatement (oracle/display.py) on hand-checkable
cases -- AnalyzerSurface.kt:599-743 and ColorMaps.kt:41-51.  The reference has no
tests for these routines, so these pin the restatement by construction (parity
for this row is otherwise unpinned)."""
import numpy as np

from oracle import display as od

N, R, W = 1024, 6, 200


def test_gqrx_colormap_levels():
    m = od.gqrx_colormap()
    assert m.size == 256 and m.dtype == np.uint32
    assert m[0] == m[19] == od.argb(255, 0, 0, 0)            # level 0: black
    assert m[20] == od.argb(255, 0, 0, 0) and m[69] == od.argb(255, 0, 0, 137)
    assert m[100] == od.argb(255, 60, 125, 255)               # level 3 start
    assert m[150] == od.argb(255, 255, 255, 0)                # level 4 start: yellow
    assert m[255] == od.argb(255, 255, 255, 255)              # red -> white end


def _draw(ring, **kw):
    args = dict(read_index=0, peaks=None, frequency=100_000_000, sample_rate=2_000_000, width=W, fft_height=400,
                viewport_frequency=100_000_000, viewport_sample_rate=2_000_000, min_db=-80.0, max_db=0.0,
                average_length=0, colormap=od.gqrx_colormap())
    args.update(kw)
    return od.draw_preprocess(ring, **args)


def test_full_span_constant_rows():
    v = np.float32(-30.0)
    ring = np.full((R, N), v, np.float32)
    colors, path, _, (mn, mx) = _draw(ring)
    # viewport == data span: start 0, end N, lastPixel = W, pixels 1 .. W-2 drawn
    idx = int((v - np.float32(-80.0)) * (np.float32(256) / np.float32(80.0)))
    assert (colors[:, 1:W - 1] == od.gqrx_colormap()[idx]).all()
    assert (colors[:, [0, W - 1]] == od.BLACK).all()
    assert np.isnan(path[[0, W - 1]]).all()
    np.testing.assert_array_equal(path[1:W - 1], np.float32(400) - (v - np.float32(-80.0)) * (np.float32(400) / np.float32(80.0)))
    assert (mn, mx) == (-30.0, -30.0)


def test_zoom_out_black_margins_and_time_average():
    rng = np.random.default_rng(5)
    ring = rng.uniform(-90, -10, (R, N)).astype(np.float32)
    colors, path, peaks_y, _ = _draw(ring, viewport_sample_rate=4_000_000, average_length=2, read_index=3,
                                     peaks=ring.max(0))
    # the data covers the middle half of a 4 MHz viewport: outer quarters black
    assert (colors[:, : W // 4 - 1] == od.BLACK).all() and (colors[:, 3 * W // 4 + 1:] == od.BLACK).all()
    assert (peaks_y[: W // 4 - 1] == -1).all()
    drawn = ~np.isnan(path)
    assert drawn.sum() > W // 2 - 4
    # time average = mean of the newest 3 rows' pixel means (rows 3, 4, 5 of the ring)
    i = W // 2
    # start = ((0 - 4e6/2 + 2e6/2) * (N / 2e6 as float32)).toInt(): float32(N/2e6) is just
    # below 0.000512, so the product truncates to -511, not -512 (Kotlin semantics)
    sph = float(np.float32(N) / np.float32(2_000_000))
    start = int(-1_000_000.0 * sph)
    end = N + int(1_000_000.0 * sph)
    assert start == -511
    spp = np.float32(end - start) / np.float32(W)
    lo, hi = int(np.float32(i) * spp), np.float32(i + 1) * spp
    js = [j for j in range(lo, int(np.ceil(hi)) + 1) if np.float32(j) < hi]
    px = [np.float32(sum(ring[r, j + start] for j in js) / len(js)) for r in (3, 4, 5)]
    ta = np.float32(np.float32(np.float32(px[0] + px[1]) + px[2]) / np.float32(3))
    assert abs(path[i] - (np.float32(400) - (ta + np.float32(80)) * np.float32(5))) < 1e-3


def test_no_valid_pixels_gives_initial_autoscale():
    ring = np.full((R, N), -50, np.float32)
    colors, path, _, mm = _draw(ring, viewport_frequency=100_000_000 + 10_000_000)  # far outside the data
    assert (colors == od.BLACK).all() and np.isnan(path).all()
    assert mm == (10.0, -100.0)


def test_surface_dirty_rows_converge():
    """od.Surface (the reference's dirty-row bookkeeping, AnalyzerSurface.kt:619-640,
    678-684): a first draw of R > L + 6 rows refreshes L + 6 of them, newest first;
    the next draw refreshes the rest; then it equals the full refresh."""
    rng = np.random.default_rng(9)
    R2 = 12
    ring = rng.uniform(-90, -10, (R2, N)).astype(np.float32)
    args = dict(read_index=5, peaks=None, frequency=100_000_000, sample_rate=2_000_000, width=W, fft_height=400,
                viewport_frequency=100_000_000, viewport_sample_rate=2_000_000, min_db=-80.0, max_db=0.0,
                average_length=2, colormap=od.gqrx_colormap())
    surf = od.Surface(R2)
    c1 = surf.draw(ring, **args)[0]
    done = [(5 + j) % R2 for j in range(2 + 6)]
    assert (c1[done] != 0).any(axis=1).all()
    assert (c1[[r for r in range(R2) if r not in done]] == 0).all()
    c2, p2, _, mm2 = surf.draw(ring, **args)
    full = od.draw_preprocess(ring, **args)
    np.testing.assert_array_equal(c2, full[0])
    np.testing.assert_array_equal(p2, full[1])
    assert mm2 == full[3]
    # a row changed without a dirty mark keeps its old colours (the reference's lazy refresh)
    ring2 = ring.copy()
    ring2[(5 + 9) % R2] = -5.0
    np.testing.assert_array_equal(surf.draw(ring2, **args)[0], c2)
    surf.mark_row((5 + 9) % R2)
    np.testing.assert_array_equal(surf.draw(ring2, **args)[0], od.draw_preprocess(ring2, **args)[0])
