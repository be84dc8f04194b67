"""GPU: waterfall ring, retune shift, peak-hold, boxcar and EMA vs the numpy
restatement of FftProcessor.kt (oracle/processor.py) and the stored sequence."""
import numpy as np
import pytest

import golden_util as gu
import signals
import oracle
from oracle import processor

pytestmark = pytest.mark.gpu

MANIFEST = gu.manifest()


def _gpu_sequence(rfa, spec, data, batch):
    n, nf = spec["n"], spec["n_frames"]
    e = rfa.SpectrumEngine(n, spec["window"], spec["fmt"], avg="ema", avg_length=spec["boxcar_length"],
                           ema_alpha=spec["ema_alpha"], peak_hold=True, ring_rows=spec["ring_rows"])
    f = 0
    while f < nf:
        freq, sr = [t for t in spec["tuning"] if t[0] <= f][-1][1:]
        nxt = min([t[0] for t in spec["tuning"] if t[0] > f] + [nf, f + batch])
        e.set_tuning(freq, sr)
        e.process(data[f * 2 * n:nxt * 2 * n], nxt - f, rows=False)
        f = nxt
    return e


@pytest.mark.parametrize("batch", [1, 7, 40])
def test_state_sequence_vs_reference(rfa, batch):
    spec = MANIFEST["state"]
    data = gu.fixture_input(spec)
    exp = gu.expected(spec)
    e = _gpu_sequence(rfa, spec, data, batch)
    # the stored sequence was built from pffft rows
    assert gu.pffft_diff(e.peaks(), exp["peaks"]) <= gu.DB_TOL
    assert gu.pffft_diff(e.boxcar(spec["boxcar_length"]), exp["boxcar"]) <= gu.DB_TOL
    assert gu.pffft_diff(e.ema(), exp["ema"]) <= gu.DB_TOL
    ring, ri, wi = e.ring()
    newest = np.stack([ring[(ri + r) % ring.shape[0]] for r in range(8)])
    # rows beyond the retune are -9999 fill in both
    for g, x in zip(newest, exp["ring_newest8"]):
        fill = x == -9999
        np.testing.assert_array_equal(g[fill], x[fill])
        if (~fill).any():
            assert gu.pffft_diff(g[~fill], x[~fill]) <= gu.DB_TOL
            assert gu.full_row_diff(g[~fill], x[~fill]) <= gu.DB_TOL  # every bin (s8 input)
    assert gu.full_row_diff(e.peaks(), exp["peaks"]) <= gu.DB_TOL
    e.close()


def test_ring_indices_and_rows_match_processor_restatement(rfa):
    n, rows_r = 256, 5
    data = np.random.default_rng(3).integers(-128, 128, size=2 * n * 13, dtype=np.int8).tobytes()
    ref_rows = oracle.spectrum_rows(data, oracle.IN_S8, n, 13, None, oracle.WIN_BLACKMAN)
    p = processor.FftProcessorRef(n, rows_r, peak_hold=True)
    e = rfa.SpectrumEngine(n, "blackman", "s8", peak_hold=True, ring_rows=rows_r)
    e.set_tuning(100, 1000)
    for chunk in ([0, 3], [3, 4], [4, 13]):  # batches larger than the ring too
        got = e.process(data[chunk[0] * 2 * n:chunk[1] * 2 * n], chunk[1] - chunk[0])
        assert gu.db_diff(got, ref_rows[chunk[0]:chunk[1]]) <= gu.DB_TOL
        for f in range(*chunk):
            p.push(ref_rows[f], 100, 1000)
        ring, ri, wi = e.ring()
        assert (ri, wi) == (p.read_index, p.write_index)
        for r in range(rows_r):
            if np.all(p.ring[r] == -9999):
                assert np.all(ring[r] == -9999)
            else:
                assert gu.db_diff(ring[r], p.ring[r]) <= gu.DB_TOL
    assert gu.db_diff(e.peaks(), p.peaks) <= gu.DB_TOL
    e.close()


@pytest.mark.parametrize("n", [256, 65536, 131072, 1048576])
@pytest.mark.parametrize("new_freq,new_sr", [(100 + 37, 1000), (100 - 300, 1000), (100 + 999, 1000), (100, 2000)])
def test_retune_shift_and_clear(rfa, n, new_freq, new_sr):
    """FftProcessor.kt:197-220 shift / clear; at 64 K and 128 K the device ring is stored
    residue-major (rfa_get_ring_order 2 / 4), at 1 M in the large-N kernel B's column
    order (32 blocks of bins 32 q + s), and the shift runs in that order."""
    rows_r = 4
    data = np.random.default_rng(4).integers(-128, 128, size=2 * n * 3, dtype=np.int8).tobytes()
    ref_rows = oracle.spectrum_rows(data, oracle.IN_S8, n, 3, None, oracle.WIN_BLACKMAN)
    p = processor.FftProcessorRef(n, rows_r, peak_hold=True)
    e = rfa.SpectrumEngine(n, "blackman", "s8", peak_hold=True, ring_rows=rows_r)
    assert e.ring_order == {65536: 2, 131072: 4, 1048576: 32}.get(n, 1)
    e.set_tuning(100, 1000)
    e.process(data[: 2 * 2 * n], 2, rows=False)
    p.push(ref_rows[0], 100, 1000)
    p.push(ref_rows[1], 100, 1000)
    e.set_tuning(new_freq, new_sr)
    e.process(data[2 * 2 * n:], 1, rows=False)
    p.push(ref_rows[2], new_freq, new_sr)
    ring, ri, wi = e.ring()
    assert (ri, wi) == (p.read_index, p.write_index)
    for r in range(rows_r):
        fill = p.ring[r] == -9999
        np.testing.assert_array_equal(ring[r][fill], p.ring[r][fill])
        if (~fill).any():
            assert gu.db_diff(ring[r][~fill], p.ring[r][~fill]) <= gu.DB_TOL
    assert gu.db_diff(e.peaks(), p.peaks) <= gu.DB_TOL  # peaks reset on retune
    e.close()


@pytest.mark.parametrize("n", [65536, 131072, 1048576])
def test_boxcar_over_residue_major_ring(rfa, n):
    """rfa_get_boxcar (AnalyzerSurface.kt:710-714 at bin level) gathers the bins of the
    residue-major ring rows back into natural order."""
    frames, rows_r, L = 6, 5, 3
    data = np.random.default_rng(14).integers(-128, 128, size=2 * n * frames, dtype=np.int8).tobytes()
    ref_rows = oracle.spectrum_rows(data, oracle.IN_S8, n, frames, None, oracle.WIN_BLACKMAN)
    p = processor.FftProcessorRef(n, rows_r)
    with rfa.SpectrumEngine(n, "blackman", "s8", avg="boxcar", avg_length=L, ring_rows=rows_r) as e:
        e.set_tuning(100, 1000)
        e.process(data, frames, rows=False)
        for r in ref_rows:
            p.push(r, 100, 1000)
        assert gu.db_diff(e.boxcar(L), p.boxcar(L)) <= gu.DB_TOL


def test_ema_matches_sequential_extension(rfa):
    n, b = 4096, 50
    data = np.random.default_rng(5).integers(-128, 128, size=2 * n * b, dtype=np.int8).tobytes()
    ref_rows = oracle.spectrum_rows(data, oracle.IN_S8, n, b, None, oracle.WIN_BLACKMAN)
    with rfa.SpectrumEngine(n, "blackman", "s8", avg="ema", ema_alpha=0.2, ring_rows=0) as e:
        e.process(data[: 2 * n * 20], 20, rows=False)
        e.process(data[2 * n * 20:], b - 20, rows=False)
        got = e.ema()
    assert gu.db_diff(got, processor.ema_batch(ref_rows, 0.2)) <= gu.DB_TOL


@pytest.mark.parametrize("batches", [(100,), (13, 87), (1, 2, 97)])
def test_chunked_state_with_silent_frames(rfa, batches):
    """Large batches take the chunked peak/EMA update; all-zero frames give
    -inf rows, which restart the EMA (extension semantics, oracle/processor.py)."""
    n, total = 2048, sum(batches)
    raw = np.random.default_rng(11).integers(-128, 128, size=(total, 2 * n), dtype=np.int8)
    raw[[0, 30, 31, 32, 77, total - 1]] = 0
    data = raw.tobytes()
    ref_rows = oracle.spectrum_rows(data, oracle.IN_S8, n, total, None, oracle.WIN_BLACKMAN)
    with rfa.SpectrumEngine(n, "blackman", "s8", avg="ema", ema_alpha=0.3, peak_hold=True, ring_rows=0) as e:
        f = 0
        for b in batches:
            e.process(data[f * 2 * n:(f + b) * 2 * n], b, rows=False)
            f += b
        ema, peaks = e.ema(), e.peaks()
    exp = processor.ema_batch(ref_rows, 0.3)
    assert np.all(np.isneginf(exp)) and np.all(np.isneginf(ema))  # the last frame is silent
    ema_before = processor.ema_batch(ref_rows[:-1], 0.3)
    assert gu.db_diff(peaks, ref_rows.max(0)) <= gu.DB_TOL
    with rfa.SpectrumEngine(n, "blackman", "s8", avg="ema", ema_alpha=0.3, ring_rows=0) as e:
        e.process(data[: (total - 1) * 2 * n], total - 1, rows=False)
        assert gu.db_diff(e.ema(), ema_before) <= gu.DB_TOL


# channel mean vs the reference's sequential fp32 loop over the same rows: the device
# folds the bins in a tree; for means around -40 dB over <= 5000 bins the two rounding
# orders differ by ~1e-5 dB (fp32 ulp of the running sum x sqrt(bins))
CHAN_SUM_TOL = 2e-4


@pytest.mark.parametrize("n,freq,sr,chan", [(4096, 100_000_000, 2_000_000, (100_010_000, 100_060_000)),
                                            (65536, 433_920_000, 20_000_000, (433_000_000, 434_500_000)),
                                            (1048576, 433_920_000, 250_000_000, (400_000_000, 401_000_000)),
                                            (1024, 100_000_000, 2_000_000, (98_000_000, 99_500_000)),  # below: empty
                                            (1024, 100_000_000, 2_000_000, (99_100_000, 103_000_000))])  # clamped
def test_channel_mean_per_frame(rfa, n, freq, sr, chan):
    """FftProcessor.kt:143-157 squelch input: mean dB of the channel bins, every frame."""
    frames = 12
    data = signals.frames_bytes(n, frames, "s8", 17, tones=((0.01, 0.3), (-0.2, 0.05)), noise=0.05)
    ref_rows = oracle.spectrum_rows(data, oracle.IN_S8, n, frames, None, oracle.WIN_BLACKMAN)
    exp = [processor.channel_mean(r, n, freq, sr, *chan) for r in ref_rows]
    # 64 K: the batch fits the ring, so the means read the residue-major ring rows;
    # the other sizes read the caller rows (batch larger than the ring)
    with rfa.SpectrumEngine(n, "blackman", "s8", ring_rows=12 if n == 65536 else 8) as e:
        e.set_tuning(freq, sr)
        e.set_channel(*chan)
        if n == 65536:
            e.process(data, frames, rows=False)
            ring, _, _ = e.ring()
            gpu_rows = ring[[(-g) % 12 for g in range(frames)]]
        else:
            gpu_rows = e.process(data, frames)
        got = e.channel_means()
    if exp[0] is None:
        assert got.size == 0
        return
    assert got.size == frames
    np.testing.assert_allclose(got, np.array(exp, np.float32), rtol=0, atol=gu.DB_TOL)
    # the reference's own loop (sequential fp32 sum, :150-152) over the rows the GPU
    # produced: the device sums the same bins in a fixed tree order, so the two agree
    # to fp32 rounding of the sum (CHAN_SUM_TOL), far below the FFT tolerance
    same = [processor.channel_mean(r, n, freq, sr, *chan) for r in gpu_rows]
    np.testing.assert_allclose(got, np.array(same, np.float32), rtol=0, atol=CHAN_SUM_TOL)


def test_channel_mean_many_frames_wide_channel(rfa):
    """channel_mean_kernel on 130 frames and a 1001-bin channel (four strided loads
    per thread, a tail, the tree fold) read from the ring in store-tile order: equal to
    the reference's sequential loop over the GPU's own rows to fp32 rounding of the
    sum, and bit-identical between two runs."""
    n, frames, freq, sr = 32768, 130, 100_000_000, 32_768_000  # 1000 Hz per bin
    chan = (freq - 500_500, freq + 500_500)
    data = signals.frames_bytes(n, frames, "s8", 23, tones=((0.01, 0.3), (-0.2, 0.05)), noise=0.05)
    with rfa.SpectrumEngine(n, "blackman", "s8", ring_rows=frames) as e:
        e.set_tuning(freq, sr)
        e.set_channel(*chan)
        e.process(data, frames, rows=False)
        ring, _, _ = e.ring()
        gpu_rows = ring[[(-g) % frames for g in range(frames)]]
        got = e.channel_means()
    same = [processor.channel_mean(r, n, freq, sr, *chan) for r in gpu_rows]
    assert got.size == frames
    np.testing.assert_allclose(got, np.array(same, np.float32), rtol=0, atol=CHAN_SUM_TOL)
    # deterministic: the same batch again gives the same means bit for bit
    with rfa.SpectrumEngine(n, "blackman", "s8", ring_rows=frames) as e:
        e.set_tuning(freq, sr)
        e.set_channel(*chan)
        e.process(data, frames, rows=False)
        np.testing.assert_array_equal(e.channel_means(), got)


def test_channel_mean_spans_wide_channel(rfa):
    """Channels wider than 16384 bins are summed by several workgroups per frame and
    folded in span order (channel_mean_spans): 40001 bins at 64 K -> three spans.  The
    sequential fp32 loop's own rounding grows with the bin count, so the comparison is
    relative (3e-5 of the mean) here; still deterministic bit for bit."""
    n, frames, freq, sr = 65536, 20, 100_000_000, 65_536_000
    chan = (freq - 20_000_500, freq + 20_000_500)
    data = signals.frames_bytes(n, frames, "u8", 29, tones=((0.05, 0.3),), noise=0.05)
    outs = []
    for _ in range(2):
        with rfa.SpectrumEngine(n, "blackman", "u8", ring_rows=frames) as e:
            e.set_tuning(freq, sr)
            e.set_channel(*chan)
            e.process(data, frames, rows=False)
            ring, _, _ = e.ring()
            gpu_rows = ring[[(-g) % frames for g in range(frames)]]
            outs.append(e.channel_means())
    same = np.array([processor.channel_mean(r, n, freq, sr, *chan) for r in gpu_rows], np.float32)
    np.testing.assert_allclose(outs[0], same, rtol=3e-5, atol=0)
    np.testing.assert_array_equal(outs[0], outs[1])


# ---------------------------------------------------------------- config 3 at its real size
# BASELINE config 3: N = 65536, EMA + peak-hold, one stream, B frames per launch,
# ring of 500 rows (waterfall SLOW, FftProcessor.kt:103).  The batch sizes pick
# every state-kernel form launch_state() has at this N (fft_kernels.hip):
#   B >= 121 -> state_fused_kernel<16>,  64 <= B < 121 -> <8>,
#   8 < B < 64 -> partial + combine kernels,  B <= 8 -> the one-thread-per-bin kernel,
# and whether the rows are read back from the ring (B <= ring rows) or from the
# staging buffer (B > ring rows).  The prefix makes the ring wrap, so the
# ring-resident read starts at write_index != 0.  N = 32768 reaches <32>.
# Model: FftProcessor.kt:222-245 (ring write, reverse order, peak-hold), EMA
# extension (oracle/processor.py ema_batch).

_CFG3 = {}


def _cfg3_rows(n, total, seed):
    key = (n, total, seed)
    if key not in _CFG3:
        data = signals.frames_bytes(n, total, "s8", seed, tones=((0.1, 0.4), (-0.27, 0.02)), noise=0.05,
                                    drift=0.002)
        rows = oracle.spectrum_rows(data, oracle.IN_S8, n, total, None, oracle.WIN_BLACKMAN)
        _CFG3.clear()
        _CFG3[key] = (data, rows)
    return _CFG3[key]


@pytest.mark.parametrize("n,ring_rows,batches", [
    (65536, 500, (137, 100, 400)),  # <16> (ring read), <8>, <16> after the wrap
    (65536, 500, (1, 40, 596)),     # serial, partial+combine, <16> from the staging rows (B > ring)
    (32768, 300, (300, 45)),        # <32> (ring read), partial+combine
])
def test_config3_state_at_size(rfa, n, ring_rows, batches):
    total = sum(batches)
    data, rows = _cfg3_rows(n, total, 3)
    fb = 2 * n
    alpha = 0.1
    with rfa.SpectrumEngine(n, "blackman", "s8", avg="ema", ema_alpha=alpha, peak_hold=True,
                            ring_rows=ring_rows) as e:
        e.set_tuning(433_920_000, 20_000_000)
        f = 0
        for b in batches:
            e.process(data[f * fb:(f + b) * fb], b, rows=False)
            f += b
            assert gu.db_diff(e.peaks(), rows[:f].max(0)) <= gu.DB_TOL, (b, f)
            assert gu.db_diff(e.ema(), processor.ema_batch(rows[:f], alpha)) <= gu.DB_TOL, (b, f)
            ring, ri, wi = e.ring()
            # frame g (0-based, in arrival order) sits at ring row (-g) mod R (writeIndex-- order)
            assert ri == (-(f - 1)) % ring_rows and wi == (-f) % ring_rows
            live = range(max(0, f - ring_rows), f)
            picks = sorted(set(list(live)[:4] + list(live)[-8:] + list(live)[::97]))
            assert gu.db_diff(ring[[(-g) % ring_rows for g in picks]], rows[picks]) <= gu.DB_TOL
            if f < ring_rows:
                assert np.all(ring[[(-g) % ring_rows for g in range(f, ring_rows)]] == -9999)


def test_state_over_a_ring_beyond_2_gib(rfa):
    """state_fused_kernel walks a ring under 2 GiB by 32-bit buffer offsets and a larger one by
    flat addresses (fft_kernels.hip, RFA_STATE_BUF).  At N = 64 K a 8200-row ring is 2.15 GB:
    the same frames through it and through a 500-row ring give bit-identical peaks and EMA
    (same chunking, same arithmetic, only the addressing differs), and both match the
    oracle."""
    n, batches, alpha = 65536, (137, 300), 0.1
    total = sum(batches)
    data, rows = _cfg3_rows(n, total, 3)
    fb = 2 * n
    out = []
    for ring_rows in (500, 8200):
        with rfa.SpectrumEngine(n, "blackman", "s8", avg="ema", ema_alpha=alpha, peak_hold=True,
                                ring_rows=ring_rows) as e:
            e.set_tuning(433_920_000, 20_000_000)
            f = 0
            for b in batches:
                e.process(data[f * fb:(f + b) * fb], b, rows=False)
                f += b
            out.append((e.peaks(), e.ema()))
    np.testing.assert_array_equal(out[0][0], out[1][0])
    np.testing.assert_array_equal(out[0][1], out[1][1])
    assert gu.db_diff(out[1][0], rows[:total].max(0)) <= gu.DB_TOL
    assert gu.db_diff(out[1][1], processor.ema_batch(rows[:total], alpha)) <= gu.DB_TOL


@pytest.mark.parametrize("n,batches", [(262144, (3, 9, 2)), (524288, (5, 6)), (1048576, (1, 7, 4))])
def test_column_order_ring_state_tiles(rfa, n, batches):
    """N >= 256 K keeps the ring in column order (RS = N / 32 K blocks); the peak / EMA
    update reads it through state_tile_kernel (fft_kernels.hip), whose tiles move the
    natural-order peaks / EMA through LDS.  Ring of 8 rows, so the batches wrap it."""
    total, ring_rows, alpha = sum(batches), 8, 0.3
    data, rows = _cfg3_rows(n, total, 21)
    fb = 2 * n
    with rfa.SpectrumEngine(n, "blackman", "s8", avg="ema", ema_alpha=alpha, peak_hold=True,
                            ring_rows=ring_rows) as e:
        assert e.ring_order == n // 32768
        e.set_tuning(433_920_000, 250_000_000)
        f = 0
        for b in batches:
            e.process(data[f * fb:(f + b) * fb], b, rows=False)
            f += b
            assert gu.db_diff(e.peaks(), rows[:f].max(0)) <= gu.DB_TOL, (b, f)
            assert gu.db_diff(e.ema(), processor.ema_batch(rows[:f], alpha)) <= gu.DB_TOL, (b, f)


# ---------------------------------------------------------------- waterfall speed / FFT size change
@pytest.mark.parametrize("sizes", [(5, 8), (8, 3), (5, 5, 2, 7)])
def test_ring_resize_keeps_history(rfa, sizes):
    """FftProcessor.kt:185-195: a speed change rebuilds the ring with the next frame,
    new row i = old row (writeIndex + i) % old_rows, -9999 beyond, writeIndex = 0."""
    n = 512
    total = 6 * len(sizes) + 3
    data = np.random.default_rng(8).integers(-128, 128, size=2 * n * total, dtype=np.int8).tobytes()
    ref_rows = oracle.spectrum_rows(data, oracle.IN_S8, n, total, None, oracle.WIN_BLACKMAN)
    p = processor.FftProcessorRef(n, sizes[0], peak_hold=True)
    with rfa.SpectrumEngine(n, "blackman", "s8", peak_hold=True, ring_rows=sizes[0]) as e:
        e.set_tuning(100, 1000)
        f = 0
        for k, r in enumerate(sizes):
            if k:
                e.set_ring_rows(r)
                p.set_waterfall_rows(r)
                ring_before, ri_b, _ = e.ring()  # still the old ring until a frame arrives
                assert ring_before.shape[0] == sizes[k - 1] and ri_b == p.read_index
            b = 6 if k < len(sizes) - 1 else 9
            e.process(data[f * 2 * n:(f + b) * 2 * n], b, rows=False)
            for g in range(f, f + b):
                p.push(ref_rows[g], 100, 1000)
            f += b
            ring, ri, wi = e.ring()
            assert ring.shape == p.ring.shape and (ri, wi) == (p.read_index, p.write_index)
            for row_g, row_p in zip(ring, p.ring):
                fill = row_p == -9999
                np.testing.assert_array_equal(row_g[fill], row_p[fill])
                if (~fill).any():
                    assert gu.db_diff(row_g[~fill], row_p[~fill]) <= gu.DB_TOL
        assert gu.db_diff(e.peaks(), p.peaks) <= gu.DB_TOL


@pytest.mark.parametrize("na,nb", [(1024, 2048), (65536, 1048576), (1048576, 4096)])
def test_fft_size_change_restarts_ring_and_peaks(rfa, na, nb):
    """FftProcessor.kt:178-183 (new size -> fresh -9999 ring, writeIndex 0) and :233-236
    (peaks re-initialised), also across the large-N pair (its scratch, tables and ring order)."""
    data = np.random.default_rng(9).integers(-128, 128, size=2 * (3 * na + 2 * nb), dtype=np.int8).tobytes()
    rows_a = oracle.spectrum_rows(data, oracle.IN_S8, na, 3, None, oracle.WIN_BLACKMAN)
    rows_b = oracle.spectrum_rows(data[3 * 2 * na:], oracle.IN_S8, nb, 2, None, oracle.WIN_BLACKMAN)
    p = processor.FftProcessorRef(na, 4, peak_hold=True, ema_alpha=0.25)
    with rfa.SpectrumEngine(na, "blackman", "s8", avg="ema", ema_alpha=0.25, peak_hold=True, ring_rows=4) as e:
        e.set_tuning(100_000_000, 2_000_000)
        e.process(data[: 3 * 2 * na], 3, rows=False)
        for r in rows_a:
            p.push(r, 100_000_000, 2_000_000)
        e.set_fft_size(nb)
        assert e.n == nb
        e.process(data[3 * 2 * na:3 * 2 * na + 2 * 2 * nb], 2, rows=False)
        for r in rows_b:
            p.push(r, 100_000_000, 2_000_000)
        ring, ri, wi = e.ring()
        assert ring.shape == (4, nb) and (ri, wi) == (p.read_index, p.write_index)
        for row_g, row_p in zip(ring, p.ring):
            if np.all(row_p == -9999):
                assert np.all(row_g == -9999)
            else:
                assert gu.db_diff(row_g, row_p) <= gu.DB_TOL
        assert gu.db_diff(e.peaks(), p.peaks) <= gu.DB_TOL
        assert gu.db_diff(e.ema(), p.ema) <= gu.DB_TOL
        assert gu.db_diff(e.ema(), processor.ema_batch(rows_b, 0.25)) <= gu.DB_TOL


def test_state_generation_tracks_device_pointers(rfa):
    """rfa_get_device_state pointers are valid while rfa_get_state_generation is
    unchanged: a shifting retune swaps the ring buffer, a resize and an FFT-size change
    reallocate; an unchanged tuning or a plain batch keeps them."""
    import ctypes
    n = 1024
    data = np.random.default_rng(2).integers(-128, 128, size=2 * n * 4, dtype=np.int8).tobytes()
    with rfa.SpectrumEngine(n, "blackman", "s8", peak_hold=True, ring_rows=4) as e:
        lib = rfa.lib()

        def ptrs():
            r, p, m = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_void_p()
            assert lib.rfa_get_device_state(e.handle, ctypes.byref(r), ctypes.byref(p), ctypes.byref(m)) == 0
            return r.value, p.value
        e.set_tuning(100_000_000, 2_000_000)
        e.process(data, 2, rows=False)
        g0, p0 = e.state_generation(), ptrs()
        e.set_tuning(100_000_000, 2_000_000)
        e.process(data, 2, rows=False)
        assert (e.state_generation(), ptrs()) == (g0, p0)
        e.set_tuning(100_001_000, 2_000_000)  # shift: the ring moves to the other buffer
        g1 = e.state_generation()
        assert g1 > g0 and ptrs()[0] != p0[0]
        e.set_ring_rows(6)
        e.process(data, 1, rows=False)         # the resize is applied with the next frame
        g2 = e.state_generation()
        assert g2 > g1
        e.set_fft_size(2048)
        assert e.state_generation() > g2


@pytest.mark.parametrize("packed", [True, False])
def test_process_batches_equals_consecutive_calls(rfa, packed):
    """rfa_process_batches (config 4's multi-batch enqueue) is exactly n_batches
    consecutive rfa_process calls: rows bit-identical, same ring, peaks and EMA;
    packed batches take one launch, strided ones one per batch."""
    import torch
    n, fpb, nb = 8192, 12, 5
    gap = 0 if packed else 3 * 2 * n  # strided: 3 unused frames between batches
    stride_b = fpb * 2 * n + gap
    raw = np.random.default_rng(31).integers(-128, 128, size=nb * stride_b, dtype=np.int8)
    dev = torch.from_numpy(raw.view(np.uint8).copy()).cuda()
    kw = dict(avg="ema", ema_alpha=0.2, peak_hold=True, ring_rows=40)
    with rfa.SpectrumEngine(n, "blackman", "s8", **kw) as a, rfa.SpectrumEngine(n, "blackman", "s8", **kw) as b:
        for e in (a, b):
            e.set_tuning(100_000_000, 2_000_000)
            e.set_channel(99_900_000, 100_300_000)  # a squelch channel: its per-frame means
        rows_a = torch.empty((nb * fpb, n), dtype=torch.float32, device="cuda")
        a.process_batches(dev.data_ptr(), nb, stride_b, fpb, 0, rows_a.data_ptr())
        a.synchronize()
        rows_b = []
        for k in range(nb):
            rows_b.append(b.process(raw[k * stride_b:k * stride_b + fpb * 2 * n].tobytes(), fpb))
        np.testing.assert_array_equal(rows_a.cpu().numpy(), np.concatenate(rows_b))
        ra, ria, wia = a.ring()
        rb, rib, wib = b.ring()
        assert (ria, wia) == (rib, wib)
        np.testing.assert_array_equal(ra, rb)
        np.testing.assert_array_equal(a.peaks(), b.peaks())
        # the EMA recursion is re-associated by the chunked scan (one batch of 60 frames
        # vs five of 12): equal to fp32 rounding, not bit for bit
        np.testing.assert_allclose(a.ema(), b.ema(), rtol=0, atol=2e-4)
        # channel means: the last batch's fpb frames in either form
        ca, cb = a.channel_means(), b.channel_means()
        assert ca.shape == (fpb,) and cb.shape == (fpb,)
        np.testing.assert_array_equal(ca, cb)


@pytest.mark.parametrize("n", [1024, 32768, 65536, 131072, 1048576])
def test_ring_positions_map_device_rows(rfa, n):
    """rfa_get_ring_positions (zero-copy consumers): the raw device ring row gathered
    at the reported positions is the natural row rfa_get_ring returns -- including the
    32 K kernel's store-tile order at N = 32 K .. 128 K."""
    import ctypes
    data = np.random.default_rng(n).integers(-128, 128, size=2 * n * 3, dtype=np.int8).tobytes()
    with rfa.SpectrumEngine(n, "blackman", "s8", ring_rows=3) as e:
        e.set_tuning(100_000_000, 2_000_000)
        e.process(data, 3, rows=False)
        pos = e.ring_positions()
        assert np.array_equal(np.sort(pos), np.arange(n))  # a permutation
        ring, ri, _ = e.ring()
        r, p, m = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_void_p()
        assert rfa.lib().rfa_get_device_state(e.handle, ctypes.byref(r), ctypes.byref(p), ctypes.byref(m)) == 0
        raw = np.empty((3, n), np.float32)
        hip = ctypes.CDLL("libamdhip64.so")
        e.synchronize()
        assert hip.hipMemcpy(ctypes.c_void_p(raw.ctypes.data), r, ctypes.c_size_t(raw.nbytes), 2) == 0
        np.testing.assert_array_equal(raw[:, pos], ring)


# ---------------------------------------------------------------- pipelined state (rfa_set_pipelined)
def _pipe_pair(rfa, n, ring_rows, state_cus, chan=None, **kw):
    kw = dict(avg="ema", ema_alpha=0.1, peak_hold=True, ring_rows=ring_rows, **kw)
    a, b = rfa.SpectrumEngine(n, "blackman", "s8", **kw), rfa.SpectrumEngine(n, "blackman", "s8", **kw)
    for e in (a, b):
        e.set_tuning(433_920_000, 20_000_000)
        if chan:
            e.set_channel(*chan)
    b.set_pipelined(state_cus)
    return a, b


def _same_state(a, b, n_frames_last):
    """Serial engine a and pipelined engine b hold bit-identical ring, peaks, EMA and channel
    means (the same kernels on the same rows; only the streams and CU sets differ)."""
    ra, ria, wia = a.ring()
    rb, rib, wib = b.ring()
    assert (ria, wia) == (rib, wib)
    np.testing.assert_array_equal(ra, rb)
    np.testing.assert_array_equal(a.peaks(), b.peaks())
    np.testing.assert_array_equal(a.ema(), b.ema())
    np.testing.assert_array_equal(a.channel_means(), b.channel_means())


@pytest.mark.parametrize("n,ring_rows,batches", [
    (65536, 500, (500, 500, 500, 500)),    # B = R: every call writes the other ring buffer
    (65536, 500, (200, 250, 100, 40, 60)),  # B_k + B_k-1 <= R: rows the last call did not write
    (65536, 500, (300, 300, 500, 137, 500)),  # neither: joins, then flips again
    (8192, 64, (64, 64, 30, 30, 64, 1)),
    (1048576, 32, (16, 16, 8, 16)),         # column-order ring, state_tile_kernel on the state stream
])
def test_pipelined_state_equals_serial(rfa, n, ring_rows, batches):
    """rfa_set_pipelined (the peak / EMA pass of call k on reserved CUs under call k + 1's FFT,
    DESIGN.md §5.3c): the same batches through a serial engine and a pipelined one give
    bit-identical rings, peaks, EMA and channel means, read after the last call (the getters
    join), and both match the oracle.  Device-resident input, several calls in flight."""
    import torch
    total = sum(batches)
    data, rows = _cfg3_rows(n, total, 5)
    dev = torch.from_numpy(np.frombuffer(data, np.uint8).copy()).cuda()
    torch.cuda.synchronize()
    fb = 2 * n
    a, b = _pipe_pair(rfa, n, ring_rows, 16, chan=(433_900_000, 433_990_000))
    with a, b:
        f = 0
        g0 = b.state_generation()
        for k, nb in enumerate(batches):
            for e in (a, b):
                e.process_device(dev.data_ptr() + f * fb, nb, 0, None)
            f += nb
        _same_state(a, b, batches[-1])
        if all(x == ring_rows for x in batches):
            assert b.state_generation() == g0 + len(batches)  # one ring swap per call
        assert gu.db_diff(b.peaks(), rows[:total].max(0)) <= gu.DB_TOL
        assert gu.db_diff(b.ema(), processor.ema_batch(rows[:total], 0.1)) <= gu.DB_TOL


def test_pipelined_state_with_retune_resize_and_reads_between_calls(rfa):
    """Every other entry point joins the pipeline first: a shifting retune, a ring resize, a
    mid-stream peaks / ring read and rfa_get_device_state between pipelined calls leave the
    pipelined engine bit-identical to the serial one."""
    import ctypes
    import torch
    n, R = 65536, 100
    data, rows = _cfg3_rows(n, 520, 7)
    dev = torch.from_numpy(np.frombuffer(data, np.uint8).copy()).cuda()
    torch.cuda.synchronize()
    fb = 2 * n
    a, b = _pipe_pair(rfa, n, R, 24)
    with a, b:
        f = 0
        for k, nb in enumerate((100, 100, 40, 50, 100, 30, 100)):
            for e in (a, b):
                if k == 2:
                    e.set_tuning(433_920_000 + 150_000, 20_000_000)  # shift by 491 bins
                if k == 4:
                    e.set_ring_rows(120)
                e.process_device(dev.data_ptr() + f * fb, nb, 0, None)
            f += nb
            if k in (1, 3):
                np.testing.assert_array_equal(a.peaks(), b.peaks())
            if k == 5:
                r, p, m = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_void_p()
                assert rfa.lib().rfa_get_device_state(b.handle, ctypes.byref(r), ctypes.byref(p), ctypes.byref(m)) == 0
                got = np.empty(n, np.float32)
                hip = ctypes.CDLL("libamdhip64.so")
                b.synchronize()
                assert hip.hipMemcpy(ctypes.c_void_p(got.ctypes.data), m, ctypes.c_size_t(got.nbytes), 2) == 0
                np.testing.assert_array_equal(got, a.ema())
        _same_state(a, b, 100)


def test_pipelined_state_arguments(rfa):
    """state_cus must be a multiple of the XCD count and leave CUs for the FFT; 0 turns the
    mode off (host getters keep working in either mode)."""
    import torch
    props = torch.cuda.get_device_properties(0)
    with rfa.SpectrumEngine(1024, "blackman", "s8", peak_hold=True, ring_rows=8) as e:
        for bad in (3, props.multi_processor_count):
            with pytest.raises(RuntimeError):
                e.set_pipelined(bad)
        e.set_pipelined(8)
        e.set_pipelined(0)
        e.set_tuning(1_000_000, 100_000)
        e.process(np.zeros(2 * 1024 * 8, np.int8).tobytes(), 8, rows=False)
        assert np.all(np.isneginf(e.peaks()) | (e.peaks() < -100))
