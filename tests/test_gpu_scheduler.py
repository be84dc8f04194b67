"""GPU: the Scheduler fan-out (rfanalyzer_amd/scheduler.py, Scheduler.kt:140-298)
driving the real branches -- FFT rows through SpectrumEngine, the demod front end,
the recorder -- equals each branch run on its own over the same packets."""
import numpy as np
import pytest

import oracle
from oracle import demod as od
from rfanalyzer_amd import demod, recording, scheduler

pytestmark = pytest.mark.gpu

N, PACKET, F0, CH, SR = 4096, 16384, 433_000_000, 433_150_000, 2_400_000


def test_scheduler_branches_match_standalone(rfa, tmp_path):
    rng = np.random.default_rng(21)
    pk = [rng.integers(0, 256, PACKET, dtype=np.uint8).tobytes() for _ in range(150)]
    squelch = [not (40 <= i < 120) for i in range(len(pk))]
    eng = rfa.SpectrumEngine(N, "blackman", "s8", peak_hold=True, ring_rows=64)
    eng.set_tuning(F0, SR)
    fe = demod.FrontEnd("s8", SR, 48_000)
    rec = recording.RecordingWriter(str(tmp_path), "s.iq", only_when_squelch=True)
    rows, dre, dim = [], [], []
    s = scheduler.Scheduler(PACKET, 2, frequency=F0, engine=eng, fft_batch=32, recorder=rec, frontend=fe,
                            channel_frequency=CH, on_rows=rows.append,
                            on_demod=lambda re, im: (dre.append(re), dim.append(im)))
    for p, q in zip(pk, squelch):
        s.squelch_satisfied = q
        s.on_packet(p)
    s.flush()
    rec.close()
    rows = np.concatenate(rows)
    stream = b"".join(pk)
    # FFT branch: one frame per packet (N < packet), the same rows as one batched call and the oracle
    assert rows.shape == (150, N)
    ref_rows = oracle.spectrum_rows(stream, oracle.IN_S8, N, 150, PACKET, oracle.WIN_BLACKMAN)
    import golden_util as gu
    assert gu.db_diff(rows, ref_rows) <= gu.DB_TOL
    with rfa.SpectrumEngine(N, "blackman", "s8", peak_hold=True, ring_rows=64) as e2:
        e2.set_tuning(F0, SR)
        np.testing.assert_array_equal(e2.process(stream, 150, frame_stride=PACKET), rows)
        np.testing.assert_array_equal(e2.peaks(), eng.peaks())
    # demod branch: only packets passing squelch + debounce (i < 89 or i >= 120), bit-exact
    passed = [p for i, p in enumerate(pk) if i < 89 or i >= 120]
    ref = od.FrontEnd(od.IN_S8, SR, 48_000)
    ref.set_frequencies(F0, CH)
    r = [ref.process(p) for p in passed]
    np.testing.assert_array_equal(np.concatenate(dre).view(np.int32), np.concatenate([x[0] for x in r]).view(np.int32))
    np.testing.assert_array_equal(np.concatenate(dim).view(np.int32), np.concatenate([x[1] for x in r]).view(np.int32))
    # recording branch: the same gated packets, byte for byte
    assert open(rec.paths[0], "rb").read() == b"".join(passed)
    eng.close(), fe.close()
