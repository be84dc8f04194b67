"""CPU: the Scheduler fan-out (rfanalyzer_amd/scheduler.py, Scheduler.kt:140-298)
with stand-in branches -- squelch gating of the demod branch, framing of the FFT
branch, recording through the real writer."""
import numpy as np

from rfanalyzer_amd import recording, scheduler


class FakeEngine:
    def __init__(self, n, bps):
        self.n, self.bps, self.calls = n, bps, []

    def process(self, data, n_frames, frame_stride=0, rows=True):
        self.calls.append((bytes(data), n_frames, frame_stride))
        return np.zeros((n_frames, self.n), np.float32) if rows else None


class FakeFrontEnd:
    def __init__(self):
        self.packets = []

    def process(self, packet, frequency, channel_frequency):
        self.packets.append((bytes(packet), frequency, channel_frequency))
        return np.zeros(1, np.float32), np.zeros(1, np.float32)


def _packets(k, size=4096):
    rng = np.random.default_rng(3)
    return [rng.integers(0, 256, size, dtype=np.uint8).tobytes() for _ in range(k)]


def test_demod_gated_by_squelch_with_debounce(tmp_path):
    pk = _packets(200)
    fe = FakeFrontEnd()
    rec = recording.RecordingWriter(str(tmp_path), "x.iq", only_when_squelch=True)
    s = scheduler.Scheduler(4096, 2, frequency=100, recorder=rec, frontend=fe, channel_frequency=250)
    expected = []
    for i, p in enumerate(pk):
        s.squelch_satisfied = i < 20 or i >= 150
        s.on_packet(p)
    rec.close()
    # packets 20..68 still pass (debounce 1..49), 69..149 are dropped, 150.. pass again
    expected = [p for i, p in enumerate(pk) if i < 69 or i >= 150]
    assert [q[0] for q in fe.packets] == expected
    assert all(q[1:] == (100, 250) for q in fe.packets)
    assert open(rec.paths[0], "rb").read() == b"".join(expected)   # the recorder applies the same rule


def test_fft_frames_follow_the_packet_framing():
    pk = _packets(70)
    eng = FakeEngine(4096, 2)                       # 2048 samples per packet -> 2 packets per frame
    got_rows = []
    s = scheduler.Scheduler(4096, 2, engine=eng, fft_batch=8, on_rows=got_rows.append)
    for p in pk:
        s.on_packet(p)
    s.flush()
    assert s.frames == 35 and sum(r.shape[0] for r in got_rows) == 35
    stream = b"".join(pk)
    joined = b"".join(c[0] for c in eng.calls)
    assert joined == stream and all(c[2] == 8192 for c in eng.calls)
    eng2 = FakeEngine(1024, 2)                      # N < packet: one frame per packet, rest dropped
    s2 = scheduler.Scheduler(4096, 2, engine=eng2, fft_batch=16)
    for p in pk[:33]:
        s2.on_packet(p)
    s2.flush()
    assert s2.frames == 33 and all(c[2] == 4096 for c in eng2.calls)
