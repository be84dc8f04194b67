"""CPU: recording format, file names, replay metadata (rfanalyzer_amd/recording.py;
RecordingDao.kt:87-90, HelperComposables.kt:168-179, MainViewModel.kt:1815-1846,
2034-2078, Scheduler.kt:52-53,161-234) and a record -> replay round trip through
the packet framing (checked with the oracle restatement)."""
import datetime as dt

import numpy as np

import oracle
import signals
from rfanalyzer_amd import recording as rec
from rfanalyzer_amd import source


def test_as_string_with_unit():
    assert rec.as_string_with_unit(100_000_000, "Hz") == "100 MHz"
    assert rec.as_string_with_unit(2_400_000_000, "Hz") == "2 400 MHz"   # 2.4 GHz is not exact in G
    assert rec.as_string_with_unit(6_000_000, "Sps") == "6 MSps"
    assert rec.as_string_with_unit(1_234_567, "Sps") == "1 234 567 Sps"
    assert rec.as_string_with_unit(3 * 10 ** 15, "Hz") == "3 000 THz"


def test_file_name_matches_documented_example_and_parses_back():
    ms = int(dt.datetime(2025, 1, 11, 14, 30, 22).timestamp() * 1000)
    name = rec.recording_file_name("MyRecording", "AIRSPY", 100_000_000, 6_000_000, ms)
    assert name == "20250111-143022_MyRecording_AIRSPY_100MHz_6MSps.iq"  # IQ_FILE_FORMAT.md:100
    meta = rec.parse_file_name(name)
    assert (meta.file_format, meta.sample_rate, meta.frequency) == ("AIRSPY", 6_000_000, 100_000_000)
    assert rec.recording_file_name("x", "HACKRF", 1, 2, ms, split_index=3).endswith("_1Hz_2Sps-003.iq")


def test_parse_literal_reference_rules():
    # only the listed spellings count ("kSps" and "kHz" are not among them), later rules
    # win, the last occurrence of a pattern is taken, GHz is never parsed
    m = rec.parse_file_name("rtl-sdr_capture_2400kSps_433920kHz.iq")
    assert (m.file_format, m.sample_rate, m.frequency) == ("RTLSDR", None, None)
    m = rec.parse_file_name("rtl-sdr_capture_2400KSps_433920KHz.iq")
    assert (m.file_format, m.sample_rate, m.frequency) == ("RTLSDR", 2_400_000, 433_920_000)
    m = rec.parse_file_name("hackrf airspy-10MSPS_7000Khz_2400MHz.iq")
    assert (m.file_format, m.sample_rate, m.frequency) == ("AIRSPY", 10_000_000, 2_400_000_000)
    assert rec.parse_file_name("x_3GHz_1Msps.iq").frequency is None


def test_writer_split_and_squelch(tmp_path):
    pkt = bytes(range(256)) * 2  # 512 bytes
    with rec.RecordingWriter(str(tmp_path), "a.iq", split_size=1500) as w:
        for _ in range(7):
            w.write_packet(pkt)
    sizes = [p.stat().st_size for p in sorted(tmp_path.iterdir())]
    assert [p.name for p in sorted(tmp_path.iterdir())] == ["a-001.iq", "a-002.iq", "a-003.iq", "a-004.iq"]
    assert sizes == [1024, 1024, 1024, 512] and w.recorded_size == 7 * 512
    d2 = tmp_path / "single"
    d2.mkdir()
    with rec.RecordingWriter(str(d2), "b.iq", only_when_squelch=True) as w:
        w.write_packet(pkt, squelch_satisfied=False)           # counter 0 -> 1: still written (debounce)
        for _ in range(60):
            w.write_packet(pkt, squelch_satisfied=False)       # after 50 packets writing stops
        w.write_packet(pkt, squelch_satisfied=True)
    assert [p.name for p in d2.iterdir()] == ["b.iq"]
    assert (d2 / "b.iq").stat().st_size == (49 + 1) * 512


def test_record_then_replay_frames(tmp_path):
    n, packet = 1024, 8192
    raw = signals.frames_bytes(packet // 2, 12, "s8", seed=9)   # a 2-byte-per-sample s8 stream
    name = rec.recording_file_name("t", "HACKRF", 100_000_000, 2_000_000, 0)
    with rec.RecordingWriter(str(tmp_path), name) as w:
        for k in range(0, len(raw), packet):
            w.write_packet(raw[k:k + packet])
    meta = rec.parse_file_name(name)
    src = source.FileIQSource()
    src.init(w.paths[0], meta.sample_rate, meta.frequency, packet_size=packet, file_format=source.FILE_FORMAT_8BIT_SIGNED)
    assert src.open()
    got = b"".join(iter(lambda: src.getPacket(), None))
    assert got == raw  # the recording is the raw packet stream, byte for byte
    stride = source.frame_stride(n, packet, 2)
    frames = source.file_frames(len(got), n, packet, 2)
    rows = oracle.spectrum_rows(got, oracle.IN_S8, n, frames, stride, oracle.WIN_BLACKMAN)
    ref = np.stack([oracle.spectrum_rows(raw[f * stride:f * stride + 2 * n], oracle.IN_S8, n, 1, None,
                                         oracle.WIN_BLACKMAN)[0] for f in range(frames)])
    np.testing.assert_array_equal(rows, ref)
