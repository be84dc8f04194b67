"""IQ recordings: on-disk format, file names and replay metadata.

Host-side mirror of the reference's recording path (paths relative to
app/src/main/java/com/mantz_it/rfanalyzer/ unless stated otherwise):

* format: headerless interleaved raw IQ exactly as the source delivered it --
  HACKRF s8, RTLSDR u8, AIRSPY / HYDRASDR s16le (IQ_FILE_FORMAT.md:5-81);
* writer: packets appended unchanged, optionally only while the squelch is
  satisfied (with the scheduler's 50-packet debounce), a new file begun before a
  packet would reach 4 000 000 000 bytes (analyzer/Scheduler.kt:52-53,77,161-234);
* file name: ``{yyyyMMdd-HHmmss}_{name}_{FORMAT}_{frequency}Hz_{rate}Sps.iq`` with
  the SI-prefixed numbers of ``Long.asStringWithUnit`` (database/RecordingDao.kt:87-90,
  ui/composable/HelperComposables.kt:168-179); a split recording's files are
  ``-001``, ``-002``, ... (ui/MainViewModel.kt:1815-1846);
* replay metadata: format, sample rate and frequency recovered from a file name
  by the reference's regular expressions (ui/MainViewModel.kt:2034-2078).

Replayed bytes go to the device unchanged (``SpectrumEngine.process`` with the
packet stride, ``rfanalyzer_amd.source``), so a recording made here replays
bit-identically through the GPU path.
"""
from __future__ import annotations

import datetime as _dt
import os
import re
from dataclasses import dataclass

FORMATS = ("HACKRF", "RTLSDR", "AIRSPY", "HYDRASDR")        # FilesourceFileFormat
ENGINE_FORMAT = {"HACKRF": "s8", "RTLSDR": "u8", "AIRSPY": "s16", "HYDRASDR": "s16"}
FILE_SPLIT_SIZE_BYTES = 4_000_000_000                        # Scheduler.kt:53
SQUELCH_DEBOUNCE_COUNT = 50                                  # Scheduler.kt:52
_LONG_MAX = 2 ** 63 - 1


def as_string_with_unit(value: int, unit: str) -> str:
    """Long.asStringWithUnit (HelperComposables.kt:168-179): divide by 1000 while exact
    (up to T), thousands separated by a space."""
    units = ["", "k", "M", "G", "T"]
    index = 0
    while value % 1000 == 0 and value >= 1000 and index < len(units) - 1:
        value //= 1000
        index += 1
    digits = f"{abs(value):,}".replace(",", " ")
    return f"{'-' if value < 0 else ''}{digits} {units[index]}{unit}"


def recording_file_name(name: str, file_format: str, frequency: int, sample_rate: int, date_ms: int,
                        split_index: int | None = None) -> str:
    """Recording.calculateFileName (RecordingDao.kt:87-90, local time) + split suffix (MainViewModel.kt:1834-1836)."""
    if file_format not in FORMATS:
        raise ValueError(f"unknown format {file_format!r}")
    ts = _dt.datetime.fromtimestamp(date_ms / 1000.0).strftime("%Y%m%d-%H%M%S")
    base = (f"{ts}_{name}_{file_format}_{as_string_with_unit(frequency, 'Hz').replace(' ', '')}_"
            f"{as_string_with_unit(sample_rate, 'Sps').replace(' ', '')}.iq")
    return base.replace(".iq", f"-{split_index:03d}.iq") if split_index is not None else base


@dataclass
class ReplayMetadata:
    file_format: str | None
    sample_rate: int | None
    frequency: int | None


_FMT_RULES = [  # MainViewModel.kt:2043-2054, later rules win
    ("HACKRF", [r".*hackrf.*", r".*HackRF.*", r".*HACKRF.*", r".*hackrfone.*"]),
    ("RTLSDR", [r".*rtlsdr.*", r".*rtl-sdr.*", r".*RTLSDR.*", r".*RTL-SDR.*"]),
    ("AIRSPY", [r".*airspy.*", r".*Airspy.*", r".*AIRSPY.*", r".*AirSpy.*"]),
    ("HYDRASDR", [r".*hydrasdr.*", r".*HydraSDR.*", r".*HYDRASDR.*", r".*HydraSdr.*"]),
]
_RATE_RULES = [(r".*(_|-|\s)([0-9]+)(sps|Sps|SPS).*", 1), (r".*(_|-|\s)([0-9]+)(ksps|Ksps|KSps|KSPS).*", 1000),
               (r".*(_|-|\s)([0-9]+)(msps|Msps|MSps|MSPS).*", 1_000_000)]
_FREQ_RULES = [(r".*(_|-|\s)([0-9]+)(hz|Hz|HZ).*", 1), (r".*(_|-|\s)([0-9]+)(khz|Khz|KHz|KHZ).*", 1000),
               (r".*(_|-|\s)([0-9]+)(mhz|Mhz|MHz|MHZ).*", 1_000_000)]


def parse_file_name(filename: str) -> ReplayMetadata:
    """setFilesourceUri's name parsing (MainViewModel.kt:2040-2078).  Kotlin ``matches`` is a
    whole-string match (``re.fullmatch``); ``replaceFirst`` after the greedy ``.*`` keeps the
    last occurrence; a number beyond Long aborts the remaining rules (NumberFormatException)
    and keeps what was found before; ``* 1000`` wraps like a Long.  None = not in the name."""
    out = ReplayMetadata(None, None, None)
    for fmt, pats in _FMT_RULES:
        if any(re.fullmatch(p, filename) for p in pats):
            out.file_format = fmt
    for attr, rules in (("sample_rate", _RATE_RULES), ("frequency", _FREQ_RULES)):
        for pat, mult in rules:
            m = re.fullmatch(pat, filename)
            if m:
                v = int(m.group(2))
                if v > _LONG_MAX:
                    return out
                setattr(out, attr, (v * mult + 2 ** 63) % 2 ** 64 - 2 ** 63)
    return out


class RecordingWriter:
    """Scheduler.kt:161-234 recording branch: raw packets appended unchanged, a new file
    begun before a packet would reach the split size, writes gated by the squelch with the
    debounce counter.  close() names the files like RecordingFinished: one file keeps
    ``base_name``, a split recording becomes ``-001``, ``-002``, ..."""

    def __init__(self, directory: str, base_name: str, split_at_4gb: bool = True, only_when_squelch: bool = False,
                 split_size: int = FILE_SPLIT_SIZE_BYTES):
        if not base_name.endswith(".iq"):
            raise ValueError("base_name must end in .iq")
        self.directory, self.base_name = directory, base_name
        self.split_at_4gb, self.only_when_squelch, self.split_size = split_at_4gb, only_when_squelch, split_size
        self.current_size = 0
        self.total_size = 0
        self.debounce = 0                   # Scheduler.kt:77
        self._tmp = []
        self.paths = []
        self._fh = self._open()

    def _open(self):
        path = os.path.join(self.directory, f"ongoing_recording_{len(self._tmp) + 1:03d}.iq")
        self._tmp.append(path)
        return open(path, "wb")

    def write_packet(self, packet: bytes, squelch_satisfied: bool = True) -> None:
        if self._fh is None:
            raise ValueError("recording closed")
        if squelch_satisfied:               # Scheduler.kt:162-165
            self.debounce = 0
        elif self.debounce < SQUELCH_DEBOUNCE_COUNT:
            self.debounce += 1
        if self.split_at_4gb and self.current_size + len(packet) >= self.split_size:  # Scheduler.kt:170-186
            self._fh.close()
            self.total_size += self.current_size
            self.current_size = 0
            self._fh = self._open()
        if squelch_satisfied or not self.only_when_squelch or self.debounce < SQUELCH_DEBOUNCE_COUNT:  # :199
            self._fh.write(packet)
            self.current_size += len(packet)

    @property
    def recorded_size(self) -> int:
        return self.total_size + self.current_size

    def close(self) -> list:
        if self._fh is not None:
            self._fh.close()
            self._fh = None
            names = ([self.base_name] if len(self._tmp) == 1 else
                     [self.base_name.replace(".iq", f"-{i + 1:03d}.iq") for i in range(len(self._tmp))])
            for tmp, nm in zip(self._tmp, names):
                dst = os.path.join(self.directory, nm)
                os.replace(tmp, dst)
                self.paths.append(dst)
        return self.paths

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
