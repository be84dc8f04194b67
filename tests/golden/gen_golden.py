#!/usr/bin/env python3
"""Generate tests/golden fixtures from the REFERENCE's own pffft.

Run in the build container (where /root/reference exists) after
``make -C oracle``.  Expected rows come from oracle/_ref/libpffft_ref.so
(the reference's vendored pffft.c compiled from /root/reference plus our
JNI-free restatement of nativedsp.cpp:44-81), fed with the reference's LUT
conversion and window applied in float32 exactly as NativeDsp.kt:55-58 does.
State sequences are replayed through oracle/processor.py (FftProcessor.kt
restatement).  Inputs are NOT committed: they are regenerated from the seeds
in manifest.json by tests/signals.py and checked against the stored SHA-256.

Usage:  python tests/golden/gen_golden.py
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(HERE))

import oracle  # noqa: E402
from oracle import processor  # noqa: E402
import signals  # noqa: E402

WINDOWS = {"blackman": oracle.WIN_BLACKMAN, "hann": oracle.WIN_HANN, "none": oracle.WIN_NONE}


def fixture_input(spec: dict) -> bytes:
    g = spec["gen"]
    if g["kind"] == "frames":
        return signals.frames_bytes(spec["n"], spec["n_frames"], spec["fmt"], g["seed"],
                                    tones=tuple(tuple(t) for t in g["tones"]), noise=g["noise"],
                                    drift=g.get("drift", 0.0))
    if g["kind"] == "kat":
        return signals.kat_bytes(g["kat"], spec["n"])
    if g["kind"] == "file":
        return signals.file_capture(g["n_bytes"], g["seed"], g["sample_rate"])
    raise ValueError(g["kind"])


def frames_spec(name, n, fmt, window, n_frames, seed, tones, noise, drift=0.0, subset=1):
    return {"name": name, "n": n, "fmt": fmt, "window": window, "n_frames": n_frames, "subset_stride": subset,
            "gen": {"kind": "frames", "seed": seed, "tones": [list(t) for t in tones], "noise": noise,
                    "drift": drift}}


def kat_spec(kat, n, window="none"):
    fmt = "s8" if kat == "zeros" else "f32"
    return {"name": f"kat_{kat}_n{n}_{window}", "n": n, "fmt": fmt, "window": window, "n_frames": 1,
            "subset_stride": 1, "gen": {"kind": "kat", "kat": kat}}


SPECS = [
    kat_spec("impulse", 1024), kat_spec("dc", 1024), kat_spec("nyquist", 1024), kat_spec("tone_bin", 1024),
    kat_spec("tone_halfbin", 1024, "blackman"), kat_spec("zeros", 1024, "blackman"),
    kat_spec("tone_bin", 16384), kat_spec("impulse", 65536),
    frames_spec("s8_n1024_x4", 1024, "s8", "blackman", 4, 11, ((0.125, 0.5),), 0.05),
    frames_spec("u8_n1024_x2", 1024, "u8", "blackman", 2, 12, ((-0.2, 0.4),), 0.05),
    frames_spec("s16_n1024_x2", 1024, "s16", "blackman", 2, 13, ((0.3, 0.25),), 0.01),
    frames_spec("f32p_n1024_x2", 1024, "f32p", "blackman", 2, 14, ((0.05, 0.5),), 0.02),
    frames_spec("s8_n8192_x4", 8192, "s8", "blackman", 4, 4, ((0.1, 0.5),), 0.05),
    frames_spec("f32_n8192_x2", 8192, "f32", "hann", 2, 4, ((0.1, 0.5),), 0.01),
    frames_spec("f32_n16384_hann", 16384, "f32", "hann", 2, 2, ((1000 / 16384, 0.5), (5000.5 / 16384, 0.05)), 0.01),
    frames_spec("s8_n16384", 16384, "s8", "blackman", 1, 21, ((0.21, 0.5),), 0.05),
    frames_spec("s16_n16384", 16384, "s16", "blackman", 1, 22, ((-0.33, 0.5),), 0.001),
    frames_spec("s8_n32768", 32768, "s8", "blackman", 1, 23, ((0.01, 0.5),), 0.05),
    frames_spec("s8_n65536", 65536, "s8", "blackman", 1, 3, ((0.07, 0.5),), 0.05, drift=0.001),
    frames_spec("f32_n65536", 65536, "f32", "blackman", 1, 3, ((0.07, 0.5),), 0.01, drift=0.001),
    frames_spec("s8_n1048576", 1048576, "s8", "blackman", 1, 5, ((0.19, 0.5),), 0.05, subset=64),
    {"name": "file_s8_2msps_n1024", "n": 1024, "fmt": "s8", "window": "blackman", "packet_size": 262144,
     "subset_stride": 1, "gen": {"kind": "file", "n_bytes": 4_000_000, "seed": 1, "sample_rate": 2_000_000}},
]

STATE_SPEC = {
    "name": "state_s8_n1024", "n": 1024, "fmt": "s8", "window": "blackman", "n_frames": 40, "ring_rows": 300,
    "boxcar_length": 5, "ema_alpha": 0.1,
    # (frame index from which it applies, frequency, sample_rate): retune at frame 25 by +37 kHz,
    # sample-rate change at frame 33
    "tuning": [[0, 100_000_000, 2_000_000], [25, 100_037_000, 2_000_000], [33, 100_037_000, 2_400_000]],
    "gen": {"kind": "frames", "seed": 7, "tones": [[0.125, 0.5], [-0.31, 0.05]], "noise": 0.05, "drift": 2.0},
}


def run_state(spec, rows_fn):
    n, nf = spec["n"], spec["n_frames"]
    data = fixture_input(spec)
    rows = rows_fn(data, spec)
    p = processor.FftProcessorRef(n, spec["ring_rows"], peak_hold=True, ema_alpha=spec["ema_alpha"])
    tuning = spec["tuning"]
    for f in range(nf):
        freq, sr = [t for t in tuning if t[0] <= f][-1][1:]
        p.push(rows[f], freq, sr)
    ring_newest = np.stack([p.ring[(p.read_index + r) % p.ring.shape[0]] for r in range(8)])
    return data, {"peaks": p.peaks, "boxcar": p.boxcar(spec["boxcar_length"]), "ema": p.ema,
                  "ring_newest8": ring_newest}


def pffft_rows(data, spec):
    fmt = signals.FORMATS[spec["fmt"]]
    if "packet_size" in spec:
        frames = processor.file_frames(len(data), spec["packet_size"], oracle.BYTES_PER_SAMPLE[fmt], spec["n"])
        stride = frames[1][0] - frames[0][0] if len(frames) > 1 else 0
        return oracle.ref_spectrum_rows(data, fmt, spec["n"], len(frames), stride, WINDOWS[spec["window"]])
    return oracle.ref_spectrum_rows(data, fmt, spec["n"], spec["n_frames"], None, WINDOWS[spec["window"]])


def main():
    oracle.build()
    if not oracle.ref_available():
        sys.exit("oracle/_ref/libpffft_ref.so missing: run in the container with /root/reference")
    manifest = {"generator": "tests/golden/gen_golden.py", "source": "reference pffft.c via oracle/_ref",
                "fixtures": []}
    for spec in SPECS:
        data = fixture_input(spec)
        rows = pffft_rows(data, spec)
        if "packet_size" in spec:
            spec["n_frames"] = rows.shape[0]
        sub = spec["subset_stride"]
        np.save(os.path.join(HERE, spec["name"] + ".npy"), np.ascontiguousarray(rows[:, ::sub]))
        spec["input_sha256"] = signals.sha256(data)
        spec["argmax"] = [int(a) for a in np.argmax(rows, axis=1)]
        spec["expected"] = spec["name"] + ".npy"
        manifest["fixtures"].append(spec)
        print(f"{spec['name']}: frames={rows.shape[0]} argmax={spec['argmax'][:4]}")
    data, st = run_state(STATE_SPEC, pffft_rows)
    spec = dict(STATE_SPEC)
    spec["input_sha256"] = signals.sha256(data)
    np.savez(os.path.join(HERE, spec["name"] + ".npz"), **st)
    spec["expected"] = spec["name"] + ".npz"
    manifest["state"] = spec
    with open(os.path.join(HERE, "manifest.json"), "w") as fh:
        json.dump(manifest, fh, indent=1)
    print("wrote", len(manifest["fixtures"]), "fixtures + state")


if __name__ == "__main__":
    main()
