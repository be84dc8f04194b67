"""Fixture loading and the dB parity metric shared by the CPU and GPU tests."""
from __future__ import annotations

import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(HERE, "golden")
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, GOLDEN)

import signals  # noqa: E402

# north star: "output log-magnitude spectra match the reference CPU/nativedsp
# path ... to within 0.01 dB with bit-exact bin ordering"
DB_TOL = 0.01
# The row unit is 10*log10(|X|/N) (a magnitude dB, nativedsp.cpp:78).  The
# 0.01 dB bar is applied to bins above a floor below the row's total
# (Parseval) level; below it a bin holds fp32 rounding noise (pffft leaves
# exact zeros where a float64 FFT has -300 dB) and both sides only have to be
# deep.  Two floors, because the reference is itself an fp32 FFT:
#   vs the float64 oracle:   FLOOR_DB = 50 (magnitude 1e-5 of the total)
#   vs pffft golden rows:    FLOOR_PFFFT_DB = 45
# At 50 the reference's own pffft is 0.0077 dB off float64 on the s16/16K
# fixture (tests/test_oracle.py measures it), so two correct fp32 FFTs can
# differ by > 0.01 dB there; at 45 every bin is >= 1e4 x the fp32 rounding
# noise and pffft-vs-float64 stays <= 0.0031 dB on every fixture.
FLOOR_DB = 50.0
FLOOR_PFFFT_DB = 45.0

WINDOW_IDS = {"blackman": 0, "hann": 1, "none": 2}


def manifest() -> dict:
    with open(os.path.join(GOLDEN, "manifest.json")) as fh:
        return json.load(fh)


def fixture_input(spec: dict) -> bytes:
    g = spec["gen"]
    if g["kind"] == "frames":
        data = signals.frames_bytes(spec["n"], spec["n_frames"], spec["fmt"], g["seed"],
                                    tones=tuple(tuple(t) for t in g["tones"]), noise=g["noise"],
                                    drift=g.get("drift", 0.0))
    elif g["kind"] == "kat":
        data = signals.kat_bytes(g["kat"], spec["n"])
    elif g["kind"] == "file":
        data = signals.file_capture(g["n_bytes"], g["seed"], g["sample_rate"])
    else:
        raise ValueError(g["kind"])
    assert signals.sha256(data) == spec["input_sha256"], f"{spec['name']}: regenerated input differs"
    return data


def expected(spec: dict):
    path = os.path.join(GOLDEN, spec["expected"])
    if path.endswith(".npz"):
        with np.load(path, allow_pickle=False) as z:
            return {k: z[k] for k in z.files}
    return np.load(path, allow_pickle=False)


def assert_same_peak_bins(got: np.ndarray, exp_argmax) -> None:
    """Bit-exact bin ordering: the reference's peak bin is our peak bin.  An
    exact tie (e.g. a tone at k+0.5 under a symmetric window) is decided by
    rounding on either side, so the reference's bin only has to be within
    DB_TOL of our maximum."""
    got = np.atleast_2d(got)
    for row, a in zip(got, exp_argmax):
        assert row[a] >= row.max() - DB_TOL, (int(np.argmax(row)), a)


def pffft_diff(got: np.ndarray, exp: np.ndarray) -> float:
    """db_diff against rows produced by the reference's own pffft (see FLOOR_PFFFT_DB)."""
    return db_diff(got, exp, FLOOR_PFFFT_DB)


def db_diff(got: np.ndarray, exp: np.ndarray, floor_db: float | None = None) -> float:
    """Max |dB difference| over bins within floor_db (default FLOOR_DB) of the row's total level.

    Raises AssertionError on a structural mismatch: -inf vs finite above the
    floor, a NaN, or a deep bin on one side that is shallow on the other."""
    got = np.atleast_2d(np.asarray(got, np.float32))
    exp = np.atleast_2d(np.asarray(exp, np.float32))
    assert got.shape == exp.shape, (got.shape, exp.shape)
    assert not np.isnan(got).any(), "NaN in output"
    floor = FLOOR_DB if floor_db is None else floor_db
    worst = 0.0
    for g, e in zip(got, exp):
        if np.all(np.isneginf(e)):
            assert np.all(np.isneginf(g)), "expected an all -inf row (all-zero input)"
            continue
        mag = np.power(10.0, e.astype(np.float64) / 10.0)
        top = 10.0 * np.log10(np.sqrt(np.sum(mag * mag)))
        live = e >= top - floor
        assert np.all(np.isfinite(g[live])), "non-finite bin above the floor"
        worst = max(worst, float(np.max(np.abs(g[live] - e[live]))))
        deep = ~live
        if deep.any():
            assert np.all(g[deep] < top - floor + 20.0), "deep bin came out shallow"
    return worst
