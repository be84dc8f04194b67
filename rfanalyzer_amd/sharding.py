"""Multi-GPU partitioning of the spectrum path (no data-path collective).

Frames are independent through FFT and log-mag, so:

* a batch of frames is split into contiguous per-rank ranges
  (``frame_range``), each rank runs its own handle on its own GPU;
* independent streams map one per rank.

The only cross-rank dependency is state of ONE stream split over ranks, which
the reference never does (one FftProcessor thread per stream).  For
completeness the exact combines are provided: peak-hold is an element-wise
max; the EMA over a segment of m frames is affine in the incoming state,
``avg_end = (1-alpha)^m * avg_start + partial`` (``ema_partial`` /
``ema_combine``) -- one host-side N-float step per batch, not a collective.
"""
from __future__ import annotations

import numpy as np


def frame_range(n_frames: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous [start, end) of frames for `rank` (sizes differ by at most one)."""
    base, extra = divmod(n_frames, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def ema_partial(rows: np.ndarray, alpha: float):
    """Segment summary for the EMA: (partial, first_row, decay, restarted) with
    partial = sum_k alpha (1-alpha)^(m-1-k) x_k and decay = (1-alpha)^m.
    Bins that see a -inf inside the segment restart there (the state becomes
    -inf and the next frame re-seeds it): for them `restarted` is set and
    `partial` already holds the exact end state."""
    a = np.float64(alpha)
    m = rows.shape[0]
    partial = np.zeros(rows.shape[1], np.float64)
    restarted = np.zeros(rows.shape[1], bool)
    fresh = np.full(rows.shape[1], np.nan)
    for k in range(m):
        x = rows[k].astype(np.float64)
        neg = np.isneginf(x)
        # bins restarted earlier follow the sequential rule on `fresh`
        fresh = np.where(restarted, np.where(np.isneginf(fresh) | np.isnan(fresh), x, fresh + a * (x - fresh)), fresh)
        newly = neg & ~restarted
        fresh = np.where(newly, -np.inf, fresh)
        restarted |= neg
        partial = (1 - a) * partial + a * x
    partial = np.where(restarted, fresh, partial)
    return partial, rows[0].astype(np.float64), float((1 - a) ** m), restarted


def ema_combine(state: np.ndarray | None, segments) -> np.ndarray:
    """Fold segment summaries (from `ema_partial`) in order; `state` None/-inf = uninitialised."""
    s = None if state is None else np.asarray(state, np.float64).copy()
    for partial, first, decay, restarted in segments:
        if s is None:
            s = np.full(partial.shape, -np.inf)
        init = np.where(s > -np.inf, s, first)
        s = np.where(restarted, partial, decay * init + partial)
    return s.astype(np.float32)


def peak_combine(parts) -> np.ndarray:
    out = None
    for p in parts:
        out = p.copy() if out is None else np.maximum(out, p)
    return out
