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
    """Segment summary of the EMA over `rows` (m frames), the same form the
    chunked device update uses (state_partial_kernel, fft_kernels.hip):

    ``(decay, b, fresh)`` with ``em_out = decay * em_in + b`` for a finite
    ``em_in`` when no frame of the segment is -inf for that bin, and
    ``em_out = fresh`` (the segment's EMA started from -inf) when ``em_in`` is
    -inf or the segment restarts (after a -inf frame both runs coincide).
    ``decay`` is -1 for bins that restart."""
    al = np.float32(alpha)
    keep = np.float32(1) - al
    n = rows.shape[1]
    am = np.ones(n, np.float32)
    b = np.zeros(n, np.float32)
    fresh = np.full(n, -np.inf, np.float32)
    restart = np.zeros(n, bool)
    with np.errstate(invalid="ignore"):
        for x in np.asarray(rows, np.float32):
            fresh = np.where(fresh > -np.inf, fresh + al * (x - fresh), x).astype(np.float32)
            restart |= np.isneginf(x)
            am = (am * keep).astype(np.float32)
            b = (b + al * (x - b)).astype(np.float32)
    return np.where(restart, np.float32(-1), am), b, fresh


def ema_combine(state: np.ndarray | None, segments) -> np.ndarray:
    """Fold segment summaries (from `ema_partial`) in frame order; `state`
    None or -inf = uninitialised (the first frame seeds the average)."""
    em = None if state is None else np.asarray(state, np.float32).copy()
    for decay, b, fresh in segments:
        if em is None:
            em = np.full(b.shape, -np.inf, np.float32)
        with np.errstate(invalid="ignore"):
            em = np.where((em == -np.inf) | (decay < 0), fresh, decay * em + b).astype(np.float32)
    return em


def peak_combine(parts) -> np.ndarray:
    out = None
    for p in parts:
        out = p.copy() if out is None else np.maximum(out, p)
    return out
