#!/usr/bin/env python3
"""Analyse RFA_STAMPS_FILE phase stamps (profiling-only DIAG 32 build).
Each launch = [2048 blocks][16 items][8] u64 s_memrealtime (100 MHz) stamps:
0 item start, 1 staged frame landed (after barrier), 2 inputs in VGPRs,
3 after exchange 0, 4 after exchange 1, 5 after pass 2, 6 epilogue stores issued,
7 after the barrier that ends the pre-stage (the slowest wave's pre-stage + pass 0).
Phases are also split by the workgroup's residue (64 K: r = (block mod 16) >> 3).
usage: stamps.py FILE [launch index, default last]"""
import sys

import numpy as np

W = 2048 * 16 * 8
d = np.fromfile(sys.argv[1], dtype=np.uint64)
nl = d.size // W
li = int(sys.argv[2]) if len(sys.argv) > 2 else nl - 1
s = d[li * W:(li + 1) * W].reshape(2048, 16, 8).astype(np.int64)
valid = s[:, :, 0] > 0
t0 = s[:, :, 0][valid].min()
names = ["wait-staged", "load/convert/window+dft32", "barrier+xchg0", "pass1+xchg1", "pass2 (+DMA issue)", "epilogue"]
print(f"launches {nl}, using {li}; blocks with items: {valid.any(1).sum()}, items: {valid.sum()}")
res = ((np.arange(2048) % 16) >> 3)[:, None] * np.ones((1, 16), np.int64)


def phase(name, a, b, sel):
    m = sel & (a > 0) & (b > 0)
    if m.sum() == 0:
        return
    dt = (b - a)[m] * 10e-3  # us
    print(f"{name:26s} mean {dt.mean():7.2f} us  p10 {np.percentile(dt,10):7.2f}  p90 {np.percentile(dt,90):7.2f}")


for tag, sel in (("all", valid), ("r0", valid & (res == 0)), ("r1", valid & (res == 1))):
    print(f"-- {tag}")
    for k in range(1, 7):
        phase(names[k - 1], s[:, :, k - 1], s[:, :, k], sel)
    phase("  skew: stamp2 -> barrier", s[:, :, 2], s[:, :, 7], sel)
    phase("  xchg0 after barrier", s[:, :, 7], s[:, :, 3], sel)
for it in range(8):
    m = valid[:, it]
    if m.sum() == 0:
        break
    st = (s[:, it, 0][m] - t0) * 10e-3
    m = m & (s[:, it, 6] > 0)
    st = (s[:, it, 0][m] - t0) * 10e-3
    en = (s[:, it, 6][m] - t0) * 10e-3
    print(f"item {it}: {m.sum()} blocks, start {st.min():6.2f}..{st.max():6.2f} (median {np.median(st):6.2f}) "
          f"end {en.min():6.2f}..{en.max():6.2f} (median {np.median(en):6.2f}) us")
last = s[:, :, 6][valid].max()
print(f"span first start -> last epilogue {(last - t0) * 10e-3:.2f} us")
