#!/usr/bin/env python3
"""Per-wave phase stamps of the wave-decoupled 64 K kernel (fft_w64.hip DIAG 32, A/B build,
RFA_STAMPS_FILE).  Each launch = [2048 * 16 * 8] u64 words, of which [256 blocks][4 items]
[16 waves][8] are used (s_memrealtime, 100 MHz): 0 item start, 1 own DMA landed, 2 pass 0 done,
3 exchange-0 entry barrier passed, 4 exchange 0 done, 5 pass 1 done, 6 exchange 1 (+ DMA issue)
done, 7 pass 2 + epilogue done.
usage: stamps_w64.py FILE [launch index, default last]"""
import sys

import numpy as np

W = 2048 * 16 * 8
d = np.fromfile(sys.argv[1], dtype=np.uint64)
nl = d.size // W
li = int(sys.argv[2]) if len(sys.argv) > 2 else nl - 1
s = d[li * W:li * W + 256 * 4 * 16 * 8].reshape(256, 4, 16, 8).astype(np.int64)
names = ["DMA wait", "pre-stage + pass 0", "barrier wait (exchange-0 entry)", "exchange 0", "pass 1",
         "exchange 1 + DMA issue", "pass 2 + epilogue"]
ok = (s[..., 0] > 0) & (s[..., 7] > 0)
print(f"launches {nl}, using {li}; (block, item, wave) samples: {ok.sum()}")
for k in range(1, 8):
    dt = (s[..., k] - s[..., k - 1])[ok] * 10e-3
    print(f"{names[k - 1]:34s} mean {dt.mean():6.2f} us  p10 {np.percentile(dt, 10):6.2f}  p90 {np.percentile(dt, 90):6.2f}")
tot = (s[..., 7] - s[..., 0])[ok] * 10e-3
print(f"{'item total (per wave)':34s} mean {tot.mean():6.2f} us")
# skew between waves of one workgroup at each stamp
for k in (0, 2, 3, 4, 6, 7):
    v = np.where(ok, s[..., k], 0)
    m = ok.all(axis=2)
    if m.sum() == 0:
        continue
    sk = (v.max(axis=2) - v.min(axis=2))[m] * 10e-3
    print(f"skew across the 16 waves at stamp {k}: mean {sk.mean():6.2f} us  p90 {np.percentile(sk, 90):6.2f}")
# item period per block (item start of wave 0 to next item start)
per = (s[:, 1:, :, 0] - s[:, :-1, :, 0])[ok[:, 1:] & ok[:, :-1]] * 10e-3
print(f"item period: mean {per.mean():6.2f} us")
# the arrival order at the exchange-0 barrier: which wave arrives last (stamp 2) per SIMD slot w % 4
v2 = s[..., 2]
last = np.argmax(np.where(ok, v2, 0), axis=2)[ok.all(axis=2)]
print("last wave to finish pass 0 (histogram over wave index):", np.bincount(last, minlength=16).tolist())
