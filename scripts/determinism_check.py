#!/usr/bin/env python3
"""Run the same batch through one librfa.so several times (and through the 1 M front kernel's
two alignment paths) and report whether the rows are bit-identical.  Loads RFA_LIB if set.
usage: determinism_check.py [n ...]"""
import sys

import numpy as np
import torch

sys.path.insert(0, "tests")
sys.path.insert(0, ".")
import signals  # noqa: E402
from rfanalyzer_amd.engine import SpectrumEngine  # noqa: E402

sizes = [int(x) for x in sys.argv[1:]] or [1 << 20, 32768, 65536]
for n in sizes:
    for fmt in ("s8", "f32"):
        frames = 7 if n >= (1 << 18) else 300
        data = signals.frames_bytes(n, frames, fmt, seed=77, tones=((0.0123, 0.3), (-0.41, 0.02)), noise=0.04)
        raw = np.frombuffer(data, np.uint8)
        outs = []
        with SpectrumEngine(n, "blackman", fmt, ring_rows=0) as e:
            for off in (0, 0, 0, 8, 2):
                if fmt == "f32" and off == 2:
                    continue
                buf = torch.zeros(raw.size + 64, dtype=torch.uint8, device="cuda")
                buf[off:off + raw.size] = torch.from_numpy(raw.copy()).cuda()
                rows = torch.empty((frames, n), dtype=torch.float32, device="cuda")
                e.process_tensor(buf[off:off + raw.size], frames, 0, rows)
                torch.cuda.synchronize()
                outs.append(rows.cpu().numpy())
        diffs = [int((o != outs[0]).sum()) for o in outs[1:]]
        mx = [float(np.max(np.abs(o - outs[0]))) for o in outs[1:]]
        print(f"n={n} {fmt}: bins differing from run 0 (runs: same x2, +8 B, +2 B): {diffs} max {mx}", flush=True)
