#!/usr/bin/env python3
"""A/B-build diagnostics of the in-grid state path (rfa_debug_igs): for a config-3 batch, how many
units the main kernel summarised and the chunk counters after the state launch."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import rfanalyzer_amd
    from rfanalyzer_amd import _lib
    L = _lib.lib()
    L.rfa_debug_igs.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint)]
    n, frames = 65536, 500
    pool = [torch.randint(-100, 100, (n * frames * 2,), dtype=torch.int8, device="cuda") for _ in range(3)]
    out = (ctypes.c_uint * 80)()
    with rfanalyzer_amd.SpectrumEngine(n, "blackman", "s8", avg="ema", peak_hold=True, ring_rows=500) as e:
        for k in range(6):
            e.process_tensor(pool[k % 3], frames, 0, None)
            rc = L.rfa_debug_igs(e.handle, out)
            print(f"call {k}: rc {rc} gen {out[0]} in-grid units {out[1]} path {out[2]} counters {list(out[3:3 + 16])} tickets {list(out[35:35 + 16])} signals {out[3 + 66]} run {out[3 + 67]} exhausted {out[3 + 68]} none {out[3 + 69]} entered {out[3 + 70]} igs_on {out[3 + 71]}",
                  flush=True)


if __name__ == "__main__":
    main()
