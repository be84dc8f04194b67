#!/usr/bin/env python3
"""Kernel micro-bench: main FFT kernel time (HIP events on the handle stream)
for a grid of (N, format, frames) with inputs resident in HBM.  Prints one
line per config: us/launch, algorithmic GB/s, Msamples/s."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

BPS = {"s8": 2, "u8": 2, "s16": 4, "f32": 8, "f32p": 8}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="1024,8192,16384,65536")
    ap.add_argument("--formats", default="s8,f32")
    ap.add_argument("--samples", type=int, default=1 << 24, help="samples per launch")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--state", action="store_true", help="EMA + peak-hold + ring")
    ap.add_argument("--no-prof", action="store_true", help="time steps without the per-launch HIP events")
    ap.add_argument("--channel-bins", type=int, default=0,
                    help="with --state: a squelch channel this many bins wide (channel mean per frame)")
    args = ap.parse_args()
    import torch

    import rfanalyzer_amd

    torch.cuda.set_stream(torch.cuda.Stream())
    for fmt in args.formats.split(","):
        for n in [int(x) for x in args.sizes.split(",")]:
            frames = max(1, args.samples // n)
            nbytes = frames * n * BPS[fmt]
            pools = [torch.randint(-100, 100, (nbytes,), dtype=torch.int8, device="cuda") for _ in range(4)]
            if fmt in ("f32", "f32p"):
                pools = [torch.randn(nbytes // 4, device="cuda") * 0.3 for _ in range(4)]
            rows = torch.empty(frames * n, dtype=torch.float32, device="cuda")
            kw = dict(avg="ema", peak_hold=True, ring_rows=max(frames, 300)) if args.state else dict(ring_rows=0)
            with rfanalyzer_amd.SpectrumEngine(n, "blackman", fmt, **kw) as e:
                e.set_stream(torch.cuda.current_stream().cuda_stream)
                if args.channel_bins and args.state:  # 1000 Hz per bin: sample rate = 1000 N
                    f0 = 100_000_000
                    e.set_tuning(f0, 1000 * n)
                    e.set_channel(f0 - 500 * args.channel_bins, f0 + 500 * args.channel_bins)
                out = None if args.state else rows
                for k in range(3):
                    e.process_tensor(pools[k % 4], frames, 0, out)
                torch.cuda.synchronize()
                e.set_profiling(not args.no_prof)
                ms0, l0 = e.kernel_time()
                ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                ev0.record()
                for k in range(args.iters):
                    e.process_tensor(pools[k % 4], frames, 0, out)
                ev1.record()
                torch.cuda.synchronize()
                ms1, l1 = e.kernel_time()
                kus = (ms1 - ms0) / (l1 - l0) * 1e3 if l1 > l0 else float("nan")
                step_us = ev0.elapsed_time(ev1) / args.iters * 1e3
                alg = frames * n * (BPS[fmt] + 4)
                print(f"{fmt:5s} N={n:8d} frames={frames:6d} kernel {kus:9.1f} us  {alg / kus / 1e3:7.1f} GB/s  "
                      f"{frames * n / kus:9.1f} Msps | step {step_us:9.1f} us {frames * n / step_us:9.1f} Msps",
                      flush=True)
            del pools, rows


if __name__ == "__main__":
    main()
