#!/usr/bin/env python3
"""Throughput bench of the MI355X spectrum hot path (one JSON line on rank 0).

Default workload = BASELINE.json config 3, the one the metric is quoted on
("IQ Msamples/s + waterfall lines/s at 64k FFT"): 65536-point FFT, Blackman,
exponential averaging + peak-hold, synthetic 8-bit signed IQ, one stream per
GPU, B frames per step written into the device waterfall ring.

A step = one rfa_process() call over one batch of B frames already resident in
HBM (the batch rotates through a pool larger than the 256 MiB Infinity Cache so
every step streams from HBM).  For N>1 each rank runs its own independent
stream on its own GPU (weak scaling, no data-path collective); the timed region
is bracketed by barrier + torch.cuda.synchronize() and the max over ranks is
reported.  `value` is whole-job throughput in Msamples/s.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBPS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
BPS = {"s8": 2, "u8": 2, "s16": 4, "f32": 8, "f32p": 8}


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--fft-size", type=int, default=65536)
    p.add_argument("--format", default="s8", choices=list(BPS))
    p.add_argument("--window", default="blackman")
    p.add_argument("--frames", type=int, default=500,
                   help="frames per step (batch); default one full waterfall ring (500 rows, FftProcessor.kt:103)")
    p.add_argument("--avg", default="ema", choices=["none", "ema", "boxcar"])
    p.add_argument("--ema-alpha", type=float, default=0.1)
    p.add_argument("--no-peak", action="store_true")
    p.add_argument("--ring-rows", type=int, default=500)
    p.add_argument("--pool-mib", type=int, default=768, help="input pool size (> Infinity Cache)")
    p.add_argument("--cpu-seconds", type=float, default=10.0, help="cpu_baseline time budget (0 = skip)")
    p.add_argument("--f32-steps", type=int, default=20, help="steps of the float32-input companion run (0 = skip)")
    p.add_argument("--demod-steps", type=int, default=5,
                   help="calls of the demod front-end companion (SURVEY §8(f) row 4; 0 = skip)")
    p.add_argument("--traffic-file", default=os.path.join(ROOT, "profiles", "pmc_traffic.json"))
    return p.parse_args()


def make_pool(torch, n, frames, fmt, pool_mib, seed, device):
    """Synthetic IQ batches on device: slowly drifting tone + complex AWGN."""
    samples = n * frames
    batch_bytes = samples * BPS[fmt]
    count = max(2, -(-pool_mib * 2 ** 20 // batch_bytes))
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    pool = []
    for b in range(count):
        t = torch.arange(samples, device=device, dtype=torch.float64) + b * samples
        ph = 2 * torch.pi * (0.07 * t + 0.5e-3 * t * t / max(samples * count, 1))
        re = 0.5 * torch.cos(ph) + 0.05 * torch.randn(samples, device=device, generator=g, dtype=torch.float64)
        im = 0.5 * torch.sin(ph) + 0.05 * torch.randn(samples, device=device, generator=g, dtype=torch.float64)
        if fmt in ("s8", "u8", "s16"):
            scale, off, lo, hi, dt = {"s8": (128, 0.0, -128, 127, torch.int8), "u8": (128, 127.4, 0, 255, torch.uint8),
                                      "s16": (32768, 0.0, -32768, 32767, torch.int16)}[fmt]
            iq = torch.stack([re, im], 1).reshape(-1) * scale + off
            pool.append(torch.clamp(torch.round(iq), lo, hi).to(dt))
        elif fmt == "f32":
            pool.append(torch.stack([re, im], 1).reshape(-1).to(torch.float32))
        else:  # planar per frame
            pool.append(torch.cat([re.view(frames, n), im.view(frames, n)], 1).reshape(-1).to(torch.float32))
        del t, ph, re, im
    return pool


def max_over_ranks(value: float, world: int, device) -> float:
    """Slowest rank's time: the timed region ends when the last GPU finishes."""
    if world <= 1:
        return value
    import torch
    import torch.distributed as dist

    t = torch.tensor([value], device=device, dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def cpu_baseline(args, n, seconds, threads=1):
    """Reference loop (pffft + restated JVM loops, oracle/_ref) on 1 host core, bounded time."""
    import numpy as np

    import oracle

    fmt = {"s8": 0, "f32": 3}.get(args.format)
    frames = max(1, (8 * 2 ** 20) // (n * 8))  # ~8 MB sample, processed repeatedly
    rng = np.random.Generator(np.random.PCG64(3))
    t = np.arange(n * frames)
    x = 0.5 * np.exp(2j * np.pi * 0.07 * t) + 0.05 * (rng.standard_normal(t.size) + 1j * rng.standard_normal(t.size))
    iq = np.empty(2 * t.size)
    iq[0::2], iq[1::2] = x.real, x.imag
    if fmt == 0 or fmt is None:
        data, fmt = np.clip(np.rint(iq * 128), -128, 127).astype(np.int8), 0
    else:
        data = iq.astype(np.float32)
    w = oracle.window(n, oracle.WIN_BLACKMAN)
    ring_rows = 500
    fp = ctypes.POINTER(ctypes.c_float)

    def run_ref(budget):
        """One thread = one reference FftProcessor loop (own ring + peaks)."""
        lib = oracle.ref()
        ring = np.full((ring_rows, n), -9999, np.float32)
        peaks = np.full(n, -999999, np.float32)
        done, t0 = 0, time.perf_counter()
        while time.perf_counter() - t0 < budget:
            rc = lib.ref_loop(data.ctypes.data, fmt, n, frames, n * (2 if fmt == 0 else 8), w.ctypes.data_as(fp),
                              ring.ctypes.data_as(fp), ring_rows, peaks.ctypes.data_as(fp))
            assert rc == 0
            done += frames
        return done, time.perf_counter() - t0

    if oracle.ref_available():
        done, el = run_ref(seconds)
        kind = "reference"
        what = ("reference pffft.c (oracle/_ref, -O3 -ffast-math) + restated FftProcessor loop: LUT convert, "
                "Blackman, FFT, log-mag+shift, ring copy, peak-hold")
    else:
        done, t0 = 0, time.perf_counter()
        while time.perf_counter() - t0 < seconds:
            oracle.spectrum_rows(data, fmt, n, frames, None, oracle.WIN_BLACKMAN)
            done += frames
        el = time.perf_counter() - t0
        kind = "port"
        what = "oracle C restatement (float64 FFT) -- reference pffft build absent"
    out = {"value": round(done * n / el / 1e6, 3), "unit": "Msamples/s", "cores": 1, "kind": kind,
           "sample": f"{frames} x {n}-pt {'s8' if fmt == 0 else 'f32'} frames looped for {el:.1f} s; {what}",
           "lines_per_s": round(done / el, 2)}
    if kind == "reference" and threads > 1:
        # frame-parallel on the host's cores: one independent loop per thread;
        # ctypes releases the GIL for the duration of each ref_loop call
        import threading

        res = [None] * threads
        ths = [threading.Thread(target=lambda i=i: res.__setitem__(i, run_ref(seconds / 2))) for i in range(threads)]
        for t in ths:
            t.start()
        for t in ths:
            t.join()
        el = max(r[1] for r in res)
        out["multi_core"] = {"value": round(sum(r[0] for r in res) * n / el / 1e6, 3), "cores": threads,
                             "sample": f"{threads} threads x the same loop for {el:.1f} s"}
    return out


def copy_ceiling(torch, device, mib=1024, iters=10):
    """Device stream-copy ceiling in the same run (SURVEY.md §8(d) primary denominator):
    torch's copy kernel over two 1 GiB buffers, GB/s = 2 x bytes / time."""
    src = torch.empty(mib * 2 ** 20 // 4, dtype=torch.float32, device=device).fill_(1.0)
    dst = torch.empty_like(src)
    dst.copy_(src)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        dst.copy_(src)
    e1.record()
    torch.cuda.synchronize()
    gbps = 2 * src.numel() * 4 * iters / (e0.elapsed_time(e1) * 1e-3) / 1e9
    del src, dst
    return round(gbps, 1)


def demod_companion(torch, device, steps, samples=1 << 26):
    """§8(f) row 4 beside the headline (never `value`): RTL-SDR u8 2.4 Msps mixed and
    decimated to the 96 kHz quadrature rate (Decimator.java:175-191), raw bytes
    resident in HBM, wall clock over `steps` calls of rfa_ddc_process."""
    from rfanalyzer_amd import demod
    raw = torch.randint(0, 256, (2 * samples,), dtype=torch.uint8, device=device)
    fe = demod.FrontEnd("u8", 2_400_000, 96_000, device=device.index or 0)
    fe.set_frequencies(100_000_000, 100_150_000)
    cap = fe.max_outputs(samples)
    re = torch.empty(cap, device=device)
    im = torch.empty(cap, device=device)
    torch.cuda.synchronize()
    fe.process_device(raw.data_ptr(), samples, re.data_ptr(), im.data_ptr(), cap)
    fe.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        fe.process_device(raw.data_ptr(), samples, re.data_ptr(), im.data_ptr(), cap)
    fe.synchronize()
    dt = (time.perf_counter() - t0) / steps
    _, d, t = fe.ratio()
    fe.close()
    return {"workload": "u8 2.4 Msps -> 96 kHz, mix + 273-tap decimating FIR (D 25)", "value": round(samples / dt / 1e6, 1),
            "unit": "Msamples/s", "ms_per_call": round(dt * 1e3, 4), "samples_per_call": samples, "decimation": d,
            "taps": t}


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        dist.init_process_group(backend="nccl" if torch.cuda.is_available() else "gloo")
    torch.cuda.set_device(local)
    device = torch.device("cuda", local)

    import rfanalyzer_amd

    n, frames, fmt = args.fft_size, args.frames, args.format
    stream = torch.cuda.Stream(device)  # a real stream shared by torch and librfa (not the null stream)
    torch.cuda.set_stream(stream)

    def run(fmt, steps, warmup, seed, sync_ranks):
        """Warm up, then time `steps` rfa_process() steps of one batch each (barrier +
        synchronize on both sides).  Returns (wall seconds, main-kernel ms per launch, kernel)."""
        eng = rfanalyzer_amd.SpectrumEngine(n, args.window, fmt, avg=args.avg, avg_length=min(30, args.ring_rows - 1),
                                            ema_alpha=args.ema_alpha, peak_hold=not args.no_peak,
                                            ring_rows=args.ring_rows, device=local)
        eng.set_stream(stream.cuda_stream)
        pool = make_pool(torch, n, frames, fmt, args.pool_mib, seed, device)
        eng.set_tuning(100_000_000, 20_000_000)

        def step(k):
            eng.process_tensor(pool[k % len(pool)], frames, 0, None)

        for k in range(warmup):
            step(k)
        torch.cuda.synchronize()
        if sync_ranks:
            dist.barrier()
        torch.cuda.synchronize()
        eng.set_profiling(True)
        ms0, l0 = eng.kernel_time()
        t0 = time.perf_counter()
        for k in range(steps):
            step(warmup + k)
        torch.cuda.synchronize()
        if sync_ranks:
            dist.barrier()
        torch.cuda.synchronize()
        elapsed = time.perf_counter() - t0
        ms1, l1 = eng.kernel_time()
        eng.set_profiling(False)
        name = eng.main_kernel_name()
        eng.close()
        del pool
        return elapsed, (ms1 - ms0) / max(1, l1 - l0), name

    elapsed, kernel_ms, kernel_name = run(fmt, args.steps, args.warmup, 3 + rank, world > 1)
    elapsed = max_over_ranks(elapsed, world, device)

    samples = world * args.steps * frames * n
    msps = samples / elapsed / 1e6
    s_in = BPS[fmt]
    alg_bytes = frames * n * (s_in + 4)  # per main-kernel launch: raw IQ in + one fp32 row out
    achieved = alg_bytes / (kernel_ms * 1e-3) / 1e9
    traffic = None
    try:
        with open(args.traffic_file) as fh:
            tr = json.load(fh)
        key = f"{fmt}_{n}_{frames}"
        if key in tr:
            traffic = tr[key]["hbm_bytes_per_launch"]
    except (OSError, ValueError, KeyError):
        pass
    result = {
        "metric": "IQ Msamples/s + waterfall lines/s at 64k FFT; achieved HBM GB/s vs roofline",
        "value": round(msps, 2),
        "unit": "Msamples/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed * 1e3 / args.steps, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic",
        "lines_per_s": round(samples / n / elapsed, 1),
        "config": {"workload": f"config3: {n}-pt FFT, {args.window} window, {fmt} IQ, "
                               f"{'EMA' if args.avg == 'ema' else args.avg} + "
                               f"{'peak-hold' if not args.no_peak else 'no peak'}, ring {args.ring_rows} rows, "
                               f"one stream per GPU",
                   "fft_size": n, "frames_per_step": frames, "input_format": fmt, "avg": args.avg,
                   "ema_alpha": args.ema_alpha, "peak_hold": not args.no_peak, "ring_rows": args.ring_rows,
                   "parallelism": f"streams{world}"},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBPS, 4), "traffic": traffic,
                     "kernel": kernel_name, "kernel_ms": round(kernel_ms, 4),
                     "alg_bytes_per_launch": alg_bytes},
    }
    if rank == 0 and world == 1:
        result["roofline"]["copy_GBps"] = copy_ceiling(torch, device)
        result["roofline"]["frac_of_copy"] = round(achieved / result["roofline"]["copy_GBps"], 4)
    if rank == 0 and world == 1 and fmt != "f32" and args.f32_steps > 0:
        # BASELINE.json asks for 8-bit AND float32 IQ: the same workload on complex-float32
        # input (12 B/sample algorithmic), reported beside the headline (never `value`)
        el32, k32, _ = run("f32", args.f32_steps, args.warmup, 103, False)
        alg32 = frames * n * (BPS["f32"] + 4)
        result["f32"] = {"value": round(args.f32_steps * frames * n / el32 / 1e6, 2), "unit": "Msamples/s",
                         "ms_per_step": round(el32 * 1e3 / args.f32_steps, 4), "kernel_ms": round(k32, 4),
                         "roofline_achieved_GBps": round(alg32 / (k32 * 1e-3) / 1e9, 1),
                         "roofline_frac": round(alg32 / (k32 * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4),
                         "alg_bytes_per_launch": alg32}
    if rank == 0 and world == 1 and args.demod_steps > 0:
        result["demod"] = demod_companion(torch, device, args.demod_steps)
    if rank == 0 and world == 1 and args.cpu_seconds > 0:
        result["cpu_baseline"] = cpu_baseline(args, n, args.cpu_seconds, min(16, os.cpu_count() or 1))
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
