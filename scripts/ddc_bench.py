#!/usr/bin/env python3
"""Throughput of the demod front end (rfa_ddc_process) on
one GPU, beside the reference's per-sample loop in C (oracle orc_ddc_process,
1 thread) on the host.

Configurations follow the reference's rates: Decimator to the demodulator's
quadrature rate (Demodulator.kt:52-60: 2*48 kHz for AM/NFM/SSB, 8*48 kHz WFM)
from typical source rates (RTL-SDR 2.4 Msps u8, HackRF 20 Msps s8, Airspy
10 Msps s16).  One call processes S samples already resident in HBM; time is
wall clock over K calls bracketed by rfa_ddc_synchronize (kernel-only times
come from rocprofv3 over the same command).

Algorithmic bytes per call = S * bytes_per_sample + n_out * 8; work = 4 * T
flops per output (re/im multiply + add per tap, no FMA: the reference rounds
both).  Prints one JSON line per configuration.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

CONFIGS = [  # name, format, input rate, output rate, resampler (Resampler.kt) instead of Decimator
    ("rtlsdr_u8_2.4M_to_96k", "u8", 2_400_000, 96_000, False),
    ("hackrf_s8_20M_to_384k_wfm", "s8", 20_000_000, 384_000, False),
    ("hackrf_s8_20M_to_96k", "s8", 20_000_000, 96_000, False),
    ("airspy_s16_10M_to_96k", "s16", 10_000_000, 96_000, False),
    ("resampler_u8_2.4M_to_96k", "u8", 2_400_000, 96_000, True),
    ("resampler_s8_20M_to_384k_wfm", "s8", 20_000_000, 384_000, True),
]
BPS = {"s8": 2, "u8": 2, "s16": 4}


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--samples", type=int, default=1 << 27, help="complex samples per call")
    p.add_argument("--steps", type=int, default=10)
    p.add_argument("--cpu-seconds", type=float, default=3.0)
    p.add_argument("--only", default="")
    args = p.parse_args()
    import numpy as np
    import torch
    torch.cuda.init()
    from rfanalyzer_amd import demod
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(1)
    for name, fmt, sr, out, rsmp in CONFIGS:
        if args.only and args.only not in name:
            continue
        S = args.samples
        raw = torch.randint(0, 256, (S * BPS[fmt],), dtype=torch.uint8, device=dev, generator=g)
        torch.cuda.synchronize()
        fe = demod.FrontEnd(fmt, sr, out, resampler=rsmp)
        fe.set_frequencies(100_000_000, 100_150_000)
        cap = fe.max_outputs(S)
        re = torch.empty(cap, device=dev)
        im = torch.empty(cap, device=dev)
        fe.process_device(raw.data_ptr(), S, re.data_ptr(), im.data_ptr(), cap)   # warm-up
        fe.synchronize()
        t0 = time.perf_counter()
        n_out = 0
        for _ in range(args.steps):
            n_out = fe.process_device(raw.data_ptr(), S, re.data_ptr(), im.data_ptr(), cap)
        fe.synchronize()
        dt = (time.perf_counter() - t0) / args.steps
        I, D, T = fe.ratio()
        alg_bytes = S * BPS[fmt] + n_out * 8
        res = {"config": name, "format": fmt, "sample_rate": sr, "output_rate": out, "interpolation": I, "decimation": D, "taps_per_output": T,
               "samples_per_call": S, "ms_per_call": round(dt * 1e3, 4), "Msps": round(S / dt / 1e6, 1),
               "alg_GBps": round(alg_bytes / dt / 1e9, 1), "TFLOPs": round(4 * T * n_out / dt / 1e12, 2)}
        if args.cpu_seconds > 0:
            from oracle import demod as od
            if rsmp:
                print(json.dumps(res), flush=True)
                fe.close()
                continue
            cfe = od.CFrontEnd({"s8": od.IN_S8, "u8": od.IN_U8, "s16": od.IN_S16LE}[fmt], sr, out)
            cfe.set_frequencies(100_000_000, 100_150_000)
            chunk = np.random.default_rng(2).integers(0, 256, (1 << 20) * BPS[fmt], dtype=np.uint8)
            done, c0 = 0, time.perf_counter()
            while time.perf_counter() - c0 < args.cpu_seconds:
                cfe.process(chunk)
                done += 1 << 20
            cdt = time.perf_counter() - c0
            res["cpu_baseline"] = {"Msps": round(done / cdt / 1e6, 2), "cores": 1, "kind": "port",
                                   "sample": f"{done} samples in {cdt:.1f} s, orc_ddc_process (per-sample loop)"}
        print(json.dumps(res), flush=True)
        fe.close()
        del raw, re, im


if __name__ == "__main__":
    main()
