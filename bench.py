#!/usr/bin/env python3
"""Throughput bench of the MI355X spectrum hot path (one JSON line on rank 0).

Default workload = BASELINE.json config 3, the one the metric is quoted on
("IQ Msamples/s + waterfall lines/s at 64k FFT"): 65536-point FFT, Blackman,
exponential averaging + peak-hold, synthetic 8-bit signed IQ, ring of 500
rows, one stream per GPU (``--mode streams``).

A step = ``--calls-per-step`` consecutive rfa_process() calls, each over one
batch of B frames already resident in HBM (B = one full ring by default, so a
step is a run of waterfall-sized batches, each updating ring + peak + EMA as
FftProcessor does frame by frame).  Batches rotate through a pool larger than
the 256 MiB Infinity Cache, so every call streams from HBM.  ``value`` is
whole-job Msamples/s.

Multi-GPU (no data-path collective):
* ``--mode streams`` (config 5's shape): every rank runs its own independent
  stream on its own GPU; weak scaling.
* ``--mode shard`` (config 4): batches of 256 frames x 8192 points; each batch
  is split into contiguous frame ranges (sharding.frame_range), one per rank;
  strong scaling (the batch is fixed as N grows).  A call enqueues
  ``--batches-per-call`` consecutive batches (rfa_process_batches: one kernel
  launch) so small per-rank shards are not launch-bound.  ``--gather`` also
  gathers the rows to rank 0 each call (the one real exchange of this mode).

Companions on the same line (never ``value``), run by every rank in multi-GPU
runs with per-rank times: ``f32`` (the headline on float32 IQ), ``config2``
(16 K cf32 Hann), ``config4`` / ``config4_f32`` (the shard workload on s8 and cf32
input), ``config5`` (a 1 M-point
stream per rank), ``host_fed`` (configs 3 and 2 fed from pinned host memory over
PCIe, H2D overlapped on a second stream), ``demod`` and, on rank 0 of a 1-GPU run,
``cpu_baseline`` and ``config4.one_batch_per_call.c_loop`` (tools/call_bench: the
C-ABI's per-call cost timed from C).

Launch: ``python bench.py --gpus N`` spawns N ranks itself (one process per
GPU, started before anything touches the GPU, 127.0.0.1 rendezvous); under
torchrun (WORLD_SIZE set) each process is one rank.  The timed region is
bracketed by barrier + synchronize on both sides; the max over ranks is
reported.  ``--dry-run`` replaces the GPU work by a sleep and runs the
launcher + barrier + max-over-ranks path on gloo (CPU tests).
"""
from __future__ import annotations

import argparse
import ctypes
import hashlib
import json
import os
import socket
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBPS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
BPS = {"s8": 2, "u8": 2, "s16": 4, "f32": 8, "f32p": 8}
METRIC = "IQ Msamples/s + waterfall lines/s at 64k FFT; achieved HBM GB/s vs roofline"


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--mode", default="streams", choices=["streams", "shard"])
    p.add_argument("--calls-per-step", type=int, default=0,
                   help="rfa_process calls per step (0 = 250 for streams, 200 for shard: >= 0.5 s timed at 20 steps)")
    p.add_argument("--fft-size", type=int, default=0, help="0 = 65536 (streams) / 8192 (shard)")
    p.add_argument("--format", default="s8", choices=list(BPS))
    p.add_argument("--window", default="blackman")
    p.add_argument("--frames", type=int, default=0,
                   help="frames per call: 0 = 500 (streams: one full waterfall ring, FftProcessor.kt:103) / 256 (shard)")
    p.add_argument("--avg", default="ema", choices=["none", "ema", "boxcar"])
    p.add_argument("--ema-alpha", type=float, default=0.1)
    p.add_argument("--no-peak", action="store_true")
    p.add_argument("--ring-rows", type=int, default=500)
    p.add_argument("--state-cus", type=int, default=0,
                   help="streams mode: rfa_set_pipelined -- the peak / EMA pass on this many reserved CUs "
                        "under the next call's FFT (0 = serial on the handle stream)")
    p.add_argument("--gather", action="store_true", help="shard mode: gather every call's rows to rank 0")
    p.add_argument("--batches-per-call", type=int, default=64,
                   help="shard mode: batches per rfa_process_batches call (1 = one launch per batch)")
    p.add_argument("--pool-mib", type=int, default=768, help="input pool size (> Infinity Cache)")
    p.add_argument("--cpu-seconds", type=float, default=10.0, help="cpu_baseline time budget (0 = skip)")
    p.add_argument("--f32-steps", type=int, default=4, help="steps of the float32-input companion run (0 = skip)")
    p.add_argument("--c5-steps", type=int, default=3, help="steps of the 1 M-point (config 5) companion (0 = skip)")
    p.add_argument("--c2-steps", type=int, default=3, help="steps of the 16 K cf32 Hann (config 2) companion (0 = skip)")
    p.add_argument("--c4-steps", type=int, default=3, help="steps of the 256 x 8192 shard (config 4) companion (0 = skip)")
    p.add_argument("--demod-steps", type=int, default=5,
                   help="calls of the demod front-end companion (SURVEY §8(f) row 4; 0 = skip)")
    p.add_argument("--host-fed-calls", type=int, default=40,
                   help="calls of the host-fed companions (pinned host IQ, H2D overlapped; 0 = skip)")
    p.add_argument("--profile-every", type=int, default=8,
                   help="HIP-event timing of every K-th main-kernel launch in the timed region (1 = all)")
    p.add_argument("--traffic-file", default=os.path.join(ROOT, "profiles", "pmc_traffic.json"))
    p.add_argument("--dry-run", action="store_true", help="no GPU: launcher / barrier / timing path only (gloo)")
    a = p.parse_args(argv)
    if a.fft_size == 0:
        a.fft_size = 65536 if a.mode == "streams" else 8192
    if a.frames == 0:
        a.frames = 500 if a.mode == "streams" else 256
    if a.calls_per_step == 0:
        a.calls_per_step = 250 if a.mode == "streams" else max(1, 200 // max(1, a.batches_per_call))
    return a


# ----------------------------------------------------------------------------- launcher
def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(args, argv) -> int:
    """One child process per GPU (RANK/LOCAL_RANK/WORLD_SIZE/MASTER_* in its env).  The
    parent never touches the GPU; it waits for every rank and returns the worst code."""
    port = _free_port()
    procs = []
    for r in range(args.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus),
                   LOCAL_WORLD_SIZE=str(args.gpus), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv, env=env))
    rc = 0
    for i, p in enumerate(procs):
        code = p.wait()
        if code != 0 and rc == 0:
            rc = code
            for q in procs[i + 1:]:  # a failed rank would leave the others waiting at a barrier
                if q.poll() is None:
                    q.terminate()
    return rc


# ----------------------------------------------------------------------------- workload
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


class Ranks:
    """The process group (or a single process): barrier, max-over-ranks, gather."""

    def __init__(self, dry):
        import torch
        import torch.distributed as dist

        self.torch, self.dist = torch, dist
        self.rank = int(os.environ.get("RANK", "0"))
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.local = int(os.environ.get("LOCAL_RANK", "0"))
        self.dry = dry
        self.device = torch.device("cpu") if dry else torch.device("cuda", self.local)
        if self.world > 1:
            dist.init_process_group(backend="gloo" if dry else "nccl")

    def sync(self):
        if not self.dry:
            self.torch.cuda.synchronize()

    def barrier(self):
        if self.world > 1:
            self.dist.barrier()

    def all_values(self, x: float):
        """Every rank's value of x (rank order)."""
        if self.world <= 1:
            return [x]
        t = self.torch.tensor([x], device=self.device, dtype=self.torch.float64)
        parts = [self.torch.empty_like(t) for _ in range(self.world)]
        self.dist.all_gather(parts, t)
        return [float(p.item()) for p in parts]

    def close(self):
        if self.world > 1:
            self.dist.destroy_process_group()


def timed(ranks, step, steps, warmup):
    """W untimed steps, then EXACTLY `steps` steps between barrier + synchronize on
    both sides.  Returns (slowest rank's seconds, every rank's seconds)."""
    for k in range(warmup):
        step(k)
    ranks.sync()
    ranks.barrier()
    ranks.sync()
    t0 = time.perf_counter()
    for k in range(steps):
        step(warmup + k)
    ranks.sync()
    ranks.barrier()
    ranks.sync()
    el = time.perf_counter() - t0
    per = ranks.all_values(el)
    return max(per), per


def run_streams(args, ranks, fmt, steps, warmup, seed):
    """Config 3 per rank: one stream, B frames per call into ring + peak + EMA.
    Returns (slowest seconds, per-rank seconds, main-kernel ms per launch, kernel name)."""
    import rfanalyzer_amd

    torch = ranks.torch
    n, frames, calls = args.fft_size, args.frames, args.calls_per_step
    stream = torch.cuda.current_stream(ranks.device)
    eng = rfanalyzer_amd.SpectrumEngine(n, args.window, fmt, avg=args.avg, avg_length=min(30, args.ring_rows - 1),
                                        ema_alpha=args.ema_alpha, peak_hold=not args.no_peak,
                                        ring_rows=args.ring_rows, device=ranks.local)
    if args.state_cus:
        # pipelined state: a non-blocking stream (work on the HIP null stream would wait for the
        # CU-masked streams, which are blocking streams); the timed region still ends with a
        # device-wide synchronize, so every call's state pass is inside it
        stream = torch.cuda.Stream(ranks.device)
    eng.set_stream(stream.cuda_stream)
    if args.state_cus:
        eng.set_pipelined(args.state_cus)
    pool = make_pool(torch, n, frames, fmt, args.pool_mib, seed, ranks.device)
    eng.set_tuning(100_000_000, 20_000_000)
    ctr = [0]

    ptrs = [b.data_ptr() for b in pool]

    every, sampling = max(1, args.profile_every), [False]

    def step(_k):
        for _ in range(calls):  # rfa_process on the torch stream set above (no per-call Python stream lookup)
            if sampling[0] and ctr[0] % every == 0:  # events around a sample of the launches
                eng.set_profiling(True)
                eng.process_device(ptrs[ctr[0] % len(ptrs)], frames, 0, None)
                eng.set_profiling(False)
            else:
                eng.process_device(ptrs[ctr[0] % len(ptrs)], frames, 0, None)
            ctr[0] += 1

    for _ in range(warmup):  # untimed, before the kernel clock starts
        step(0)
    ms0, l0 = eng.kernel_time()
    sampling[0] = True
    slow, per = timed(ranks, step, steps, 0)
    sampling[0] = False
    ms1, l1 = eng.kernel_time()
    name = eng.main_kernel_name()
    eng.close()
    del pool
    return slow, per, (ms1 - ms0) / max(1, l1 - l0), name


def run_shard(args, ranks, steps, warmup):
    """Config 4: every batch of `frames` independent frames is split over the ranks
    (sharding.frame_range); a call enqueues `batches_per_call` consecutive batches of
    this rank's frames (rfa_process_batches, one launch); rows stay on each rank's
    device unless --gather.  Returns (slowest s, per-rank s, kernel ms, name, range, batches per call)."""
    import rfanalyzer_amd
    from rfanalyzer_amd import sharding

    torch = ranks.torch
    n, frames, fmt, calls = args.fft_size, args.frames, args.format, args.calls_per_step
    kb = max(1, args.batches_per_call)
    s, e = sharding.frame_range(frames, ranks.rank, ranks.world)
    mine = e - s
    stream = torch.cuda.current_stream(ranks.device)
    eng = rfanalyzer_amd.SpectrumEngine(n, args.window, fmt, ring_rows=0, device=ranks.local)
    eng.set_stream(stream.cuda_stream)
    # this rank's frame range of every batch, packed batch after batch (host-pinned in a
    # deployment; device-resident here so the timed region measures the GPU path)
    bb = max(1, mine) * n * BPS[fmt]
    src = make_pool(torch, n, frames, fmt, args.pool_mib, 4, ranks.device)
    # at least the pool size of the other modes (past the Infinity Cache), a whole number of calls
    count = max(len(src), -(-args.pool_mib * 2 ** 20 // bb))
    count = -(-count // kb) * kb
    pool = torch.empty(count * bb, dtype=torch.uint8, device=ranks.device)
    for b in range(count):
        pool[b * bb:b * bb + mine * n * BPS[fmt]].copy_(src[b % len(src)].view(torch.uint8)[s * n * BPS[fmt]:e * n * BPS[fmt]])
    del src
    rows = torch.empty(kb * max(1, mine) * n, dtype=torch.float32, device=ranks.device)
    gathered = None
    if args.gather and ranks.world > 1:
        gathered = [torch.empty(kb * ((frames + ranks.world - 1) // ranks.world) * n, dtype=torch.float32,
                                device=ranks.device) for _ in range(ranks.world)]
        padded = torch.zeros_like(gathered[0])
    ctr = [0]
    base, rows_ptr = pool.data_ptr(), rows.data_ptr()
    every, sampling = max(1, args.profile_every), [False]

    def step(_k):
        for _ in range(calls):
            if mine:
                prof = sampling[0] and ctr[0] % every == 0
                if prof:
                    eng.set_profiling(True)
                b0 = (ctr[0] * kb) % count
                eng.process_batches(base + b0 * bb, kb, bb, mine, 0, rows_ptr)
                if prof:
                    eng.set_profiling(False)
            if gathered is not None:
                padded[:kb * mine * n].copy_(rows[:kb * mine * n])
                ranks.dist.all_gather(gathered, padded)
            ctr[0] += 1

    for _ in range(warmup):
        step(0)
    ms0, l0 = eng.kernel_time()
    sampling[0] = True
    slow, per = timed(ranks, step, steps, 0)
    sampling[0] = False
    ms1, l1 = eng.kernel_time()
    name = eng.main_kernel_name()
    eng.close()
    return slow, per, (ms1 - ms0) / max(1, l1 - l0), name, (s, e), kb


# ----------------------------------------------------------------------------- companions
def copy_ceiling(torch, device, mib=1024, iters=20):
    """Device stream-copy ceiling in the same run (SURVEY.md §8(d) primary denominator):
    librfa's float4 copy kernel (rfa_stream_copy) over two 1 GiB buffers, 2 x bytes / time."""
    from rfanalyzer_amd import _lib

    L = _lib.lib()
    src = torch.empty(mib * 2 ** 20 // 4, dtype=torch.float32, device=device).fill_(1.0)
    dst = torch.empty_like(src)
    st = torch.cuda.current_stream(device)
    nb = src.numel() * 4
    _lib.check(L.rfa_stream_copy(dst.data_ptr(), src.data_ptr(), nb, st.cuda_stream), "rfa_stream_copy")
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(iters):
        L.rfa_stream_copy(dst.data_ptr(), src.data_ptr(), nb, st.cuda_stream)
    e1.record(st)
    torch.cuda.synchronize()
    ok = bool(torch.equal(dst[:1024], src[:1024]))
    gbps = 2 * nb * iters / (e0.elapsed_time(e1) * 1e-3) / 1e9
    del src, dst
    return round(gbps, 1), ok


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


def host_fed_run(torch, device, n, fmt, frames, calls, window="blackman", avg="ema", peak=True, ring_rows=500,
                 host_batches=2, seed=7, state_out=False):
    """Host-fed end to end (SURVEY.md §7 "Host feed vs device throughput"; the reference path
    is host-fed by construction: FileIQSource.java:318-369 -> Scheduler.kt:252-279 ->
    FftProcessor.kt:111-140).  The raw IQ batches sit in pinned host memory; each call's batch
    is copied H2D on a second stream into one of two device buffers (double buffering: the
    copy of batch i+1 runs while batch i is processed), then rfa_process() reads it into the
    device ring + peak / EMA state only (no rows back).  Returns wall-clock Msamples/s over
    `calls` calls, the H2D-only rate of the same copies, and the per-call split (state_out: also
    the engine's peaks / EMA after the run, for tests/test_host_feed.py)."""
    import rfanalyzer_amd

    st = torch.cuda.current_stream(device)
    cp = torch.cuda.Stream(device)
    eng = rfanalyzer_amd.SpectrumEngine(n, window, fmt, avg=avg, avg_length=min(30, ring_rows - 1), ema_alpha=0.1,
                                        peak_hold=peak, ring_rows=ring_rows, device=device.index or 0)
    eng.set_stream(st.cuda_stream)
    eng.set_tuning(100_000_000, 20_000_000)
    src = make_pool(torch, n, frames, fmt, 1, seed, device)[:host_batches]  # synthetic batches, made on device
    host = [b.view(torch.uint8).cpu().pin_memory() for b in src]
    del src
    nbytes = host[0].numel()
    dev = [torch.empty(nbytes, dtype=torch.uint8, device=device) for _ in range(2)]
    ready = [torch.cuda.Event() for _ in range(2)]
    done = [torch.cuda.Event() for _ in range(2)]
    for e in done:
        e.record(st)

    def run(k_calls, process=True):
        for i in range(k_calls):
            j = i & 1
            with torch.cuda.stream(cp):
                cp.wait_event(done[j])  # the batch that last used this buffer has been read
                dev[j].copy_(host[i % len(host)], non_blocking=True)
                ready[j].record(cp)
            if process:
                st.wait_event(ready[j])
                eng.process_device(dev[j].data_ptr(), frames, 0, None)
                done[j].record(st)
            else:
                done[j].record(cp)

    run(4)
    torch.cuda.synchronize(device)
    t0 = time.perf_counter()
    run(calls)
    torch.cuda.synchronize(device)
    el = time.perf_counter() - t0
    t0 = time.perf_counter()
    run(calls, process=False)
    torch.cuda.synchronize(device)
    el_copy = time.perf_counter() - t0
    state = {"peaks": eng.peaks(), "ema": eng.ema()} if state_out else {}
    eng.close()
    samples = calls * frames * n
    return {"value": round(samples / el / 1e6, 2), "unit": "Msamples/s", "ms_per_call": round(el / calls * 1e3, 4),
            "h2d_GBps": round(calls * nbytes / el_copy / 1e9, 2),
            "h2d_only_ms_per_call": round(el_copy / calls * 1e3, 4), "bytes_per_call": nbytes,
            "frames_per_call": frames, "calls": calls, **state}


def c_call_cost(calls=4000):
    """tools/call_bench (built by __graft_entry__.build()): the C-ABI's per-call cost for
    config 4's 256 x 8192 s8 batches timed from a C loop (no Python / ctypes), one batch per
    rfa_process_batches call and 64 per call.  None when the binary is absent."""
    exe = os.path.join(ROOT, "tools", "call_bench")
    if not os.path.exists(exe):
        return None
    out = {}
    for kb in (1, 64):
        r = subprocess.run([exe, str(calls if kb == 1 else max(1, calls // 64)), str(kb)], capture_output=True,
                           text=True, timeout=300)
        if r.returncode != 0:
            out[f"batches_per_call_{kb}"] = {"error": (r.stderr or r.stdout)[-300:]}
            continue
        out[f"batches_per_call_{kb}"] = json.loads(r.stdout.strip().splitlines()[-1])
    return out


def pmc_traffic(args, fmt, n, frames):
    """roofline.traffic: HBM bytes per launch from the rocprofv3 PMC passes of the
    committed profile, used only when they were measured on this exact librfa.so."""
    from rfanalyzer_amd import _lib

    try:
        with open(args.traffic_file) as fh:
            tr = json.load(fh)
    except (OSError, ValueError):
        return None, "no PMC record"
    rec = tr.get(f"{fmt}_{n}_{frames}")
    if not rec:
        return None, "no PMC record for this workload"
    with open(_lib.LIB_PATH, "rb") as fh:
        sha = hashlib.sha256(fh.read()).hexdigest()[:16]
    if rec.get("librfa_sha16") != sha:
        return None, f"PMC record is for another build ({rec.get('librfa_sha16')}, this {sha})"
    return rec["hbm_bytes_per_launch"], f"{rec.get('source', args.traffic_file)} (librfa {sha})"


def sq_valu(args, fmt, n, frames):
    """roofline.valu: VALU busy fraction of the main kernel from the committed SQ-counter
    record (SURVEY §8(d) asks for VALU busy %), used only for this exact librfa.so."""
    from rfanalyzer_amd import _lib

    try:
        with open(os.path.join(os.path.dirname(args.traffic_file), "sq_valu.json")) as fh:
            rec = json.load(fh).get(f"{fmt}_{n}_{frames}")
    except (OSError, ValueError):
        return None
    if not rec:
        return None
    with open(_lib.LIB_PATH, "rb") as fh:
        sha = hashlib.sha256(fh.read()).hexdigest()[:16]
    if rec.get("librfa_sha16") != sha:
        return {"busy_frac": None, "source": f"SQ record is for another build ({rec.get('librfa_sha16')}, this {sha})"}
    return {"busy_frac": rec["valu_busy_frac"], "wave_wait_frac": rec["wave_wait_frac"],
            "source": f"{rec['source']} (librfa {sha})"}


# ----------------------------------------------------------------------------- cpu baseline
def _synthetic_frames(n, frames, fmt, seed=3):
    import numpy as np
    rng = np.random.Generator(np.random.PCG64(seed))
    t = np.arange(n * frames)
    x = 0.5 * np.exp(2j * np.pi * 0.07 * t) + 0.05 * (rng.standard_normal(t.size) + 1j * rng.standard_normal(t.size))
    iq = np.empty(2 * t.size)
    iq[0::2], iq[1::2] = x.real, x.imag
    if fmt == 0:
        return np.clip(np.rint(iq * 128), -128, 127).astype(np.int8)
    return iq.astype(np.float32)


def host_info():
    """The host the CPU baseline ran on: model, online CPUs, the CPUs this process may
    use (affinity) and the cgroup CPU quota, if any."""
    info = {"nproc": os.cpu_count()}
    try:
        info["affinity_cpus"] = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        info["affinity_cpus"] = os.cpu_count()
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    info["cpu_model"] = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        with open("/sys/fs/cgroup/cpu.max") as fh:
            q, per = fh.read().split()
            info["cgroup_cpu_quota"] = None if q == "max" else round(int(q) / int(per), 2)
    except (OSError, ValueError):
        pass
    return info


def cpu_baseline(args, n, seconds):
    """Reference loop (pffft + restated JVM loops, oracle/_ref) on host cores, bounded time:
    one thread (the reference runs one FftProcessor thread) and then every CPU this
    process may run on (os.sched_getaffinity), one independent loop per thread."""
    import numpy as np

    import oracle

    hinfo = host_info()
    # every CPU this process may use: the affinity mask, bounded by the cgroup CPU quota
    # when one is set (more threads than the quota only time-slice the same CPUs)
    cpus = hinfo.get("affinity_cpus") or 1
    quota = hinfo.get("cgroup_cpu_quota")
    threads = max(1, min(256, cpus, int(quota) if quota else cpus))

    fmt = {"s8": 0, "f32": 3}.get(args.format, 0)
    frames = max(1, (8 * 2 ** 20) // (n * 8))  # ~8 MB sample, processed repeatedly
    data = _synthetic_frames(n, frames, fmt)
    w = oracle.window(n, oracle.WIN_BLACKMAN)
    ring_rows = 500
    fp = ctypes.POINTER(ctypes.c_float)

    def run_ref(budget, ring_rows=ring_rows):
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
           "lines_per_s": round(done / el, 2), "host": hinfo}
    if kind == "reference" and threads > 1:
        # frame-parallel on the host's cores: one independent loop per thread;
        # ctypes releases the GIL for the duration of each ref_loop call
        import threading

        # each thread writes its own 64-row ring (the per-frame ring copy is the same for any
        # ring length; 500 rows x 64 K x 4 B per thread would not fit hundreds of threads)
        res = [None] * threads
        ths = [threading.Thread(target=lambda i=i: res.__setitem__(i, run_ref(seconds / 2, 64)))
               for i in range(threads)]
        for t in ths:
            t.start()
        for t in ths:
            t.join()
        el = max(r[1] for r in res)
        out["multi_core"] = {"value": round(sum(r[0] for r in res) * n / el / 1e6, 3), "cores": threads,
                             "sample": f"{threads} threads (every CPU this process may use: affinity mask "
                                       f"{cpus}, cgroup quota {quota}) x the same loop for {el:.1f} s"}
    return out


def config1_replay(device_ok: bool):
    """BASELINE config 1: FileIQSource replay of a 1 s 8-bit
    capture (HackRF s8, 2 Msps, 4 000 000 B, seed 1: tone at +250 kHz, 0.5 FS, AWGN
    sigma 0.05), N = 1024, no averaging -- host plumbing.  The reference path (packet
    read FileIQSource.java:318-369, framing Scheduler.kt:252-279, LUT + Blackman +
    pffft + log-mag + ring, oracle/_ref) and the same replay through librfa
    (rfa_process_host per packet: PCIe + launch latency) both per frame."""
    import numpy as np

    import oracle
    from rfanalyzer_amd import source

    n, sr, nbytes = 1024, 2_000_000, 4_000_000
    rng = np.random.Generator(np.random.PCG64(1))
    t = np.arange(nbytes // 2)
    x = 0.5 * np.exp(2j * np.pi * 250_000 / sr * t) + 0.05 * (rng.standard_normal(t.size) +
                                                             1j * rng.standard_normal(t.size))
    iq = np.empty(2 * t.size)
    iq[0::2], iq[1::2] = x.real, x.imag
    raw = np.clip(np.rint(iq * 128), -128, 127).astype(np.int8)
    out = {"workload": "config1: FileIQSource replay, 1 s s8 2 Msps capture, 1024-pt FFT, no averaging"}
    with tempfile.TemporaryDirectory() as d:
        path = os.path.join(d, "capture_s8_2msps.iq")
        raw.tofile(path)

        def replay(per_frame):
            src = source.FileIQSource()
            src.init(path, sr, 100_000_000, repeat=False)
            assert src.open()
            frames, t0 = 0, time.perf_counter()
            while True:
                try:
                    pkt = src.getPacket()
                except (EOFError, IOError, OSError):
                    break
                if pkt is None:
                    break
                per_frame(np.frombuffer(bytes(pkt), np.int8)[:2 * n])
                frames += 1
            el = time.perf_counter() - t0
            src.close()
            return frames, el

        if oracle.ref_available():
            lib = oracle.ref()
            w = oracle.window(n, oracle.WIN_BLACKMAN)
            ring = np.full((400, n), -9999, np.float32)
            peaks = np.full(n, -999999, np.float32)
            fp = ctypes.POINTER(ctypes.c_float)

            def ref_frame(fr):
                fr = np.ascontiguousarray(fr)
                assert lib.ref_loop(fr.ctypes.data, 0, n, 1, 2 * n, w.ctypes.data_as(fp), ring.ctypes.data_as(fp),
                                    400, peaks.ctypes.data_as(fp)) == 0

            frames, el = replay(ref_frame)
            out["reference"] = {"frames": frames, "us_per_frame": round(el / max(frames, 1) * 1e6, 2), "cores": 1,
                                "kind": "reference"}
        if device_ok:
            import rfanalyzer_amd
            eng = rfanalyzer_amd.SpectrumEngine(n, "blackman", "s8", ring_rows=400)
            eng.set_tuning(100_000_000, sr)
            frames, el = replay(lambda fr: eng.process(fr.tobytes(), 1, rows=True))
            eng.close()
            out["librfa_host_buffers"] = {"frames": frames, "us_per_frame": round(el / max(frames, 1) * 1e6, 2),
                                          "note": "rfa_process_host per packet: launch + PCIe latency bound"}
    return out


# ----------------------------------------------------------------------------- main
def main():
    argv = sys.argv[1:]
    args = parse(argv)
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        sys.exit(launch_ranks(args, argv))
    if env_world is not None and int(env_world) != args.gpus:
        sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={env_world}")
    ranks = Ranks(args.dry_run)
    torch = ranks.torch
    if not args.dry_run:
        torch.cuda.set_device(ranks.local)
        # a real stream shared by torch and librfa (not the null stream)
        torch.cuda.set_stream(torch.cuda.Stream(ranks.device))

    n, frames, fmt, calls = args.fft_size, args.frames, args.format, args.calls_per_step
    result = {"metric": METRIC}
    kb = 1
    if args.dry_run:
        slow, per = timed(ranks, lambda k: time.sleep(0.001 * (1 + ranks.rank)), args.steps, args.warmup)
        kernel_ms, kernel_name, span = 0.0, "dry-run", None
        mine = frames
    elif args.mode == "streams":
        slow, per, kernel_ms, kernel_name = run_streams(args, ranks, fmt, args.steps, args.warmup, 3 + ranks.rank)
        mine = frames
    else:
        slow, per, kernel_ms, kernel_name, span, kb = run_shard(args, ranks, args.steps, args.warmup)
        mine = (span[1] - span[0]) * kb

    batches = kb if args.mode == "shard" else 1
    total_frames = (ranks.world if args.mode == "streams" else 1) * frames * batches * calls * args.steps
    samples = total_frames * n
    msps = samples / slow / 1e6
    s_in = BPS[fmt]
    alg_bytes = mine * n * (s_in + 4)  # per main-kernel launch: raw IQ in + one fp32 row value out
    achieved = alg_bytes / (kernel_ms * 1e-3) / 1e9 if kernel_ms > 0 else 0.0
    result.update({
        "value": round(msps, 2),
        "unit": "Msamples/s",
        "n_gpus": ranks.world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(slow * 1e3 / args.steps, 4),
        "higher_is_better": True,
        "scaling": "weak" if args.mode == "streams" else "strong",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic" if not args.dry_run else "none (dry run)",
        "lines_per_s": round(total_frames / slow, 1),
        "per_rank_s": [round(x, 6) for x in per],
    })
    if args.mode == "streams":
        workload = (f"config3: {n}-pt FFT, {args.window} window, {fmt} IQ, "
                    f"{'EMA' if args.avg == 'ema' else args.avg} + {'peak-hold' if not args.no_peak else 'no peak'}, "
                    f"ring {args.ring_rows} rows, one stream per GPU")
    else:
        workload = (f"config4: batches of {frames} frames x {n}-pt FFT, {args.window}, {fmt} IQ, frames sharded "
                    f"over {ranks.world} GPU(s) (contiguous ranges), {kb} batches per rfa_process_batches call"
                    f"{', rows gathered to rank 0' if args.gather else ''}")
    result["config"] = {"workload": workload, "fft_size": n, "frames_per_call": frames * batches,
                        "calls_per_step": calls, "input_format": fmt, "parallelism": f"{args.mode}{ranks.world}"}
    if args.mode == "streams":
        result["config"].update({"avg": args.avg, "ema_alpha": args.ema_alpha, "peak_hold": not args.no_peak,
                                 "ring_rows": args.ring_rows})
    else:
        result["config"]["frames_per_batch"] = frames
    result["roofline"] = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                          "frac": round(achieved / HBM_PEAK_GBPS, 4), "traffic": None,
                          "kernel": kernel_name, "kernel_ms": round(kernel_ms, 4),
                          "alg_bytes_per_launch": alg_bytes,
                          "timing": f"HIP events on the handle stream around every {max(1, args.profile_every)}-th "
                                    "main-kernel launch of the timed region"}
    single = ranks.rank == 0 and ranks.world == 1 and not args.dry_run
    if single:
        tr, src = pmc_traffic(args, fmt, n, mine)
        result["roofline"]["traffic"] = tr
        result["roofline"]["traffic_source"] = src
        va = sq_valu(args, fmt, n, mine)
        if va is not None:
            result["roofline"]["valu"] = va
    if ranks.rank == 0 and not args.dry_run:
        gbps, ok = copy_ceiling(torch, ranks.device)
        result["roofline"]["copy_GBps"] = gbps
        result["roofline"]["copy_kernel"] = "rfa_stream_copy (librfa float4 copy)" + ("" if ok else " MISMATCH")
        result["roofline"]["frac_of_copy"] = round(achieved / gbps, 4)
        if args.mode == "streams":
            # step level: every byte the step must move (raw in, ring row out, EMA + peak read+write) / step time
            step_bytes = frames * n * (s_in + 4) + 16 * n
            result["roofline"]["step_frac"] = round(step_bytes * calls * args.steps / slow / 1e9 / HBM_PEAK_GBPS, 4)
    if args.mode == "streams":
        companions(args, ranks, result)
    if ranks.rank == 0 and ranks.world == 1 and args.cpu_seconds > 0 and args.mode == "streams":
        result["cpu_baseline"] = cpu_baseline(args, n, args.cpu_seconds)
        result["cpu_baseline"]["config1"] = config1_replay(not args.dry_run)
    if ranks.rank == 0:
        print(json.dumps(result), flush=True)
    ranks.close()


def _stream_companion(args, ranks, steps, seed, **over):
    """One run_streams workload with some settings replaced; every rank takes part."""
    import copy
    a = copy.copy(args)
    for k, v in over.items():
        setattr(a, k, v)
    fmt = over.get("format", args.format)
    if args.dry_run:
        slow, per = timed(ranks, lambda k: time.sleep(0.0005 * (1 + ranks.rank)), steps, 1)
        return a, slow, per, 0.0, "dry-run"
    slow, per, k, name = run_streams(a, ranks, fmt, steps, 1, seed)
    return a, slow, per, k, name


def _roof(alg, k_ms):
    gbps = alg / (k_ms * 1e-3) / 1e9 if k_ms > 0 else 0.0
    return {"roofline_achieved_GBps": round(gbps, 1), "roofline_frac": round(gbps / HBM_PEAK_GBPS, 4),
            "alg_bytes_per_launch": alg}


def companions(args, ranks, result):
    """Other BASELINE configs beside the headline (never `value`).  In multi-GPU runs every
    rank runs them (streams: one per rank, weak; config 4: the batch split, strong) and the
    per-rank seconds are reported; values are whole-job Msamples/s."""
    W = ranks.world
    fmt, n = args.format, args.fft_size
    if fmt != "f32" and args.f32_steps > 0:
        # BASELINE.json asks for 8-bit AND float32 IQ: the headline workload on complex-float32
        # input (12 B/sample algorithmic)
        a, el, per, k, _ = _stream_companion(args, ranks, args.f32_steps, 103 + ranks.rank, format="f32")
        result["f32"] = {"value": round(W * args.f32_steps * a.calls_per_step * a.frames * n / el / 1e6, 2),
                         "unit": "Msamples/s", "ms_per_step": round(el * 1e3 / args.f32_steps, 4),
                         "kernel_ms": round(k, 4), "per_rank_s": [round(x, 6) for x in per],
                         **_roof(a.frames * n * (BPS["f32"] + 4), k)}
    if args.c2_steps > 0:
        # config 2: synthetic 20 Msps complex-float32 IQ, 16384-pt Hann, waterfall ring, no averaging
        a, el, per, k, name = _stream_companion(args, ranks, args.c2_steps, 303 + ranks.rank, format="f32",
                                                fft_size=16384, window="hann", frames=4096, calls_per_step=30,
                                                avg="none", no_peak=True)
        result["config2"] = {"workload": "config2 per GPU: 16384-pt Hann FFT, cf32 IQ (20 Msps), ring 500 rows, "
                                         "4096 frames per call, no averaging",
                             "value": round(W * args.c2_steps * a.calls_per_step * a.frames * a.fft_size / el / 1e6, 2),
                             "unit": "Msamples/s", "ms_per_step": round(el * 1e3 / args.c2_steps, 4),
                             "kernel_ms": round(k, 4), "kernel": name, "per_rank_s": [round(x, 6) for x in per],
                             **_roof(a.frames * a.fft_size * (BPS["f32"] + 4), k)}
        # real-time headroom = Msamples/s per stream / the source rate
        result["config2"]["realtime_headroom"] = round(result["config2"]["value"] / W / 20.0, 1)
    if args.c4_steps > 0:
        import copy
        a4 = copy.copy(args)
        a4.mode, a4.fft_size, a4.frames, a4.format = "shard", 8192, 256, fmt if fmt in ("s8", "u8") else "s8"
        a4.calls_per_step, a4.batches_per_call, a4.gather = 10, 64, False
        if args.dry_run:
            el, per = timed(ranks, lambda k: time.sleep(0.0005 * (1 + ranks.rank)), args.c4_steps, 1)
            k4, name4, mine = 0.0, "dry-run", 256 // W
        else:
            el, per, k4, name4, span, _ = run_shard(a4, ranks, args.c4_steps, 1)
            mine = span[1] - span[0]
        total = args.c4_steps * a4.calls_per_step * a4.batches_per_call * a4.frames * a4.fft_size
        nb = args.c4_steps * a4.calls_per_step * a4.batches_per_call
        result["config4"] = {"workload": f"config4: batches of 256 x 8192-pt {a4.format} frames sharded over {W} "
                                         f"GPU(s), {a4.batches_per_call} batches per rfa_process_batches call",
                             "value": round(total / el / 1e6, 2), "unit": "Msamples/s", "scaling": "strong",
                             "us_per_batch": round(el / nb * 1e6, 3), "us_per_batch_amortised_over": a4.batches_per_call,
                             "kernel_ms": round(k4, 4), "kernel": name4,
                             "per_rank_s": [round(x, 6) for x in per],
                             **_roof(a4.batches_per_call * mine * a4.fft_size * (BPS[a4.format] + 4), k4)}
        # the same batches one rfa_process_batches call each (per-batch latency, comparable with
        # one-batch-per-call records): launch-bound at 256 frames
        a1 = copy.copy(a4)
        a1.batches_per_call = 1
        if args.dry_run:
            el1, _ = timed(ranks, lambda k: time.sleep(0.0005 * (1 + ranks.rank)), args.c4_steps, 1)
        else:
            el1, _, _, _, _, _ = run_shard(a1, ranks, args.c4_steps, 1)
        nb1 = args.c4_steps * a1.calls_per_step
        result["config4"]["one_batch_per_call"] = {
            "us_per_batch": round(el1 / nb1 * 1e6, 3),
            "value": round(nb1 * a1.frames * a1.fft_size / el1 / 1e6, 2), "unit": "Msamples/s"}
        # SURVEY §8(d) config 4 names f32 and s8: the same batches on complex-float32 input
        a4.format = "f32"
        if args.dry_run:
            el, per = timed(ranks, lambda k: time.sleep(0.0005 * (1 + ranks.rank)), args.c4_steps, 1)
            k4, name4 = 0.0, "dry-run"
        else:
            el, per, k4, name4, span, _ = run_shard(a4, ranks, args.c4_steps, 1)
            mine = span[1] - span[0]
        result["config4_f32"] = {"workload": f"config4 on cf32 IQ: batches of 256 x 8192-pt frames sharded over {W} "
                                             f"GPU(s), {a4.batches_per_call} batches per rfa_process_batches call",
                                 "value": round(total / el / 1e6, 2), "unit": "Msamples/s", "scaling": "strong",
                                 "us_per_batch": round(el / nb * 1e6, 3), "kernel_ms": round(k4, 4), "kernel": name4,
                                 "per_rank_s": [round(x, 6) for x in per],
                                 **_roof(a4.batches_per_call * mine * a4.fft_size * (BPS["f32"] + 4), k4)}
    if n != (1 << 20) and args.c5_steps > 0:
        # config 5: one independent 1 M-point stream per GPU, same stateful settings
        a, el, per, k, name = _stream_companion(args, ranks, args.c5_steps, 203 + ranks.rank, fft_size=1 << 20,
                                                frames=16, calls_per_step=30)
        result["config5"] = {"workload": f"config5 per GPU: 1048576-pt FFT, {args.window}, {fmt} IQ, "
                                         f"{'EMA' if args.avg == 'ema' else args.avg} + peak-hold, ring "
                                         f"{args.ring_rows} rows, 16 frames per call, one stream per GPU",
                             "value": round(W * args.c5_steps * a.calls_per_step * a.frames * a.fft_size / el / 1e6, 2),
                             "unit": "Msamples/s", "scaling": "weak", "ms_per_step": round(el * 1e3 / args.c5_steps, 4),
                             "kernel_ms": round(k, 4), "kernel": name, "per_rank_s": [round(x, 6) for x in per],
                             **_roof(a.frames * a.fft_size * (BPS[fmt] + 4), k),
                             "note": "kernel_ms = the whole large-N launch (front kernel + 32 K kernel B)"}
        result["config5"]["realtime_headroom"] = round(result["config5"]["value"] / W / 250.0, 1)  # 250 Msps streams
    if args.host_fed_calls > 0 and not args.dry_run:
        # the headline is device-resident; the host-fed end-to-end rate is reported
        # beside it (never `value`).  Every rank feeds its own GPU over its own PCIe link.
        torch = ranks.torch
        hf3 = host_fed_run(torch, ranks.device, n, fmt, args.frames, args.host_fed_calls, window=args.window,
                           avg=args.avg, peak=not args.no_peak, ring_rows=args.ring_rows)
        hf2 = host_fed_run(torch, ranks.device, 16384, "f32", 1024, max(4, args.host_fed_calls // 2), window="hann",
                           avg="none", peak=False, ring_rows=500)
        v3, v2 = ranks.all_values(hf3["value"]), ranks.all_values(hf2["value"])
        result["host_fed"] = {
            "note": "pinned host IQ -> H2D on a second stream (double-buffered, overlapped with the previous "
                    "batch's kernels) -> rfa_process into the device ring + state, no rows back; wall clock; "
                    "PCIe-bound, never `value`",
            "config3": dict(hf3, workload=f"config3 host-fed: {n}-pt {args.window}, {fmt} IQ, {args.avg} + peak-hold, "
                                          f"ring {args.ring_rows}, {args.frames} frames per call",
                            value=round(sum(v3), 2), per_rank_value=v3,
                            device_resident_ratio=round(result.get("value", 0) / max(sum(v3), 1e-9), 2)
                            if "value" in result else None),
            "config2": dict(hf2, workload="config2 host-fed: 16384-pt Hann, cf32 IQ, ring 500, 1024 frames per call",
                            value=round(sum(v2), 2), per_rank_value=v2,
                            realtime_headroom_vs_20msps=round(min(v2) / 20.0, 1))}
    if ranks.rank == 0 and ranks.world == 1 and args.c4_steps > 0 and not args.dry_run and "config4" in result:
        result["config4"]["one_batch_per_call"]["c_loop"] = c_call_cost()
    if ranks.rank == 0 and args.demod_steps > 0 and not args.dry_run:
        result["demod"] = demod_companion(ranks.torch, ranks.device, args.demod_steps)


if __name__ == "__main__":
    main()
