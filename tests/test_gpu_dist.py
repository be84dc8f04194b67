"""GPU, two processes: the sharded-batch layout of SURVEY.md §8(e) config 4 run
through the product.  Each rank owns a contiguous frame range of one batch
(sharding.frame_range), runs its own SpectrumEngine (librfa) on it, and the rows
are gathered over the process group (gloo here: both ranks share the one GPU of
the test box; RCCL between GPUs in bench.py).  The gathered rows equal the
single-process rows bit for bit (frames are independent and the kernel is
deterministic), and the per-rank peak / EMA segment summaries folded on the host
equal the single-process device state."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

import signals

pytestmark = pytest.mark.gpu

N, FRAMES, ALPHA = 8192, 256, 0.2  # config 4: a batch of 256 frames x 8192 points


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _data():
    raw = np.frombuffer(signals.frames_bytes(N, FRAMES, "s8", 44, tones=((0.11, 0.4), (-0.3, 0.01)), noise=0.05),
                        np.int8).copy()
    raw[9 * 2 * N:10 * 2 * N] = 0  # a silent frame: -inf bins restart the EMA
    return raw.tobytes()


def _worker(rank, world, port, q):
    import torch
    import torch.distributed as dist

    import rfanalyzer_amd
    from rfanalyzer_amd import sharding

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        data = _data()
        s, e = sharding.frame_range(FRAMES, rank, world)
        with rfanalyzer_amd.SpectrumEngine(N, "blackman", "s8", ring_rows=0) as eng:
            rows = eng.process(data[s * 2 * N:e * 2 * N], e - s)
        decay, b, fresh = sharding.ema_partial(rows, ALPHA)
        per = (FRAMES + world - 1) // world
        mine = np.full((per, N), np.nan, np.float32)
        mine[:e - s] = rows
        parts = [torch.empty(per, N) for _ in range(world)]
        dist.all_gather(parts, torch.from_numpy(mine))
        summ = torch.from_numpy(np.stack([rows.max(0), decay, b, fresh]).astype(np.float32))
        sparts = [torch.empty_like(summ) for _ in range(world)]
        dist.all_gather(sparts, summ)
        if rank == 0:
            got = np.concatenate([p.numpy()[:sharding.frame_range(FRAMES, r, world)[1] -
                                             sharding.frame_range(FRAMES, r, world)[0]]
                                  for r, p in enumerate(parts)])
            pk = sharding.peak_combine([p[0].numpy() for p in sparts])
            em = sharding.ema_combine(None, [(p[1].numpy(), p[2].numpy(), p[3].numpy()) for p in sparts])
            q.put((got, pk, em))
    finally:
        dist.destroy_process_group()


def test_two_ranks_shard_a_batch_through_librfa(rfa):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got, pk, em = q.get(timeout=100)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    with rfa.SpectrumEngine(N, "blackman", "s8", avg="ema", ema_alpha=ALPHA, peak_hold=True, ring_rows=0) as eng:
        eng.set_tuning(100_000_000, 20_000_000)
        ref = eng.process(_data(), FRAMES)
        ref_pk, ref_em = eng.peaks(), eng.ema()
    np.testing.assert_array_equal(got.view(np.int32), ref.view(np.int32))
    np.testing.assert_array_equal(pk, ref_pk)
    assert np.array_equal(np.isneginf(em), np.isneginf(ref_em))
    fin = np.isfinite(ref_em)
    np.testing.assert_allclose(em[fin], ref_em[fin], rtol=0, atol=1e-4)
