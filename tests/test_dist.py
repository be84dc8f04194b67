"""CPU, world_size 2 over gloo: the multi-GPU layout of SURVEY.md §8(e) --
frames of a batch sharded into contiguous per-rank ranges with no data-path
collective; per-rank peak/EMA segment summaries folded on the host reproduce
the single-stream sequential state; bench.py's max-over-ranks timing.
The per-rank spectrum rows come from the oracle here (no GPU in this test)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

import oracle
import signals
from oracle import processor
from rfanalyzer_amd import sharding

N, FRAMES, ALPHA = 512, 37, 0.2


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _data():
    raw = np.frombuffer(signals.frames_bytes(N, FRAMES, "s8", 21, tones=((0.11, 0.4),), noise=0.05), np.int8).copy()
    raw[7 * 2 * N:8 * 2 * N] = 0  # one silent frame: -inf bins restart the EMA
    return raw.tobytes()


def _worker(rank, world, port, q):
    import torch
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), LOCAL_RANK=str(rank),
                      WORLD_SIZE=str(world))
    import bench

    ranks = bench.Ranks(dry=True)  # bench.py's process group (gloo here, RCCL on GPUs)
    try:

        data = _data()
        s, e = sharding.frame_range(FRAMES, rank, world)
        rows = oracle.spectrum_rows(data[s * 2 * N:e * 2 * N], oracle.IN_S8, N, e - s, None, oracle.WIN_BLACKMAN)
        decay, b, fresh = sharding.ema_partial(rows, ALPHA)
        mine = torch.from_numpy(np.stack([rows.max(0), decay, b, fresh]).astype(np.float32))
        parts = [torch.empty_like(mine) for _ in range(world)]
        dist.all_gather(parts, mine)  # host-side state hand-off (test only; the bench has none)
        slowest = max(ranks.all_values(float(rank + 1)))  # bench.py's max-over-ranks timing
        if rank == 0:
            pk = sharding.peak_combine([p[0].numpy() for p in parts])
            em = sharding.ema_combine(None, [(p[1].numpy(), p[2].numpy(), p[3].numpy()) for p in parts])
            q.put((pk, em, slowest))
    finally:
        ranks.close()


@pytest.mark.parametrize("world", [2])
def test_sharded_frames_reproduce_single_stream_state(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    pk, em, slowest = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ref_rows = oracle.spectrum_rows(_data(), oracle.IN_S8, N, FRAMES, None, oracle.WIN_BLACKMAN)
    np.testing.assert_array_equal(pk, ref_rows.max(0))
    exp = processor.ema_batch(ref_rows, ALPHA)
    assert np.array_equal(np.isneginf(em), np.isneginf(exp))
    fin = np.isfinite(exp)
    np.testing.assert_allclose(em[fin], exp[fin], rtol=0, atol=1e-4)
    assert slowest == float(world)
