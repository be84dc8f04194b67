"""CPU: bench.py's multi-GPU launcher without a GPU.

``python bench.py --gpus 2 --dry-run`` spawns two ranks itself (one process per
GPU in a real run), they rendezvous on 127.0.0.1 over gloo, time the same number
of steps between barriers and rank 0 reports the slowest rank -- the path the
driver's ``--gpus N`` runs take, with the GPU work replaced by a sleep."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(*args, env=None):
    e = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    e.update(env or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], capture_output=True, text=True,
                          timeout=240, env=e, cwd=ROOT)


@pytest.mark.parametrize("mode", ["streams", "shard"])
def test_gpus_2_spawns_two_ranks_that_agree(mode):
    r = _bench("--gpus", "2", "--dry-run", "--steps", "4", "--warmup", "1", "--mode", mode, "--cpu-seconds", "0")
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout  # only rank 0 prints
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["steps"] == 4 and out["warmup"] == 1
    per = out["per_rank_s"]
    assert len(per) == 2
    # both ranks timed the same barrier-bracketed region: equal to within the barrier skew
    assert abs(per[0] - per[1]) < 0.05
    # reported step time is the slowest rank's; rank 1 sleeps twice as long per step
    assert out["ms_per_step"] == pytest.approx(max(per) * 1e3 / 4, rel=1e-3)
    assert out["ms_per_step"] >= 2.0
    assert out["scaling"] == ("weak" if mode == "streams" else "strong")
    assert out["config"]["parallelism"] == f"{mode}2"
    if mode == "streams":
        # the other BASELINE configs ride along in multi-GPU runs, each with every rank's time
        for key in ("config2", "config4", "config5", "f32"):
            assert key in out, key
            assert len(out[key]["per_rank_s"]) == 2, key
        assert out["config4"]["scaling"] == "strong" and out["config5"]["scaling"] == "weak"


def test_world_size_mismatch_is_an_error():
    r = _bench("--gpus", "2", "--dry-run", "--steps", "1", env={"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0
    assert "WORLD_SIZE" in r.stderr


def test_single_rank_dry_run():
    r = _bench("--gpus", "1", "--dry-run", "--steps", "2", "--warmup", "0", "--cpu-seconds", "0", "--demod-steps", "0")
    assert r.returncode == 0, r.stderr[-2000:]
    out = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][0])
    assert out["n_gpus"] == 1 and len(out["per_rank_s"]) == 1
