"""The bench line's host-side measurements: the C-ABI's per-call cost from a
C loop (`tools/call_bench`, bench.py `c_call_cost`) and the host-fed end-to-end run (bench.py
`host_fed_run`: pinned host IQ -> H2D on a second stream -> rfa_process into ring + state).
CPU: the harness's parsing and error handling with stand-in executables.  GPU: the real binary
and a small host-fed run, whose device state must equal the device-resident path's."""
import importlib.util
import json
import os
import stat

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench_module():
    spec = importlib.util.spec_from_file_location("bench_under_test", os.path.join(ROOT, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def _fake_tools(tmp_path, script):
    (tmp_path / "tools").mkdir()
    exe = tmp_path / "tools" / "call_bench"
    exe.write_text("#!/bin/sh\n" + script)
    exe.chmod(exe.stat().st_mode | stat.S_IXUSR)
    return exe


def test_c_call_cost_absent_binary_is_none(tmp_path, monkeypatch):
    b = _bench_module()
    monkeypatch.setattr(b, "ROOT", str(tmp_path))
    assert b.c_call_cost(calls=10) is None


def test_c_call_cost_reads_the_last_json_line_per_shape(tmp_path, monkeypatch):
    b = _bench_module()
    _fake_tools(tmp_path, 'echo "warming up"\n'
                          'echo "{\\"calls\\": $1, \\"batches_per_call\\": $2, \\"wall_us_per_call\\": 8.0}"\n')
    monkeypatch.setattr(b, "ROOT", str(tmp_path))
    out = b.c_call_cost(calls=128)
    assert out["batches_per_call_1"] == {"calls": 128, "batches_per_call": 1, "wall_us_per_call": 8.0}
    # 64 batches per call: calls / 64 launches of the same total work
    assert out["batches_per_call_64"] == {"calls": 2, "batches_per_call": 64, "wall_us_per_call": 8.0}


def test_c_call_cost_failure_is_reported_not_raised(tmp_path, monkeypatch):
    b = _bench_module()
    _fake_tools(tmp_path, 'echo "rfa_create -> -3" >&2\nexit 1\n')
    monkeypatch.setattr(b, "ROOT", str(tmp_path))
    out = b.c_call_cost(calls=10)
    for kb in (1, 64):
        assert "rfa_create -> -3" in out[f"batches_per_call_{kb}"]["error"]


def test_call_bench_is_built_against_the_in_tree_library():
    exe = os.path.join(ROOT, "tools", "call_bench")
    if not os.path.exists(exe):
        pytest.skip("tools/call_bench not built (run __graft_entry__.build())")
    blob = open(exe, "rb").read()
    assert blob[:4] == b"\x7fELF"
    assert b"librfa.so" in blob and b"$ORIGIN/../rfanalyzer_amd" in blob  # rpath to the in-tree .so


@pytest.mark.gpu
def test_call_bench_runs_on_the_gpu():
    import subprocess
    exe = os.path.join(ROOT, "tools", "call_bench")
    if not os.path.exists(exe):
        pytest.fail("tools/call_bench missing: __graft_entry__.build() builds it")
    for kb in (1, 4):
        r = subprocess.run([exe, "40", str(kb)], capture_output=True, text=True, timeout=120)
        assert r.returncode == 0, r.stderr[-500:]
        d = json.loads(r.stdout.strip().splitlines()[-1])
        assert d["batches_per_call"] == kb and d["calls"] == 40
        for k in ("enqueue_us_per_call", "wall_us_per_call", "kernel_us", "empty_launch_us", "msamples_per_s"):
            assert d[k] > 0, (k, d)
        # a call cannot finish faster than its own kernel runs back to back
        assert d["wall_us_per_call"] >= 0.5 * d["kernel_us"], d


@pytest.mark.gpu
def test_host_fed_run_matches_the_device_resident_state():
    """The host-fed harness (H2D on a second stream, double-buffered, event-ordered) must feed
    rfa_process the same bytes in the same order as the device-resident path: after the same
    calls, peaks and EMA agree bit for bit."""
    torch = pytest.importorskip("torch")
    import rfanalyzer_amd
    b = _bench_module()
    dev = torch.device("cuda", 0)
    n, frames, calls, fmt = 16384, 24, 6, "s8"
    r = b.host_fed_run(torch, dev, n, fmt, frames, calls, ring_rows=32, host_batches=2, seed=11, state_out=True)
    assert r["value"] > 0 and r["h2d_GBps"] > 0 and r["calls"] == calls
    assert r["bytes_per_call"] == n * frames * 2

    # the same batches (make_pool with the harness's seed), device-resident, in the harness's call
    # order: 4 warm-up calls, then `calls` timed ones (its copy-only pass processes nothing)
    src = b.make_pool(torch, n, frames, fmt, 1, 11, dev)[:2]
    torch.cuda.synchronize()  # made on torch's stream; the engine runs on its own
    eng = rfanalyzer_amd.SpectrumEngine(n, "blackman", fmt, avg="ema", avg_length=30, ema_alpha=0.1,
                                        peak_hold=True, ring_rows=32, device=0)
    eng.set_tuning(100_000_000, 20_000_000)
    for i in list(range(4)) + list(range(calls)):
        eng.process_device(src[i % 2].data_ptr(), frames, 0, None)
    torch.cuda.synchronize()
    peaks, ema = eng.peaks(), eng.ema()
    eng.close()
    assert np.isfinite(peaks).all()
    np.testing.assert_array_equal(r["peaks"], peaks)
    np.testing.assert_array_equal(r["ema"], ema)
