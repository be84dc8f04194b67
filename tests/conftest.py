import os
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
for p in (ROOT, HERE, os.path.join(HERE, "golden")):
    if p not in sys.path:
        sys.path.insert(0, p)

# torch before librfa when both are used in one process: torch's wheel bundles its own
# libamdhip64.so (ROCm 7.0); loaded first, librfa resolves to that same runtime (one
# HIP runtime per process).  Without torch every test that does not need it still runs.
try:
    import torch  # noqa: F401
except ImportError:
    pass


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device) and librfa.so")


@pytest.fixture(autouse=True)
def _parity_test_name(request):
    """Name the running test in the parity logs (golden_util.CURRENT_TEST)."""
    try:
        import golden_util as gu
    except ImportError:
        yield
        return
    gu.CURRENT_TEST = request.node.nodeid
    yield
    gu.CURRENT_TEST = ""


@pytest.fixture(scope="session")
def rfa():
    """librfa on a real device; fails loudly (no CPU fallback) when absent."""
    import rfanalyzer_amd

    n = rfanalyzer_amd.device_count()
    assert n > 0, "no HIP device visible to librfa"
    return rfanalyzer_amd


def pytest_terminal_summary(terminalreporter, exitstatus, config):
    """Make the parity bar visible: every dB comparison of the session, the share of
    bins the Parseval floor excluded, and the worst difference over all finite bins."""
    try:
        import golden_util as gu
    except ImportError:
        return
    log = gu.PARITY_LOG
    if not (log or gu.FULL_ROW_LOG or gu.NOTES):
        return
    tr = terminalreporter
    tr.write_sep("-", "dB parity (tests/golden_util.py db_stats)")
    for floor in sorted({x["floor_db"] for x in log}):
        xs = [x for x in log if x["floor_db"] == floor]
        live = max(xs, key=lambda x: x["max_live"])
        fin = max(xs, key=lambda x: x["max_finite"])
        tr.write_line(f"floor {floor:.0f} dB: {len(xs)} comparisons, {sum(x['bins'] for x in xs)} bins; "
                      f"max |d| live {live['max_live']:.2e} dB (bar {gu.DB_TOL}; {live['test']}); "
                      f"excluded below floor: mean {sum(x['excluded'] for x in xs) / len(xs):.3f}, "
                      f"max {max(x['excluded'] for x in xs):.3f}; max |d| over every bin both sides resolve "
                      f"(>= 20 dB above fp32 rounding: within {gu.RESOLVE_DB:.0f} dB of the row level) {fin['max_finite']:.3e} dB "
                      f"({fin['test']}); {sum(x['subres'] for x in xs)} bins below that floor on a side "
                      f"(KAT zeros, within 20 dB of fp32 rounding noise) not compared")
    for kind, bound in (("every bin (no floor, 0 excluded)", False),
                        ("every bin beyond the reference's own float64 error", True)):
        for bar in sorted({x["bar"] for x in gu.FULL_ROW_LOG if bool(x.get("bound")) == bound}):
            xs = [x for x in gu.FULL_ROW_LOG if bool(x.get("bound")) == bound and x["bar"] == bar]
            top = max(xs, key=lambda x: x["max_full"])
            tr.write_line(f"{kind}, bar {bar} dB: {len(xs)} comparisons, {sum(x['bins'] for x in xs)} bins; "
                          f"max |d| {top['max_full']:.2e} dB ({top.get('label') or top['test']})")
    named = [x for x in gu.FULL_ROW_LOG if x.get("label")]
    for x in named:
        tr.write_line(f"  {x['label']}: {x['max_full']:.4f} dB over {x['bins']} bins (bar {x['bar']})")
    for line in gu.NOTES:
        tr.write_line(f"  {line}")
