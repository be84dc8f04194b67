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
    if not log:
        return
    tr = terminalreporter
    tr.write_sep("-", "dB parity (tests/golden_util.py db_stats)")
    for floor in sorted({x["floor_db"] for x in log}):
        xs = [x for x in log if x["floor_db"] == floor]
        tr.write_line(f"floor {floor:.0f} dB: {len(xs)} comparisons, {sum(x['bins'] for x in xs)} bins; "
                      f"max |d| live {max(x['max_live'] for x in xs):.2e} dB (bar {gu.DB_TOL}); "
                      f"excluded below floor: mean {sum(x['excluded'] for x in xs) / len(xs):.3f}, "
                      f"max {max(x['excluded'] for x in xs):.3f}; "
                      f"max |d| over all finite bins {max(x['max_finite'] for x in xs):.3e} dB")
    for kind, bound in (("every bin (no floor, 0 excluded)", False),
                        ("every bin beyond the reference's own float64 error", True)):
        for bar in sorted({x["bar"] for x in gu.FULL_ROW_LOG if bool(x.get("bound")) == bound}):
            xs = [x for x in gu.FULL_ROW_LOG if bool(x.get("bound")) == bound and x["bar"] == bar]
            tr.write_line(f"{kind}, bar {bar} dB: {len(xs)} comparisons, {sum(x['bins'] for x in xs)} bins; "
                          f"max |d| {max(x['max_full'] for x in xs):.2e} dB")
