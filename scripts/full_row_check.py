"""Every-bin parity survey (no Parseval floor): librfa rows vs the reference's own
pffft golden rows and vs the float64 oracle, for every quantized-input fixture,
the config-3 batch (64 K, B = 500) and the state sequence.  Prints one line per
comparison; used to decide what tests/test_gpu_parity.py asserts."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "tests", "golden")]
import torch  # noqa: F401,E402 - torch's HIP runtime first

import golden_util as gu  # noqa: E402
import oracle  # noqa: E402
import rfanalyzer_amd as rfa  # noqa: E402
import signals  # noqa: E402


def main():
    m = gu.manifest()
    for spec in m["fixtures"]:
        if spec["fmt"] not in ("s8", "u8", "s16"):
            continue
        data = gu.fixture_input(spec)
        with rfa.SpectrumEngine(spec["n"], spec["window"], spec["fmt"], ring_rows=0) as e:
            rows = e.process(data, spec["n_frames"], spec.get("packet_size", 0))
        exp = gu.expected(spec)
        ref64 = oracle.spectrum_rows(data, signals.FORMATS[spec["fmt"]], spec["n"], spec["n_frames"],
                                     spec.get("packet_size"), gu.WINDOW_IDS[spec["window"]])
        sub = spec["subset_stride"]
        print(f"{spec['name']:28s} gpu-pffft {gu.full_row_diff(rows[:, ::sub], exp):.5f}  "
              f"gpu-f64 {gu.full_row_diff(rows, ref64.astype(np.float32)):.5f}  "
              f"pffft-f64 {gu.full_row_diff(ref64[:, ::sub].astype(np.float32), exp):.5f}", flush=True)
    # config 3: 64 K s8, 500 frames
    n, b = 65536, 500
    data = signals.frames_bytes(n, b, "s8", 3, tones=((0.1234, 0.4), (-0.377, 0.01)), noise=0.05)
    with rfa.SpectrumEngine(n, "blackman", "s8", ring_rows=0) as e:
        rows = e.process(data, b)
    if oracle.ref_available():
        ref = oracle.ref_spectrum_rows(data, oracle.IN_S8, n, b)
        print(f"{'config3 64K B=500':28s} gpu-pffft {gu.full_row_diff(rows, ref):.5f}", flush=True)
    ref64 = oracle.spectrum_rows(data[: 8 * 2 * n], oracle.IN_S8, n, 8, None, oracle.WIN_BLACKMAN)
    print(f"{'config3 first 8 rows':28s} gpu-f64 {gu.full_row_diff(rows[:8], ref64.astype(np.float32)):.5f}")


if __name__ == "__main__":
    main()
