"""Dump GPU rows for every golden fixture (analysis aid): gpurun_out/rows_<tag>.npz"""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
import golden_util as gu
import rfanalyzer_amd
tag = sys.argv[1] if len(sys.argv) > 1 else "x"
out = {}
for spec in gu.manifest()["fixtures"]:
    if spec["n"] > 131072:
        continue
    data = gu.fixture_input(spec)
    with rfanalyzer_amd.SpectrumEngine(spec["n"], spec["window"], spec["fmt"], ring_rows=0) as e:
        out[spec["name"]] = e.process(data, spec["n_frames"], spec.get("packet_size", 0))
np.savez(os.path.join(ROOT, "gpurun_out", f"rows_{tag}.npz"), **out)
print("dumped", len(out))
