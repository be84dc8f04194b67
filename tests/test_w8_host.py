"""The W_8 form of the in-register DFT-16 / DFT-32 (rfanalyzer_amd/csrc/fft_w8.h), checked on the
host: its sqrt(1/2) factors folded into the adds (and the S0 form, whose inputs 4 and 12 arrive
unscaled) give the DFT of the inputs to fp32 rounding, like the plain DFTs of fft_common.h.  The
device path of the same functions (packed asm) is covered by the GPU parity tests."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "rfanalyzer_amd", "csrc")


def test_w8_dft_forms_match_the_dft(tmp_path):
    exe = tmp_path / "w8"
    cmd = ["/opt/rocm/bin/hipcc", "-O2", "-std=c++20", "--offload-arch=gfx950", "--cuda-host-only", "-I", CSRC,
           os.path.join(ROOT, "tests", "csrc", "w8_dft_host.cpp"), "-o", str(exe)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    if r.returncode != 0 and "not found" in r.stderr:
        pytest.skip("hipcc not available")
    assert r.returncode == 0, r.stderr[-2000:]
    out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=60)
    assert out.returncode == 0, out.stderr
    e16, e16w, e16s, e32, e32w = (float(x) for x in out.stdout.split())
    for e in (e16, e16w, e16s, e32, e32w):
        assert e < 5e-7, out.stdout  # fp32 rounding of a 16/32-point transform (measured 1.1-1.5e-7), relative to its largest bin
