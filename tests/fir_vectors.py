"""The reference's own FIR golden vectors (ApplicationTest.kt testFirFilter /
testFirFilter2, JVM output, tolerance 1e-9), loaded from
tests/golden/fir_application_test.json (made by tests/golden/gen_fir_vectors.py),
and their inputs regenerated with the test's own arithmetic."""
import json
import math
import os

import numpy as np

F32 = np.float32
PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "fir_application_test.json")


def cases():
    with open(PATH) as fh:
        return json.load(fh)["cases"]


def inputs(c):
    """reIn[i] = cos(2*PI*f1*i / sampleRate.toFloat()).toFloat() + cos(... f2 ...).toFloat()
    (ApplicationTest.kt:33-38): double argument, each term rounded to float, float sum."""
    fsr = float(F32(c["sample_rate"]))
    re = np.empty(c["samples"], F32)
    im = np.empty(c["samples"], F32)
    for i in range(c["samples"]):
        a1 = 2 * math.pi * c["f1"] * i / fsr
        a2 = 2 * math.pi * c["f2"] * i / fsr
        re[i] = F32(F32(math.cos(a1)) + F32(math.cos(a2)))
        im[i] = F32(F32(math.sin(a1)) + F32(math.sin(a2)))
    return re, im


def expected(c):
    return np.array(c["re_expected"], F32), np.array(c["im_expected"], F32)


def check(c, re, im):
    er, ei = expected(c)
    assert re.shape == er.shape and im.shape == ei.shape, (re.shape, er.shape)
    tol = c["tolerance"]
    assert np.max(np.abs(re.astype(np.float64) - er)) <= tol, c["name"]
    assert np.max(np.abs(im.astype(np.float64) - ei)) <= tol, c["name"]
