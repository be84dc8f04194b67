"""CPU: the C-ABI library builds, loads without a GPU and exports every symbol
the public headers declare; device-less behaviour is a clean status code."""
import ctypes
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
INCLUDE = os.path.join(ROOT, "include")


def declared_symbols():
    names = set()
    for fn in os.listdir(INCLUDE):
        if not fn.endswith(".h"):
            continue
        text = open(os.path.join(INCLUDE, fn)).read()
        text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
        names |= set(re.findall(r"\b(rfa_[a-z_]+)\s*\(", text))
        names |= set(re.findall(r"\b(Java_com_mantz_1it_nativedsp_NativeDsp_\w+)\s*\(", text))
    return sorted(names)


@pytest.fixture(scope="module")
def lib():
    import rfanalyzer_amd
    rfanalyzer_amd.build()
    return rfanalyzer_amd.lib()


def test_headers_declare_expected_surface():
    syms = declared_symbols()
    for must in ["rfa_create", "rfa_process", "rfa_process_host", "rfa_set_tuning", "rfa_get_peaks",
                 "rfa_get_boxcar", "rfa_get_ema", "rfa_windowed_fft_mag_planar",
                 "Java_com_mantz_1it_nativedsp_NativeDsp_performFFT",
                 "Java_com_mantz_1it_nativedsp_NativeDsp_performFFTAndLogMag"]:
        assert must in syms


def test_every_declared_symbol_is_exported(lib):
    out = subprocess.run(["nm", "-D", "--defined-only", lib._name], capture_output=True, text=True, check=True).stdout
    exported = set(line.split()[-1] for line in out.splitlines() if line.strip())
    missing = [s for s in declared_symbols() if s not in exported]
    assert not missing, missing
    for s in declared_symbols():
        assert getattr(lib, s) is not None


def test_library_embeds_gfx950_code_object(lib):
    data = open(lib._name, "rb").read()
    assert b"hipv4-amdgcn-amd-amdhsa--gfx950" in data


def test_jni_abi_version_and_framing_sentinel(lib):
    """rfa_jni.h RFA_JNI_ABI_VERSION 2: frame_stride 0 of the raw-packet natives is the
    reference's packet framing; a caller built against version 1 (0 = dense
    batch) can detect the change at load time.  No legacy call yet: last status RFA_OK."""
    text = open(os.path.join(INCLUDE, "rfa_jni.h")).read()
    ver = int(re.search(r"#define RFA_JNI_ABI_VERSION (\d+)", text).group(1))
    assert ver == 2 and lib.rfa_jni_abi_version() == ver
    assert lib.rfa_jni_last_status() == 0


def test_status_strings_and_defaults(lib):
    from rfanalyzer_amd._lib import RfaConfig
    assert lib.rfa_abi_version() == 1
    assert lib.rfa_status_string(0) == b"ok"
    assert lib.rfa_status_string(-2) == b"size mismatch"
    c = RfaConfig()
    lib.rfa_default_config(ctypes.byref(c))
    assert (c.fft_size, c.window, c.input_format, c.ring_rows, c.peak_hold) == (16384, 0, 0, 400, 0)


def test_create_without_device_or_with_bad_config(lib):
    import torch

    from rfanalyzer_amd._lib import RfaConfig
    c = RfaConfig()
    lib.rfa_default_config(ctypes.byref(c))
    h = ctypes.c_void_p()
    c.fft_size = 1000
    assert lib.rfa_create(ctypes.byref(c), ctypes.byref(h)) == -3  # unsupported size, checked first
    c.fft_size = 1024
    c.window = 9
    assert lib.rfa_create(ctypes.byref(c), ctypes.byref(h)) == -1
    c.window = 0
    rc = lib.rfa_create(ctypes.byref(c), ctypes.byref(h))
    if not torch.cuda.is_available():
        assert rc == -4 and not h.value  # RFA_ERR_NODEVICE, nothing leaked
    elif rc == 0:
        lib.rfa_destroy(h)
    assert lib.rfa_process(None, None, 0, 0, None) == -1
    assert lib.rfa_destroy(None) == -1


def test_jni_table_layout_constants():
    text = open(os.path.join(ROOT, "rfanalyzer_amd", "csrc", "jni_min.h")).read()
    # the compiled static_asserts pin these; make sure they stay in the header
    for slot in ("171", "200", "205", "213", "228"):
        assert f"== {slot} * sizeof(void *)" in text


def test_no_store_data_hazard_in_kernel_isa():
    """The gfx950 hazard behind buf_store_f32x4's inline asm (fft_common.h): no 12/16-byte
    vector store may have its data VGPRs overwritten by the next VALU instruction."""
    r = subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "rfanalyzer_amd", "csrc"), "hazard-check"],
                       capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-2000:]
    assert "0 hazards" in r.stdout


def test_product_library_reads_no_environment(lib):
    """Determinism: RFA_* switches exist only in A/B builds
    (-DRFA_AB_BUILD); the product librfa.so does not import getenv at all."""
    from rfanalyzer_amd import _lib
    r = subprocess.run(["nm", "-D", "--undefined-only", _lib.LIB_PATH], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    assert "getenv" not in r.stdout


def test_product_library_ships_only_the_wide_64k_kernel(lib):
    """N = 64 K runs the wide kernel in product builds: the wave-decoupled kernel
    (scripts/ab/fft_w64.hip, measured 8-10 % slower, profiles/r04/w64_ab.txt) is linked into A/B
    builds only, so its code object is absent from the product librfa.so."""
    from rfanalyzer_amd import _lib
    with open(_lib.LIB_PATH, "rb") as fh:
        blob = fh.read()
    assert b"fft64_kernel" not in blob
    assert b"fft_wide_kernel" in blob


def _pffft_accepts(n: int) -> bool:
    """pffft_new_setup(N, PFFFT_COMPLEX) (pffft.c:1231-1280) succeeds: 0 < N <= 2^26,
    N % 16 == 0, and decompose() of N / 4 over {5, 3, 4, 2} leaves nothing."""
    if n <= 0 or n > (1 << 26) or n % 16:
        return False
    m = n // 4
    for f in (5, 3, 4, 2):
        while m % f == 0:
            m //= f
    return m == 1


def test_seam_length_rule_matches_pffft(lib):
    """rfa_seam_supported (host only, no device) takes exactly pffft's lengths."""
    lib.rfa_seam_supported.restype = ctypes.c_int
    lib.rfa_seam_supported.argtypes = [ctypes.c_int32]
    sizes = list(range(-16, 20000)) + [3 << 20, 5 << 20, 15 << 22, 1 << 26, (1 << 26) + 16, 1 << 27, 2 ** 31 - 1]
    bad = [n for n in sizes if bool(lib.rfa_seam_supported(n)) != _pffft_accepts(n)]
    assert not bad, bad[:10]
    h = ctypes.c_void_p()
    assert lib.rfa_seam_create(1000, 0, ctypes.byref(h)) == -3 and not h.value  # unsupported, checked first
    assert lib.rfa_seam_destroy(None) == -1
