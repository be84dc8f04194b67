"""CPU: host ASan / UBSan build.  tests/sanitize/Makefile compiles the
host code of librfa (engine.hip and ddc.hip with -fsanitize after -Xarch_host,
jni_shim.cpp) and the oracle's C restatement with AddressSanitizer +
UndefinedBehaviorSanitizer (reports abort), and san_driver exercises the JNI
symbols through a bounds-checking mock JNIEnv (validation and size-mismatch
paths, NativeDsp.kt:45-46), the host-only helpers, the packet framer and the
oracle.  No GPU is needed: device work is not reached."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_sanitized_host_code_runs_clean():
    b = subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "tests", "sanitize"), "-j4"], capture_output=True,
                       text=True, timeout=900)
    assert b.returncode == 0, b.stderr[-3000:]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([os.path.join(ROOT, "alt", "san", "san_driver")], capture_output=True, text=True, timeout=300,
                       env=env)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    assert "all checks passed" in r.stdout
    assert "AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr, r.stderr[-4000:]
