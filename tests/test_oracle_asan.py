"""Host sanitizer leg: the CPU restatement built with
AddressSanitizer + UndefinedBehaviorSanitizer (`make -C oracle asan`) must pass
the oracle's golden pins (tests/test_oracle_golden.py) with no sanitizer report.

The restatement is loaded into an uninstrumented Python, so libasan is
preloaded into a child pytest process; leak checking is off (the interpreter's
own allocations), every UBSan report is fatal.  The full-size 4K/8K hash test
is left out here (~3 min under ASan; it runs un-instrumented in the main
suite) -- every other pin, incl. the 1080p plane hash, the closed loops and the
threaded config-4 pipeline, runs instrumented.  CPU only."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _libasan():
    try:
        p = subprocess.run(["gcc", "-print-file-name=libasan.so"], capture_output=True, text=True, check=True)
    except (OSError, subprocess.CalledProcessError):
        return None
    path = p.stdout.strip()
    return path if os.path.isabs(path) and os.path.exists(path) else None


def test_oracle_golden_under_asan_ubsan():
    asan = _libasan()
    if asan is None:
        pytest.skip("gcc's libasan is not available")
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "asan"], check=True)
    env = dict(os.environ)
    env.update({
        "LD_PRELOAD": asan,
        "ASAN_OPTIONS": "detect_leaks=0:abort_on_error=1",
        "UBSAN_OPTIONS": "halt_on_error=1:print_stacktrace=1",
        "NH_ORACLE_LIB": os.path.join(ROOT, "oracle", "libnh_oracle_asan.so"),
    })
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-p", "no:cacheprovider",
                        os.path.join(ROOT, "tests", "test_oracle_golden.py"),
                        "-k", "not test_oracle_at_full_size_equals_reference"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert "AddressSanitizer" not in out and "runtime error:" not in out, out[-4000:]
    assert " passed" in out
