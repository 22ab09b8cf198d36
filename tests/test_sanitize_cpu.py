"""Host-side sanitizer run: the native runtime core (JSON parser, /predict packing and
response formatting, ISO/timedelta/float-repr) built with -fsanitize=address,undefined and fuzzed."""
import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_runtime_core_tsan_threaded_paths():
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import build_ext
    exe = build_ext.build_sanitize(kind="tsan")
    r = subprocess.run([exe, "2000", "3"], capture_output=True, text=True, timeout=300,
                       env=dict(os.environ, TSAN_OPTIONS="halt_on_error=1"))
    assert r.returncode == 0, r.stdout + r.stderr
    assert "WARNING: ThreadSanitizer" not in r.stderr


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_runtime_core_asan_ubsan_fuzz():
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import build_ext
    exe = build_ext.build_sanitize()
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([exe, "30000", "11"], capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "0 failures" in r.stdout
    assert "ERROR: AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr
