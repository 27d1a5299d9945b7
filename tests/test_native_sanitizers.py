"""Race detection / memory checking of the native host runtime.

GPU AddressSanitizer is not available on this pool, so the sanitizers run on host code:
the worker-pool row streamer behind the out-of-core path (csrc/row_streamer.h, wrapped by
csrc/loader.cpp) is built standalone with -fsanitize=thread and with
-fsanitize=address,undefined and driven by a multi-threaded stress test
(tests/native/row_streamer_test.cpp).  Any report fails the test.
"""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tests", "native", "row_streamer_test.cpp")


@pytest.mark.parametrize("flags", [["-fsanitize=thread"],
                                   ["-fsanitize=address,undefined", "-fno-sanitize-recover=all"]],
                         ids=["tsan", "asan_ubsan"])
def test_row_streamer_under_sanitizer(tmp_path, flags):
    cxx = shutil.which("g++") or shutil.which("clang++")
    if cxx is None:
        pytest.skip("no host C++ compiler")
    exe = tmp_path / "rs_test"
    cmd = [cxx, "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", *flags,
           "-I", os.path.join(ROOT, "csrc"), SRC, "-o", str(exe), "-pthread"]
    subprocess.run(cmd, check=True, capture_output=True, text=True, timeout=300)
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1 second_deadlock_stack=1",
               ASAN_OPTIONS="detect_leaks=1:halt_on_error=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "row_streamer_test: ok" in r.stdout
    assert "WARNING: ThreadSanitizer" not in r.stderr and "ERROR: AddressSanitizer" not in r.stderr
