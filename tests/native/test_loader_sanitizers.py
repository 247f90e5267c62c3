"""Sanitizer builds of the native host batch assembler (native/runtime/loader.cpp).

The C++ thread-pool loader is built together with a stress driver (tests/native/loader_stress.cpp)
under AddressSanitizer + UndefinedBehaviorSanitizer and, separately, ThreadSanitizer, and run on the
CPU: any heap misuse, data race between the pool threads and submit/wait/destroy, or wrong row is a
failure.  (GPU-side sanitizers are not available on this pool; the loader is host code.)
SURVEY §2.9 A2 (race detection / sanitizers)."""

import os
import shutil
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(os.path.dirname(os.path.dirname(HERE)), "rocket_amd", "native", "runtime", "loader.cpp")
CXX = shutil.which("g++") or shutil.which("clang++")

pytestmark = pytest.mark.skipif(CXX is None, reason="no host C++ compiler")


@pytest.mark.parametrize("san", ["address,undefined", "thread"])
def test_loader_under_sanitizer(tmp_path, san):
    exe = str(tmp_path / "loader_stress")
    cmd = [CXX, "-std=c++17", "-O1", "-g", f"-fsanitize={san}", "-fno-omit-frame-pointer", "-pthread",
           os.path.join(HERE, "loader_stress.cpp"), SRC, "-o", exe]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    if r.returncode != 0 and "unsupported" in (r.stderr or ""):
        pytest.skip(f"-fsanitize={san} unsupported: {r.stderr[-200:]}")
    assert r.returncode == 0, r.stderr[-2000:]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:halt_on_error=1", UBSAN_OPTIONS="halt_on_error=1",
               TSAN_OPTIONS="halt_on_error=1")
    run = subprocess.run([exe], capture_output=True, text=True, timeout=300, env=env)
    assert run.returncode == 0, (run.stdout + run.stderr)[-3000:]
    assert "0 bad rows" in run.stdout
