"""§5.2 race detection for the native host runtime: the engine's staging pool
(engine/csrc/staging_core.h) built with ThreadSanitizer and with AddressSanitizer +
UndefinedBehaviorSanitizer and driven from several submitter threads (tests/native/staging_sanitize.cpp).
Host code only -- GPU sanitizers are not available on the test pool."""
import os
import shutil
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "native", "staging_sanitize.cpp")


@pytest.mark.parametrize("san", ["thread", "address,undefined"])
@pytest.mark.timeout(300)
def test_staging_pool_under_sanitizer(tmp_path, san):
    cxx = shutil.which("g++") or shutil.which("clang++")
    if cxx is None:
        pytest.skip("no host C++ compiler")
    exe = str(tmp_path / "staging_sanitize")
    build = subprocess.run([cxx, "-std=c++17", "-O1", "-g", f"-fsanitize={san}", "-fno-omit-frame-pointer", "-pthread",
                            SRC, "-o", exe], capture_output=True, text=True)
    assert build.returncode == 0, build.stderr[-4000:]
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1 second_deadlock_stack=1",
               ASAN_OPTIONS="detect_leaks=1:halt_on_error=1:verify_asan_link_order=0", UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    run = subprocess.run([exe], capture_output=True, text=True, env=env, timeout=240)
    assert run.returncode == 0 and "staging sanitize: ok" in run.stdout, (run.stdout[-2000:], run.stderr[-6000:])
