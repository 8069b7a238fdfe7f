"""ops/csrc/fastdiv.h -- the launch-constant integer division the conv kernels use in place of hipcc's
runtime-divisor sequence -- checked against `/` on the host: every n < 2^16 for d <= 2048, and values
around multiples of random divisors up to 2^31 (tests/native/fastdiv_check.cpp)."""
import os
import shutil
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(os.path.dirname(HERE), "mlmicroservicetemplate_amd", "ops", "csrc")


@pytest.mark.timeout(300)
def test_fastdiv_matches_division(tmp_path):
    cxx = shutil.which("g++") or shutil.which("clang++")
    if cxx is None:
        pytest.skip("no host C++ compiler")
    exe = str(tmp_path / "fastdiv_check")
    build = subprocess.run([cxx, "-std=c++17", "-O2", "-fsanitize=undefined", "-fno-sanitize-recover=undefined",
                            "-I", CSRC, os.path.join(HERE, "native", "fastdiv_check.cpp"), "-o", exe],
                           capture_output=True, text=True)
    assert build.returncode == 0, build.stderr[-4000:]
    run = subprocess.run([exe], capture_output=True, text=True, timeout=240)
    assert run.returncode == 0 and "fastdiv: ok" in run.stdout, (run.stdout[-2000:], run.stderr[-2000:])
