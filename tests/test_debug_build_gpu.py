"""Bounds-checked debug build: the -DMLS_DEBUG kernel variant, loaded with
MLS_DEBUG=1 and run under HIP_LAUNCH_BLOCKING=1, reports violated data-dependent bounds (context
bound below lens, cache slot past the cache, position past the RoPE table) as NativeError
instead of faulting, and passes the transformer kernel suite and the Llama model test."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _run(args, timeout=600):
    root = os.path.dirname(HERE)
    env = dict(os.environ, MLS_DEBUG="1", HIP_LAUNCH_BLOCKING="1",
               PYTHONPATH=os.pathsep.join([root, os.environ.get("PYTHONPATH", "")]))
    return subprocess.run([sys.executable, *args], cwd=os.path.dirname(HERE), env=env, capture_output=True,
                          text=True, timeout=timeout)


def test_debug_build_reports_violations():
    r = _run([os.path.join(HERE, "debug_build_probe.py")])
    assert r.returncode == 0 and "DEBUG-BUILD-OK" in r.stdout, r.stdout[-3000:] + r.stderr[-3000:]


def test_kernel_suite_under_debug_build():
    r = _run(["-m", "pytest", "-q", "-x", "-p", "no:cacheprovider", os.path.join(HERE, "test_transformer_ops_gpu.py"),
              os.path.join(HERE, "test_models_gpu.py"), "-k", "decode or rope or llama or flash"])
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
