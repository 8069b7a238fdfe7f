"""X2 one-shot IPC all-reduce (ops/csrc/custom_allreduce.hip): 2 and 4 processes sharing the
one GPU of a test box (IPC handles, flags, epochs and graph capture are exercised; the 8-GPU xGMI
path itself is covered by the same code on a multi-GPU node)."""
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("world", [2, 4, 8])
def test_custom_allreduce_multiprocess(world):
    root = os.path.dirname(HERE)
    port = _port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                   PYTHONPATH=os.pathsep.join([root, os.environ.get("PYTHONPATH", "")]))
        procs.append(subprocess.Popen([sys.executable, os.path.join(HERE, "custom_ar_worker.py")], env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True))
    outs = []
    for p in procs:
        try:
            out, _ = p.communicate(timeout=240)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        outs.append((p.returncode, out[-2000:]))
    assert all(rc == 0 for rc, _ in outs), outs
    for _, out in outs:  # the lost-peer case of the GEMM-fused all-reduce: time to fail, error word
        for line in out.splitlines():
            if "fused stall" in line:
                print(line)
