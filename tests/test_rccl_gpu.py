"""The RCCL (``nccl`` backend) code paths on a real GPU.  The GPU test box has one GPU and RCCL
refuses two ranks on one device, so this runs a forced world-1 ``nccl`` group
(``init_distributed(force=True)``) in a child process: X1 ``broadcast_state`` with device tensors,
X6 ``all_reduce_health``, ``max_over_ranks``, ``barrier(device_ids=...)``, the ``TPComm``
all-reduce / all-gather / broadcast paths on device tensors, and an RCCL all-reduce captured in a
hipGraph (what ``MLS_TP_GRAPHS=1`` relies on).  Multi-rank RCCL over xGMI is exercised by the
driver's 8-GPU scaling run (``bench.py --gpus N``)."""
import os
import subprocess
import sys
import textwrap

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SCRIPT = textwrap.dedent("""
    import os, sys
    sys.path.insert(0, sys.argv[1])
    os.environ.update(RANK="0", WORLD_SIZE="1", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1")
    os.environ.pop("MASTER_PORT", None)
    import torch, torch.distributed as dist
    from mlmicroservicetemplate_amd.parallel import dist as mdist
    from mlmicroservicetemplate_amd.models.llama import TPComm

    def stage(x):
        print("stage", x, flush=True)

    info = mdist.init_distributed(force=True)
    stage("init")
    assert dist.is_initialized() and dist.get_backend() == "nccl", dist.get_backend()
    dev = torch.device("cuda", 0)
    state = {"a": torch.randn(1000, 7), "b": torch.arange(33, dtype=torch.int32),
             "c": torch.randn(5).to(torch.bfloat16)}
    spec = {k: (tuple(v.shape), v.dtype) for k, v in state.items()}
    got = mdist.broadcast_state(state, src=0, device=dev, spec=spec)
    for k in state:
        assert got[k].device == dev and torch.equal(got[k].cpu(), state[k]), k
    stage("broadcast")
    got2 = mdist.broadcast_state(state, src=0, device=dev)  # spec via object broadcast
    assert all(torch.equal(got2[k].cpu(), state[k]) for k in state)
    assert mdist.all_reduce_health(True) is True and mdist.all_reduce_health(False) is False
    assert mdist.max_over_ranks(3.25) == 3.25
    mdist.barrier()
    stage("health/max/barrier")
    comm = TPComm(None, 1, device=dev, custom_ar=False)
    x = torch.randn(64, 4096, device=dev).to(torch.bfloat16)
    y = comm._all_reduce(x.clone())
    assert torch.equal(y, x)
    g = comm._all_gather(x[:2])
    assert g.shape == (1, 2, 4096) and g.is_cuda and torch.equal(g[0], x[:2])
    b = comm._broadcast(x[:3].clone(), 0)
    assert torch.equal(b, x[:3])
    stage("tpcomm")
    # split all-reduce on the RCCL stream (the TP prefill overlap's primitive): start, queue
    # independent work on the compute stream, wait; tp=2 forces the async path on the world-1 group
    from mlmicroservicetemplate_amd.models.llama import _ARPending
    comm2 = TPComm(None, 2, device=dev, custom_ar=False)
    big = torch.randn(1024, 4096, device=dev).to(torch.bfloat16)
    want = big.clone()
    h = comm2.all_reduce_start(big)
    z = torch.randn(2048, 2048, device=dev) @ torch.randn(2048, 2048, device=dev)
    red = h.wait()
    torch.cuda.synchronize()
    assert isinstance(h, _ARPending) and red is big and torch.equal(red, want) and z.isfinite().all()
    stage("async all-reduce")
    # RCCL inside a captured hipGraph (thread_local capture mode: the watchdog thread polls)
    s = torch.cuda.Stream()
    buf = torch.ones(8192, device=dev)
    s.wait_stream(torch.cuda.current_stream())  # buf was filled on the default stream
    with torch.cuda.stream(s):
        dist.all_reduce(buf)
    torch.cuda.synchronize()
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr, capture_error_mode="thread_local"):
        buf.mul_(2)
        dist.all_reduce(buf)
    for _ in range(3):
        gr.replay()
    torch.cuda.synchronize()
    assert float(buf[0]) == 8.0, float(buf[0])
    mdist.destroy()
    print("rccl-world1-ok")
""")


def test_rccl_world1_paths():
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    r = subprocess.run([sys.executable, "-c", SCRIPT, ROOT], env=env, capture_output=True, text=True, timeout=240)
    err = "\n".join(ln for ln in r.stderr.splitlines() if "frame #" not in ln)
    assert r.returncode == 0 and "rccl-world1-ok" in r.stdout, (r.stdout[-2000:], err[:3000], err[-2000:])
