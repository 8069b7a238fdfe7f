"""X1 weight broadcast / X6 health / max-over-ranks on a gloo 'fake cluster' (world 2, 4 and 8)."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    from mlmicroservicetemplate_amd.models.resnet import init_resnet50, init_resnet50_spec
    from mlmicroservicetemplate_amd.parallel import dist as mdist

    info = mdist.init_distributed(backend="gloo")
    try:
        params = init_resnet50(0) if rank == 0 else None
        spec = {k: (tuple(v.shape), v.dtype) for k, v in init_resnet50_spec().items()}
        got = mdist.broadcast_state(params, src=0, spec=spec)
        ref = init_resnet50(0)
        ok = all(torch.equal(got[k], ref[k]) for k in ref)
        # spec-less path (object broadcast of the spec first), mixed dtypes
        st = {"a": torch.arange(10, dtype=torch.int64), "b": torch.ones(3, 4, dtype=torch.bfloat16)} if rank == 0 else None
        got2 = mdist.broadcast_state(st, src=0)
        ok2 = torch.equal(got2["a"], torch.arange(10)) and got2["b"].dtype == torch.bfloat16
        healthy_all = mdist.all_reduce_health(True)
        healthy_one_bad = mdist.all_reduce_health(rank != 1)
        mx = mdist.max_over_ranks(float(rank))
        # TPComm's split all-reduce (start now, wait later: the TP prefill overlap's primitive)
        from mlmicroservicetemplate_amd.models.llama import TPComm, _ARPending

        comm = TPComm(None, world)
        t = torch.full((1000,), float(rank + 1))
        h = comm.all_reduce_start(t)
        busy = torch.randn(200, 200) @ torch.randn(200, 200)  # independent work while it flies
        red = h.wait()
        ok3 = isinstance(h, _ARPending) and red is t and bool((red == world * (world + 1) / 2).all()) and busy.numel() > 0
        q.put((rank, ok and ok3, ok2, healthy_all, healthy_one_bad, mx))
    finally:
        mdist.destroy()


@pytest.mark.parametrize("world", [2, 4, 8])
@pytest.mark.timeout(180)
def test_collectives_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=150) for _ in range(world)]
    for p in procs:
        p.join(30)
        assert p.exitcode == 0
    for rank, ok, ok2, h_all, h_bad, mx in res:
        assert ok and ok2
        assert h_all is True and h_bad is False
        assert mx == world - 1
