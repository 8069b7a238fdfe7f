"""roctx tracing.  The switch: off = shared no-op context, on = balanced push/pop
even when the traced block raises (push/pop intercepted, so this runs without a GPU).  Coverage:
every range named in ``utils/tracing.py`` is emitted by its component -- CPU parts here; the
engine's ranges (stage / h2d / replay / d2h / d2h_wait) are checked on the GPU in
``test_engine_gpu.py``."""
import asyncio
import multiprocessing as mp
import os
import socket
from types import SimpleNamespace

import pytest
import torch

from mlmicroservicetemplate_amd.utils import tracing


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.fixture
def calls(monkeypatch):
    log = []
    monkeypatch.setattr(torch.cuda.nvtx, "range_push", lambda name: log.append(("push", name)))
    monkeypatch.setattr(torch.cuda.nvtx, "range_pop", lambda: log.append(("pop",)))
    was = tracing.enabled()
    yield log
    tracing.set_enabled(was)


def test_disabled_is_noop(calls):
    tracing.set_enabled(False)
    a, b = tracing.range("x"), tracing.range("y")
    assert a is b  # one shared null context: nothing allocated per call
    with a:
        pass
    assert calls == []


def test_enabled_nests_and_pops_on_error(calls):
    tracing.set_enabled(True)
    with tracing.range("outer"):
        with pytest.raises(RuntimeError):
            with tracing.range("inner"):
                raise RuntimeError("boom")
    assert calls == [("push", "outer"), ("push", "inner"), ("pop",), ("pop",)]


def test_record_collects_names(calls):
    with tracing.record() as names:
        with tracing.range("a"):
            with tracing.range("b"):
                pass
    assert names == ["a", "b"]
    with tracing.range("outside"):  # no sink: nothing recorded
        pass
    tracing.set_enabled(True)
    with tracing.record() as names, tracing.range("c"):
        pass
    assert names == ["c"] and calls == [("push", "c"), ("pop",)]


def test_batcher_ranges():
    from mlmicroservicetemplate_amd.scheduler.batcher import DynamicBatcher

    async def main():
        b = DynamicBatcher(lambda xs: [x + 1 for x in xs], max_batch=4, max_wait_us=100)
        await b.start()
        out = await asyncio.gather(*[b.submit(i) for i in range(8)])
        await b.stop()
        return out

    with tracing.record() as names:
        assert asyncio.run(main()) == list(range(1, 9))
    assert "batch.assemble" in names and "batch.run" in names


def test_native_handoff_range():
    from mlmicroservicetemplate_amd.frontend.native import HostReplica

    rep = HostReplica(lambda x: (x.sum(axis=1),), (4,), max_batch=2, inflight=1)
    slot = rep.acquire(1.0)
    rep.buffer(slot)[:2] = 1
    with tracing.record() as names:
        (s,) = rep.run(slot, 2)
    assert s.tolist() == [4, 4] and names == ["native.handoff"]


def test_llama_step_ranges():
    from mlmicroservicetemplate_amd.models.llama import GenParams, LlamaTP, init_llama_shard, tiny_config

    cfg = tiny_config()
    m = LlamaTP(init_llama_shard(cfg, 1, 0, seed=1), cfg, max_batch=1, max_seq=64)
    with tracing.record() as names:
        m.generate(torch.tensor([[5, 6, 7]]), torch.tensor([3]), GenParams(max_new_tokens=3))
    assert names.count("llama.prefill") == 1 and names.count("llama.decode") == 2


def test_reload_range():
    from mlmicroservicetemplate_amd.parallel.reload import ReloadCoordinator

    class P:
        name = "p"

        def reload_spec(self):
            return {}

        def load_params(self, w, s):
            return {"seed": s}

        def apply_params(self, params):
            pass

    co = ReloadCoordinator(P(), SimpleNamespace(rank=0, world_size=1), SimpleNamespace(PORT=0))
    with tracing.record() as names:
        assert co.request(seed=3)["generation"] == 1
    assert names == ["reload.apply"]


def _dist_worker(rank, world, port, q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    from mlmicroservicetemplate_amd.models.llama import TPComm
    from mlmicroservicetemplate_amd.parallel import dist as mdist
    from mlmicroservicetemplate_amd.utils import tracing as tr

    mdist.init_distributed("gloo")
    comm = TPComm(None, world)
    with tr.record() as names:
        mdist.broadcast_state({"w": torch.ones(3)} if rank == 0 else None, spec={"w": ((3,), torch.float32)})
        mdist.all_reduce_health(True)
        mdist.barrier()
        mdist.max_over_ranks(float(rank))
        comm.all_reduce_(torch.ones(4))
        comm.all_gather(torch.ones(2))
        comm.broadcast_(torch.ones(2))
    mdist.destroy()
    q.put((rank, list(names)))


def test_collective_ranges_two_ranks():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_dist_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    got = dict(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(30)
        assert p.exitcode == 0
    want = ["dist.broadcast", "dist.health", "dist.barrier", "dist.max", "tp.all_reduce", "tp.all_gather",
            "tp.broadcast"]
    for r in range(2):
        assert got[r] == want, got[r]
