"""GpuEngine on MI355X: concurrent in-flight slots (per-slot streams + graph pools, per-stream
split-K workspace) must give exactly the results of one-at-a-time execution."""
import contextlib
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def test_concurrent_slots_match_serial():
    from mlmicroservicetemplate_amd.engine.worker import GpuEngine
    from mlmicroservicetemplate_amd.models import resnet
    from mlmicroservicetemplate_amd.ops.autotune import load_tuning

    p = resnet.init_resnet50(0)
    model = resnet.ResNet50Fused(p, DEV, max_batch=8, tuning=load_tuning("resnet50", 8))

    def fwd(x):
        v, i = model.classify(x, 5)
        return v, i

    rng = np.random.default_rng(0)
    batches = [rng.integers(0, 256, (8, 224, 224, 3), dtype=np.uint8) for _ in range(6)]
    serial = GpuEngine(fwd, DEV, (224, 224, 3), torch.uint8, buckets=[8], inflight=1, name="serial")
    serial.warmup()
    ref = [serial.run(b) for b in batches]
    conc = GpuEngine(fwd, DEV, (224, 224, 3), torch.uint8, buckets=[8], inflight=3, concurrent=True, name="conc")
    conc.warmup()
    assert conc.stats()["concurrent"]
    for _ in range(3):
        # keep three batches in flight: each submit beyond the third waits for a free slot, so
        # the oldest ticket is collected first
        pending, outs = [], []
        for b in batches:
            if len(pending) == 3:
                outs.append(pending.pop(0).wait())
            pending.append(conc.submit(b))
        outs += [t.wait() for t in pending]
        for (rv, ri), (ov, oi) in zip(ref, outs):
            np.testing.assert_array_equal(ri, oi)
            np.testing.assert_array_equal(rv, ov)


def test_benchmarked_config_end_to_end_vs_fp32():
    """The exact configuration bench.py times: ResNet50Fused(max_batch=32) with the shipped B=32
    tuning table, GpuEngine(4 slots on CU-masked streams in 2 partitions, hipGraphs), 5 batches of
    32 submitted back to back -- every row compared with the fp32 PyTorch reference of the same
    weights."""
    from mlmicroservicetemplate_amd.engine.worker import GpuEngine
    from mlmicroservicetemplate_amd.models import resnet
    from mlmicroservicetemplate_amd.ops.autotune import load_tuning

    tuning = load_tuning("resnet50", 32)
    assert tuning, "the shipped B=32 tuning table must load (tuned/resnet50_gfx950_b32.json)"
    p = resnet.init_resnet50(0)
    model = resnet.ResNet50Fused(p, DEV, max_batch=32, tuning=tuning)

    def fwd(x):
        logits = model(x)
        v, i = model.ops.softmax_topk(logits, 5)
        return logits, v, i

    eng = GpuEngine(fwd, DEV, (224, 224, 3), torch.uint8, buckets=[32], inflight=4, concurrent=True,
                    use_graphs=True, name="benchcfg", cu_partitions=2)
    assert eng.cu_partitions == 2 and eng.inflight == 4  # bench.py's defaults
    eng.warmup(capture=True)
    rng = np.random.default_rng(7)
    batches = [rng.integers(0, 256, (32, 224, 224, 3), dtype=np.uint8) for _ in range(5)]
    outs, pending = [], []
    for b in batches:  # 4 co-running batches (one per slot), the 5th as soon as a slot frees
        if len(pending) == eng.inflight:
            outs.append(pending.pop(0).wait())
        pending.append(eng.submit(b))
    outs += [t.wait() for t in pending]
    pd = {k: v.to(DEV) for k, v in p.items()}
    for b, (logits, vals, idx) in zip(batches, outs):
        ref = resnet.resnet50_reference(pd, torch.from_numpy(b).to(DEV)).float().cpu()
        lg = torch.from_numpy(logits).float()
        rel = ((lg - ref).abs().max() / ref.abs().max()).item()
        assert rel <= 2e-2, rel
        top2 = ref.topk(2, dim=-1).values
        margin = (top2[:, 0] - top2[:, 1]) / ref.abs().max()
        sure = margin > 1e-2
        assert sure.sum() >= 8, "too few rows with a clear reference top-1 to compare"
        assert torch.equal(torch.from_numpy(idx[:, 0]).long()[sure], ref.argmax(-1)[sure])
        # the fused softmax/top-5 head agrees with torch on the engine's own logits
        pv, pi = torch.softmax(lg, -1).topk(5, dim=-1)
        np.testing.assert_allclose(vals, pv.numpy(), rtol=2e-2, atol=1e-4)


def test_engine_roctx_ranges():
    """the engine's stage / h2d / replay / d2h / d2h_wait ranges are emitted."""
    from mlmicroservicetemplate_amd.engine.worker import GpuEngine
    from mlmicroservicetemplate_amd.utils import tracing

    eng = GpuEngine(lambda x: (x.float().sum(dim=1),), DEV, (16,), torch.uint8, buckets=[4], inflight=2,
                    concurrent=True, name="tr")
    eng.warmup(capture=True)
    tracing.set_enabled(True)  # real roctx push/pop too
    try:
        with tracing.record() as names:
            (s,) = eng.run([np.full(16, 2, np.uint8)] * 3)
    finally:
        tracing.set_enabled(False)
    assert s.tolist() == [32.0] * 3
    assert not eng.graph_copies  # default: the copies are stream operations with their own ranges
    for k in ("stage", "h2d", "replay", "d2h", "d2h_wait"):
        assert f"tr.{k}" in names, (k, names)
    # MLS_GRAPH_COPIES=1: H2D -> forward -> D2H is one replay
    os.environ["MLS_GRAPH_COPIES"] = "1"
    try:
        eng2 = GpuEngine(lambda x: (x.float().sum(dim=1),), DEV, (16,), torch.uint8, buckets=[4], inflight=2,
                         concurrent=True, name="tr2")
    finally:
        del os.environ["MLS_GRAPH_COPIES"]
    eng2.warmup(capture=True)
    tracing.set_enabled(True)
    try:
        with tracing.record() as names2:
            (s2,) = eng2.run([np.full(16, 3, np.uint8)] * 3)
    finally:
        tracing.set_enabled(False)
    assert s2.tolist() == [48.0] * 3 and eng2.graph_copies and eng2.slots[0].graph_copies[4]
    for k in ("stage", "replay", "d2h_wait"):
        assert f"tr2.{k}" in names2, (k, names2)
    assert "tr2.h2d" not in names2


def test_cu_partition_masks_select_disjoint_halves():
    """ops.partition_masks(mode="intra"): each mask's stream runs only on its own CUs -- 1 / P of
    every XCD, disjoint across partitions -- as seen by the census kernel (csrc/partition.hip)."""
    from mlmicroservicetemplate_amd import ops

    full = ops.census_cus(ops.cu_census(torch.cuda.Stream(), blocks=4096))
    assert len(full) == torch.cuda.get_device_properties(0).multi_processor_count
    for parts in (2, 4):
        masks = ops.partition_masks(parts, DEV, mode="intra")
        assert masks is not None
        seen = set()
        for m in masks:
            cus = ops.census_cus(ops.cu_census(ops.cu_masked_stream(m, DEV, key="census"), blocks=4096))
            assert len(cus) == len(full) // parts, (parts, len(cus))
            assert {x for x, _ in cus} == {x for x, _ in full}  # every XCD keeps a share
            assert not (cus & seen)
            seen |= cus
        assert seen == full


def test_release_masked_streams():
    """ops.partition.release_masked_streams destroys the pooled masked streams of one key (what the
    atexit hook does for all of them); a later request for that key creates a working stream again."""
    from mlmicroservicetemplate_amd import ops
    from mlmicroservicetemplate_amd.ops import partition

    m = ops.partition_masks(2, DEV, mode="intra")[0]
    st = ops.cu_masked_stream(m, DEV, key="release-test")
    n0 = len(ops.census_cus(ops.cu_census(st, blocks=1024)))
    partition.release_masked_streams("release-test")
    assert not any(k[2] == "release-test" for k in partition._MASKED_STREAMS)
    st2 = ops.cu_masked_stream(m, DEV, key="release-test")
    assert len(ops.census_cus(ops.cu_census(st2, blocks=1024))) == n0
    partition.release_masked_streams("release-test")


def test_partitioned_engine_matches_serial():
    """Slots on CU-masked streams (2 partitions) give exactly the results of one-at-a-time execution."""
    from mlmicroservicetemplate_amd.engine.worker import GpuEngine
    from mlmicroservicetemplate_amd.models import resnet
    from mlmicroservicetemplate_amd.ops.autotune import load_tuning

    p = resnet.init_resnet50(1)
    model = resnet.ResNet50Fused(p, DEV, max_batch=8, tuning=load_tuning("resnet50", 8))
    rng = np.random.default_rng(3)
    batches = [rng.integers(0, 256, (8, 224, 224, 3), dtype=np.uint8) for _ in range(6)]
    serial = GpuEngine(lambda x: model.classify(x, 5), DEV, (224, 224, 3), torch.uint8, buckets=[8], inflight=1,
                       name="serial")
    serial.warmup()
    ref = [serial.run(b) for b in batches]
    part = GpuEngine(lambda x: model.classify(x, 5), DEV, (224, 224, 3), torch.uint8, buckets=[8], inflight=6,
                     concurrent=True, name="part", cu_partitions=2)
    # 6 slots over the 4 masked streams (slots 4, 5 share the streams of slots 0, 1)
    assert part.cu_partitions == 2 and part.inflight == 6 and part.part_streams == 4
    assert part.stats()["cu_partitions"] == 2
    assert part.slots[4].s_comp.cuda_stream == part.slots[0].s_comp.cuda_stream
    part.warmup()
    outs, pending = [], []
    for b in batches:  # a slot returns on wait(): keep at most `inflight` batches outstanding
        if len(pending) == part.inflight:
            outs.append(pending.pop(0).wait())
        pending.append(part.submit(b))
    outs += [t.wait() for t in pending]
    for (rv, ri), (ov, oi) in zip(ref, outs):
        np.testing.assert_array_equal(ri, oi)
        np.testing.assert_array_equal(rv, ov)


def test_native_launch_matches_python_enqueue():
    """GpuEngine's one-call native enqueue (ops/csrc/engine_launch.hip: H2D -> graph -> D2H -> done
    event) gives the same outputs as the instrumented Python sequence (taken while tracing)."""
    from mlmicroservicetemplate_amd.engine.worker import GpuEngine
    from mlmicroservicetemplate_amd.utils import tracing

    w = torch.randn(16, 48, device=DEV)
    eng = GpuEngine(lambda x: ((x.float() @ w.T).to(torch.bfloat16), x.float().sum(dim=1)), DEV, (48,), torch.uint8,
                    buckets=[4, 8], inflight=3, concurrent=True, name="nat")
    eng.warmup(capture=True)
    assert eng.native_launch and all(len(s.native) == 2 for s in eng.slots)
    rng = np.random.default_rng(5)
    batches = [rng.integers(0, 256, (n, 48), dtype=np.uint8) for n in (3, 8, 5, 1, 8, 7)]
    native = [eng.run(b) for b in batches]
    with tracing.record():  # tracing active: the Python enqueue
        python = [eng.run(b) for b in batches]
    for a, b in zip(native, python):
        for x, y in zip(a, b):
            np.testing.assert_array_equal(x, y)
    # overlapping submits (three in flight) through the native path
    tickets = [eng.submit(b) for b in batches[:3]]
    for t, ref in zip(tickets, native[:3]):
        for x, y in zip(t.wait(), ref):
            np.testing.assert_array_equal(x, y)


def test_prepared_batches_match_submit():
    """GpuEngine.prepare / launch_prepared (a batch staged into a spare pinned buffer before a slot
    frees, H2D straight from it) == submit, on the native and the instrumented enqueue; the spare
    buffers cycle back as tickets complete."""
    from mlmicroservicetemplate_amd.engine.worker import GpuEngine
    from mlmicroservicetemplate_amd.utils import tracing

    w = torch.randn(16, 48, device=DEV)
    eng = GpuEngine(lambda x: ((x.float() @ w.T).to(torch.bfloat16),), DEV, (48,), torch.uint8, buckets=[4, 8],
                    inflight=2, concurrent=True, name="prep")
    eng.warmup(capture=True)
    rng = np.random.default_rng(9)
    batches = [rng.integers(0, 256, (n, 48), dtype=np.uint8) for n in (3, 8, 5, 8, 2, 7, 8, 1)]
    ref = [eng.run(b) for b in batches]
    for active in (False, True):
        ctx = tracing.record() if active else contextlib.nullcontext()
        for sl in eng.slots:  # the graphs pull a prepared batch from its own buffer, not host_in
            sl.host_in.zero_()
        with ctx:
            pending, outs = [], []
            nxt = eng.prepare(batches[0])
            for i in range(len(batches)):
                pending.append(eng.launch_prepared(nxt))
                if i + 1 < len(batches):
                    nxt = eng.prepare(batches[i + 1])
                if len(pending) >= 2:
                    outs.append(pending.pop(0).wait())
            outs += [t.wait() for t in pending]
        for a, b in zip(ref, outs):
            np.testing.assert_array_equal(a[0], b[0])
        assert not any(bool(sl.host_in.any()) for sl in eng.slots), "a prepared batch was copied into host_in"
    assert eng._spare.qsize() == eng.inflight + 1
    # plain submits after prepared launches pull from host_in again (the cell is re-pointed)
    for i in range(4):
        np.testing.assert_array_equal(eng.run(batches[i])[0], ref[i][0])
        assert any(int(sl.src_cell[0]) == sl.host_in.data_ptr() for sl in eng.slots)


def test_sdma_free_io_and_fallback():
    """Round 5: a concurrent uint8 engine pulls its input and pushes its results with copy kernels
    inside the slot graph (no SDMA copies); a bucket whose input is not a 16-B multiple keeps the
    stream copies.  Both give the eager results."""
    from mlmicroservicetemplate_amd.engine.worker import GpuEngine

    w = torch.randn(16, 48, device=DEV)
    eng = GpuEngine(lambda x: ((x.float() @ w.T).to(torch.bfloat16),), DEV, (48,), torch.uint8, buckets=[4, 8],
                    inflight=2, concurrent=True, name="pull")
    eng.warmup(capture=True)
    assert eng.pull_h2d > 0
    assert all(sl.pulled[b] and sl.pushed[b] for sl in eng.slots for b in (4, 8))
    rng = np.random.default_rng(3)
    for n in (3, 8, 1):
        x = rng.integers(0, 256, (n, 48), dtype=np.uint8)
        got = eng.run(x)[0]
        ref = (torch.from_numpy(x).to(DEV).float() @ w.T).to(torch.bfloat16).float().cpu().numpy()
        np.testing.assert_allclose(got, ref, rtol=1e-2, atol=1e-2 * np.abs(ref).max())
    w5 = torch.randn(16, 5, device=DEV)
    eng5 = GpuEngine(lambda x: ((x.float() @ w5.T).to(torch.bfloat16),), DEV, (5,), torch.uint8, buckets=[3],
                     inflight=2, concurrent=True, name="odd")
    eng5.warmup(capture=True)
    assert not any(sl.pulled[3] for sl in eng5.slots)  # 15 bytes: the copy path
    x = rng.integers(0, 256, (3, 5), dtype=np.uint8)
    ref = (torch.from_numpy(x).to(DEV).float() @ w5.T).to(torch.bfloat16).float().cpu().numpy()
    np.testing.assert_allclose(eng5.run(x)[0], ref, rtol=1e-2, atol=1e-2 * np.abs(ref).max())


@pytest.mark.parametrize("model", ["linear", "resnet50"])
def test_prepull_batches_match_serial(monkeypatch, model):
    """MLS_PREPULL=1: prepare() stages a batch AND pulls it to a spare device buffer on the I/O
    stream; the slot's graph then copies it device-to-device.  Back-to-back prepared batches (more of
    them than device buffers, slots reused while earlier batches are still in flight) give exactly
    the outputs of one-at-a-time serial runs: no buffer is overwritten before its graph read it."""
    from mlmicroservicetemplate_amd.engine.worker import GpuEngine

    monkeypatch.setenv("MLS_PREPULL", "1")
    rng = np.random.default_rng(21)
    if model == "linear":
        w = torch.randn(16, 48, device=DEV)
        fwd = lambda x: ((x.float() @ w.T).to(torch.bfloat16), x.float().sum(dim=1))  # noqa: E731
        shape, sizes, buckets = (48,), (3, 8, 5, 8, 2, 7, 8, 1, 8, 8, 4, 6), [4, 8]
    else:
        from mlmicroservicetemplate_amd.models import resnet
        from mlmicroservicetemplate_amd.ops.autotune import load_tuning

        m = resnet.ResNet50Fused(resnet.init_resnet50(2), DEV, max_batch=8, tuning=load_tuning("resnet50", 8))
        fwd = lambda x: m.classify(x, 5)  # noqa: E731
        shape, sizes, buckets = (224, 224, 3), (8, 8, 5, 8, 8, 8, 3, 8), [8]
    batches = [rng.integers(0, 256, (n, *shape), dtype=np.uint8) for n in sizes]
    serial = GpuEngine(fwd, DEV, shape, torch.uint8, buckets=buckets, inflight=1, name="ser")
    serial.warmup()
    ref = [serial.run(b) for b in batches]
    eng = GpuEngine(fwd, DEV, shape, torch.uint8, buckets=buckets, inflight=3, concurrent=True, name="prepull",
                    cu_partitions=0)
    eng.warmup(capture=True)
    assert eng.prepull and eng.pull_grid >= eng.pull_h2d and eng.s_io is not None
    for sl in eng.slots:
        sl.host_in.zero_()
    pending, outs = [], []
    nxt = eng.prepare(batches[0])
    assert nxt.dev is not None
    for i in range(len(batches)):
        pending.append(eng.launch_prepared(nxt))
        if i + 1 < len(batches):
            nxt = eng.prepare(batches[i + 1])
        if len(pending) >= eng.inflight:
            outs.append(pending.pop(0).wait())
    outs += [t.wait() for t in pending]
    for a, b in zip(ref, outs):
        for x, y in zip(a, b):
            np.testing.assert_array_equal(x, y)
    assert not any(bool(sl.host_in.any()) for sl in eng.slots)
    assert eng._dev_spare.qsize() == eng.inflight + 2 and eng._spare.qsize() == eng.inflight + 1
    # a plain submit (pulled from the slot's pinned buffer over PCIe) still works after them
    for i in range(3):
        for x, y in zip(eng.run(batches[i]), ref[i]):
            np.testing.assert_array_equal(x, y)
