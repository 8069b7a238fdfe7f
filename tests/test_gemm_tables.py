"""Dispatch tables (ops/tuned/*.json): a served GEMM shape that misses a table is logged once per
process (VERDICT r3 'What's weak' #7) -- tuned shapes are silent."""
import logging

from mlmicroservicetemplate_amd import ops
from mlmicroservicetemplate_amd.ops import tables


def test_untuned_shape_logged_once(caplog):
    caplog.set_level(logging.WARNING, logger="mlsamd.ops")
    tables._TABLE_MISSES.clear()
    assert ops.tile_cfg_for(1234, 4096, 4160) == (0, 1)
    assert ops.tile_cfg_for(1234, 4096, 4160) == (0, 1)
    assert ops.tile_cfg_for(999, 4096, 4160) == (0, 1)  # same projection, another M: not logged again
    msgs = [r.getMessage() for r in caplog.records if "not in gemm_tile_gfx950.json" in r.getMessage()]
    assert len(msgs) == 1 and "M=1234 N=4096 K=4160" in msgs[0]


def test_tuned_shapes_are_silent(caplog):
    caplog.set_level(logging.WARNING, logger="mlsamd.ops")
    tables._TABLE_MISSES.clear()
    (M, N, K), (impl, cfg, sk) = next(iter(ops.gemm_tile_plan().items()))
    assert impl == "tile" and ops.tile_cfg_for(M, N, K) == (cfg, sk)
    (M2, N2, K2), plan = next(iter(ops.gemm_plan().items()))
    assert ops.small_m_plan_for(M2, N2, K2) == plan
    assert not [r for r in caplog.records if "not in" in r.getMessage()]
    assert ops.small_m_plan_for(3, 5, 64) is None
    assert any("gemm_plan_gfx950.json" in r.getMessage() for r in caplog.records)


def test_decode256_routes_are_per_shape_winners():
    """The 256-row decode step (256 serving slots): each projection on its measured native winner --
    conv_gemm split-K for QKV / O / down, the fused-SiLU tile for gate_up, the 256 x 128 tile for the
    LM head (profiles/r4_dec256_gemm_probe.jsonl, r6_gemm_native_routes_probe.jsonl)."""
    assert ops.tile_route_for(256, 6144, 4096) == ("conv", 7, 2)
    assert ops.tile_route_for(256, 28672, 4096) == ("tile", 16, 1)
    assert ops.tile_route_for(256, 4096, 4096) == ("conv", 7, 2)
    assert ops.tile_route_for(256, 4096, 14336) == ("conv", 10, 4)
    assert ops.tile_route_for(256, 128256, 4096) == ("tile", 16, 1)


def test_prefill_row_ranges_route_without_exact_entries(caplog):
    """Row-range entries cover every prefill token count of a projection (no per-M miss logging):
    Llama-3-8B TP=1 projections from 1024 rows run the native tile kernel (256 x 256 or, for QKV below
    8192 rows, 256 x 128); shapes outside every range still fall back to the tile kernel's pick."""
    caplog.set_level(logging.WARNING, logger="mlsamd.ops")
    tables._TABLE_MISSES.clear()
    for m in (1024, 4096, 5000, 32768):
        for n, k in ((6144, 4096), (4096, 4096), (28672, 4096), (4096, 14336)):
            assert ops.tile_route_for(m, n, k)[0] == "tile"
    assert ops.tile_route_for(4096, 6144, 4096) == ("tile", 16, 1)
    assert ops.tile_route_for(32768, 6144, 4096) == ("tile", 15, 1)
    assert not [r for r in caplog.records if "not in" in r.getMessage()]
    assert ops.tile_route_for(700, 6144, 4096) == ("tile", 0, 1)  # below the range, no exact entry


def test_resnet_tuning_regimes():
    """ResNet-50 per-layer kernel tables per regime: the serial table (one batch alone) takes the
    pipelined 3x3 kernel on every stride-1 3x3; the concurrent one (4 co-running batches) keeps the
    halo kernel on layers 1-3; batches without a serial table fall back to the concurrent one."""
    from mlmicroservicetemplate_amd.ops import autotune

    conc = autotune.load_tuning("resnet50", 32)
    ser = autotune.load_tuning("resnet50", 32, regime="serial")
    assert ser["layer1.1.conv2"][0] >= ops.CFG_PIPE and ser["layer3.1.conv2"][0] >= ops.CFG_PIPE
    assert conc["layer1.1.conv2"][0] < ops.CFG_PIPE
    assert conc["layer4.1.conv2"][0] >= ops.CFG_PIPE
    assert set(ser) == set(conc)
    assert autotune.load_tuning("resnet50", 8, regime="serial") == autotune.load_tuning("resnet50", 8)


def test_default_tables_have_no_library_route():
    """No default path calls a library GEMM: the tile table has no "blas" entry,
    the small-M plan no library config, and ops.linear reaches hipBLASLt only when asked for it
    explicitly (MLS_GEMM_IMPL=blas / impl="blas", the A/B arm)."""
    import json
    import os

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    tuned = os.path.join(root, "mlmicroservicetemplate_amd", "ops", "tuned")
    with open(os.path.join(tuned, "gemm_tile_gfx950.json")) as f:
        entries = json.load(f)["entries"]
    assert all(e.get("impl", "tile") in ("tile", "conv") for e in entries), \
        [e["shape"] for e in entries if e.get("impl", "tile") not in ("tile", "conv")]
    assert all(r[0] in ("tile", "conv") for r in ops.gemm_tile_plan().values())
    assert all(route[0] in ("tile", "conv") for rs in tables.gemm_tile_ranges().values() for _, _, route in rs)
    with open(os.path.join(tuned, "gemm_plan_gfx950.json")) as f:
        assert "hipBLASLt" not in json.load(f)["doc"]


class _FakeCuda:  # just enough of a CUDA tensor for the dispatch predicates
    def __init__(self, *shape):
        self.shape = shape
        self.device = type("D", (), {"type": "cuda"})()

    def is_contiguous(self):
        return True


def test_linear_reaches_the_library_only_on_request(monkeypatch):
    """Every former library shape dispatches to our kernels by default; impl="blas" is the only way to
    hipBLASLt (the route is resolved before any GPU call, so this runs on the CPU)."""
    from mlmicroservicetemplate_amd.ops import dispatch

    calls = []
    monkeypatch.setattr(dispatch, "_linear_blas", lambda *a, **k: calls.append("blas"))
    monkeypatch.setattr(dispatch, "gemm_tile", lambda *a, **k: calls.append(("tile", k.get("cfg"), k.get("splitk"))))
    monkeypatch.setattr(dispatch, "gemm", lambda *a, **k: calls.append(("conv", k.get("cfg"), k.get("splitk"))))
    for m, n, k in ((4096, 6144, 4096), (4096, 4096, 4096), (4096, 28672, 4096), (4096, 4096, 14336),
                    (512, 6144, 4096), (512, 4096, 4096), (256, 4096, 4096), (256, 4096, 14336), (256, 128256, 4096)):
        calls.clear()
        dispatch.linear(_FakeCuda(m, k), _FakeCuda(n, k))
        assert calls and calls[0] != "blas" and calls[0][0] in ("tile", "conv"), (m, n, k, calls)
        calls.clear()
        dispatch.linear(_FakeCuda(m, k), _FakeCuda(n, k), impl="native")
        assert calls and calls[0] != "blas", (m, n, k, calls)
    calls.clear()
    dispatch.linear(_FakeCuda(4096, 4096), _FakeCuda(6144, 4096), impl="blas")
    assert calls == ["blas"]
