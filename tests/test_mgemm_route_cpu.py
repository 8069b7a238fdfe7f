"""Which projections ops.linear sends to the medium-M weight-streaming kernel (ops.dispatch.mgemm_route):
Llama-3-8B o_proj at 17..128 rows with MLS_MGEMM=1 (off by default); never gate_up / LM head, skinny-sized batches, short
reductions (BERT) or TP-split shapes."""
import pytest

from mlmicroservicetemplate_amd.ops import dispatch
from mlmicroservicetemplate_amd.ops.dispatch import mgemm_route


@pytest.fixture(autouse=True)
def _route_on(monkeypatch):
    monkeypatch.setattr(dispatch, "_MGEMM", "1")  # opt-in (MLS_MGEMM=1)


def test_off_by_default(monkeypatch):
    monkeypatch.setattr(dispatch, "_MGEMM", "0")  # MLS_MGEMM unset
    assert not mgemm_route(64, 4096, 4096)


def test_llama_decode_shapes():
    for M in (17, 64, 128):
        assert mgemm_route(M, 4096, 4096)      # o_proj
    for M in (17, 64, 128, 200, 256):
        assert not mgemm_route(M, 4096, 14336)  # down_proj (slower there)
        assert not mgemm_route(M, 6144, 4096)   # qkv (level)
        assert not mgemm_route(M, 28672, 4096)  # gate_up
        assert not mgemm_route(M, 128256, 4096)  # LM head
    assert not mgemm_route(200, 4096, 4096)     # o_proj past 128 rows: level


def test_wide_ab_rule(monkeypatch):
    monkeypatch.setattr(dispatch, "_MGEMM", "all")
    assert mgemm_route(256, 4096, 14336) and mgemm_route(128, 6144, 4096) and not mgemm_route(256, 6144, 4096)


def test_outside_the_regime():
    assert not mgemm_route(16, 4096, 4096)   # skinny kernel's batch sizes
    assert not mgemm_route(257, 4096, 4096)  # tile route
    assert not mgemm_route(128, 768, 768)    # BERT [CLS]-row projections
    assert not mgemm_route(128, 4096, 512)   # TP = 8 row-parallel slice
    assert not mgemm_route(128, 4000, 4096)  # N not a multiple of 64
