"""roctx tracing switch: off = shared no-op context, on = balanced push/pop even
when the traced block raises.  The push/pop pair is intercepted, so this runs without a GPU."""
import pytest
import torch

from mlmicroservicetemplate_amd.utils import tracing


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
