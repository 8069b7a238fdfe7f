"""roctx ranges for rocprofv3 (T9 / SURVEY.md §5.1).

``MLS_TRACE=1`` turns every :func:`range` into a roctx push/pop (torch-ROCm routes
``torch.cuda.nvtx`` to ``libroctx64``), so ``rocprofv3 --marker-trace`` shows the serving path
next to the kernels.  Off by default: a disabled range is a shared no-op context manager.

Range names (each is emitted by the component named; ``tests/test_tracing.py`` checks them):

====================  ==========================================================
``batch.assemble``    batcher: a batch is cut from the queue (``DynamicBatcher``)
``batch.run``         batcher: the batch function on the executor thread
``native.handoff``    C++ front end -> engine slot hand-off (``frontend/native.py``)
``<engine>.stage``    engine: request arrays -> pinned slot (host gather)
``<engine>.h2d``      engine: H2D enqueue on the slot stream
``<engine>.replay``   engine: hipGraph replay (or eager forward) enqueue
``<engine>.d2h``      engine: D2H enqueue
``<engine>.d2h_wait`` engine: host waits for the slot's D2H event
``dist.broadcast``    X1 weight broadcast (``broadcast_state``)
``dist.health``       X6 readiness all-reduce
``dist.barrier``      process-group barrier
``dist.max``          max-over-ranks all-reduce (bench)
``tp.all_reduce``     X2 / X3 tensor-parallel all-reduce (``TPComm``)
``tp.all_gather``     X4 candidate all-gather
``tp.broadcast``      X5 request / step broadcast
``llama.prefill``     one Llama prefill forward
``llama.decode``      one Llama decode step (graph replay or eager)
``reload.apply``      hot weight reload on a rank
====================  ==========================================================

:func:`record` collects the names of the ranges entered inside it (whether or not roctx is
enabled) -- the hook the tracing test uses, also handy to see which ranges a code path hits.
"""
from __future__ import annotations

import contextlib
import os
import threading
from typing import List, Optional

_ENABLED = os.environ.get("MLS_TRACE", "0") not in ("", "0", "false", "False")
_sink: Optional[List[str]] = None
_sink_lock = threading.Lock()


def enabled() -> bool:
    return _ENABLED


def active() -> bool:
    """Are ranges being emitted or recorded (callers may then prefer their instrumented path)?"""
    return _ENABLED or _sink is not None


def set_enabled(flag: bool) -> None:
    global _ENABLED
    _ENABLED = bool(flag)


@contextlib.contextmanager
def _roctx(name: str):
    import torch

    torch.cuda.nvtx.range_push(name)
    try:
        yield
    finally:
        torch.cuda.nvtx.range_pop()


_NULL = contextlib.nullcontext()


def range(name: str):  # noqa: A001 - mirrors nvtx/roctx naming
    if _sink is not None:
        with _sink_lock:
            if _sink is not None:
                _sink.append(name)
    if not _ENABLED:
        return _NULL
    return _roctx(name)


@contextlib.contextmanager
def record():
    """Collect the names of every range entered (any thread) while the block runs."""
    global _sink
    names: List[str] = []
    with _sink_lock:
        prev, _sink = _sink, names
    try:
        yield names
    finally:
        with _sink_lock:
            _sink = prev
