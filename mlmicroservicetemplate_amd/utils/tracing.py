"""roctx ranges for rocprofv3 (T9 / SURVEY.md §5.1).

``MLS_TRACE=1`` turns every :func:`range` into a roctx push/pop (torch-ROCm routes
``torch.cuda.nvtx`` to ``libroctx64``), so ``rocprofv3 --marker-trace`` shows batch assembly,
H2D, graph replay, D2H and collectives next to the kernels.  Off by default: a no-op context
manager costs ~100 ns.
"""
from __future__ import annotations

import contextlib
import os

_ENABLED = os.environ.get("MLS_TRACE", "0") not in ("", "0", "false", "False")


def enabled() -> bool:
    return _ENABLED


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
    if not _ENABLED:
        return _NULL
    return _roctx(name)
