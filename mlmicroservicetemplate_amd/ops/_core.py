"""Shared helpers of the ops wrappers: activation codes, argument checks, per-stream scratch."""
from __future__ import annotations

from typing import Optional, Tuple

import torch


ACT_NONE, ACT_RELU, ACT_GELU, ACT_TANH, ACT_SILU, ACT_SILU_MUL = 0, 1, 2, 3, 4, 5


_ACTS = {None: 0, "none": 0, "relu": 1, "gelu": 2, "tanh": 3, "silu": 4, "silu_mul": 5}


def _act(a) -> int:
    if isinstance(a, int):
        return a
    return _ACTS[a]


class StreamWorkspace:
    """fp32 scratch (split-K slabs) per HIP stream: batches that run concurrently on different
    streams (GpuEngine concurrent slots) must not share it.  A stream's buffer is allocated on
    its first use -- the engine's eager warm-up, before any graph capture."""

    def __init__(self, elems: int, device, zero: bool = False):
        self.elems = int(elems)
        self.device = torch.device(device)
        self.zero = zero  # zero-initialised (an accumulator its consumer re-zeroes, e.g. the fused pool)
        self._bufs: dict = {}

    def get(self) -> torch.Tensor:
        key = torch.cuda.current_stream(self.device).cuda_stream if self.device.type == "cuda" else 0
        buf = self._bufs.get(key)
        if buf is None:
            buf = (torch.zeros if self.zero else torch.empty)(self.elems, device=self.device, dtype=torch.float32)
            self._bufs[key] = buf
        return buf


def _ptr(t: Optional[torch.Tensor]) -> Optional[int]:
    return None if t is None else t.data_ptr()


def _need(t: torch.Tensor, name: str, dtype: torch.dtype, device: torch.device) -> None:
    if t.dtype != dtype:
        raise TypeError(f"{name}: expected {dtype}, got {t.dtype}")
    if t.device != device:
        raise ValueError(f"{name}: expected device {device}, got {t.device}")
    if not t.is_contiguous():
        raise ValueError(f"{name}: must be contiguous")


def conv_out_hw(h: int, w: int, k: int, stride: int, pad: int) -> Tuple[int, int]:
    return (h + 2 * pad - k) // stride + 1, (w + 2 * pad - k) // stride + 1


def _workspace_args(ws: Optional[torch.Tensor]):
    if ws is None:
        return None, 0
    return ws.data_ptr(), ws.numel() * ws.element_size()
