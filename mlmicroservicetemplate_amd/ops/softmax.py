"""Row softmax / top-k kernels (classifier heads, attention probabilities, sampling candidates)."""
from __future__ import annotations

from typing import Optional, Tuple

import torch

from ._lib import check, lib, stream_ptr
from ._core import _need, _ptr


def softmax_topk(
    x: torch.Tensor,
    k: int,
    *,
    softmax: bool = True,
    temperature: float = 1.0,
    vals: Optional[torch.Tensor] = None,
    idx: Optional[torch.Tensor] = None,
) -> Tuple[torch.Tensor, torch.Tensor]:
    """Row-wise (softmax ->) top-k of a ``[rows, N]`` bf16/fp32 matrix; fp32 values, int32 ids."""
    dev = x.device
    if x.dtype not in (torch.bfloat16, torch.float32) or not x.is_contiguous():
        raise TypeError("x must be contiguous bf16 or fp32")
    rows, N = x.shape
    if vals is None:
        vals = torch.empty(rows, k, device=dev, dtype=torch.float32)
    if idx is None:
        idx = torch.empty(rows, k, device=dev, dtype=torch.int32)
    rc = lib().mls_softmax_topk(x.data_ptr(), 0 if x.dtype == torch.bfloat16 else 1, vals.data_ptr(), idx.data_ptr(),
                                rows, N, k, int(softmax), float(temperature), stream_ptr(dev))
    check(rc, "mls_softmax_topk")
    return vals, idx


def softmax_rows(x: torch.Tensor, mask: Optional[torch.Tensor] = None, rows_per_mask: int = 1, scale: float = 1.0,
                 out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """``softmax(x * scale + mask)`` over the last dim; mask fp32 ``[rows/rows_per_mask, N]``."""
    dev = x.device
    _need(x, "x", torch.bfloat16, dev)
    N = x.shape[-1]
    rows = x.numel() // N
    if mask is not None:
        _need(mask, "mask", torch.float32, dev)
    out = torch.empty_like(x) if out is None else out
    rc = lib().mls_softmax_rows(x.data_ptr(), out.data_ptr(), _ptr(mask), rows, N, rows_per_mask, float(scale),
                                stream_ptr(dev))
    check(rc, "mls_softmax_rows")
    return out


def topk_large(x: torch.Tensor, k: int, max_chunk: int = 16384, *, lo: int = 0,
               valid: Optional[int] = None) -> Tuple[torch.Tensor, torch.Tensor]:
    """Raw-logit top-k of rows longer than one LDS-resident row (LM heads): split each row into
    equal chunks (per-chunk top-k in the kernel), then merge the ``chunks * k`` candidates.
    Returned indices are ``+ lo`` (a vocab shard's offset); columns at or past ``valid`` (a shard's
    zero-padded tail) never win.  bf16 rows whose length splits into <= 2048-wide chunks of a
    multiple of 8 take two native launches (wave-per-chunk register top-k, then
    ``mls_topk_merge``): ~10 us at vocab 128256 where the torch merge chain cost ~80 us."""
    rows, N = x.shape
    valid = N if valid is None else int(valid)
    if x.dtype == torch.bfloat16 and x.is_contiguous() and k <= 64 and N > 2048:
        c = next((c for c in range(-(-N // 2048), N // 8 + 1) if N % c == 0 and (N // c) % 8 == 0), 0)
        if c and c * k * 8 <= 65536:
            L = N // c
            cv = torch.empty(rows, c * k, device=x.device, dtype=torch.float32)
            ci = torch.empty(rows, c * k, device=x.device, dtype=torch.int32)
            check(lib().mls_topk_chunks(x.data_ptr(), cv.data_ptr(), ci.data_ptr(), rows, c, L, k, valid,
                                        stream_ptr(x.device)), "mls_topk_chunks")
            vals = torch.empty(rows, k, device=x.device, dtype=torch.float32)
            idx = torch.empty(rows, k, device=x.device, dtype=torch.int32)
            check(lib().mls_topk_merge(cv.data_ptr(), ci.data_ptr(), vals.data_ptr(), idx.data_ptr(), rows, c, k, L,
                                       int(lo), valid, stream_ptr(x.device)), "mls_topk_merge")
            return vals, idx
    if N <= max_chunk:
        vals, idx = softmax_topk(x, k, softmax=False)
    else:
        c = -(-N // max_chunk)
        while N % c:
            c += 1
        L = N // c
        vals, idx = softmax_topk(x.reshape(rows * c, L), k, softmax=False)
        vals = vals.view(rows, c * k)
        off = (torch.arange(c, device=x.device, dtype=torch.int32) * L).repeat_interleave(k)
        idx = idx.view(rows, c * k) + off
        tv, tp = torch.topk(vals, k, dim=-1)
        vals, idx = tv, idx.gather(1, tp)
    if valid < N:  # (approximate: the padded tail can displace candidates of its own chunk)
        vals = torch.where(idx < valid, vals, torch.full_like(vals, float("-inf")))
    return vals, idx + lo if lo else idx
