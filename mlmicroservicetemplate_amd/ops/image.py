"""GPU image decode (JPEG coefficient containers -> pixels) and test hooks."""
from __future__ import annotations

from typing import Optional

import torch

from ._lib import check, lib, stream_ptr
from ._core import _need, _ptr


IMAGE_CONTAINER_BYTES = 64 + 224 * 224 * 3  # frontend/csrc/jpeg_coefs.h CONTAINER_BYTES


IMAGE_SCRATCH_PER_IMAGE = 2 << 20  # jpeg_coefs.h SCRATCH_PER_IMAGE


def image_decode(containers: torch.Tensor, out: Optional[torch.Tensor] = None,
                 err: Optional[torch.Tensor] = None) -> torch.Tensor:
    """GPU half of the image path (csrc/image_decode.hip): ``[B, IMAGE_CONTAINER_BYTES]`` uint8
    containers (raw RGB, or host-Huffman-decoded JPEG coefficients + resize geometry) -> uint8
    ``[B, 224, 224, 3]``: IDCT, libjpeg chroma upsampling + YCbCr->RGB, Pillow's bilinear resize and
    the centre crop of ``plugins.builtin.decode_image``.  ``err`` (int32 ``[B]``, optional): row b is
    set to 1 when container b is unusable (that image comes out black), else 0 -- every launch, so
    a captured graph needs no clearing; :func:`fc_head` turns flagged rows into id -1 / NaN.
    Capturable (fixed launch geometry; the scratch comes from the caller's -- in a graph, the graph
    pool's -- allocator)."""
    dev = containers.device
    _need(containers, "containers", torch.uint8, dev)
    if containers.dim() != 2 or containers.shape[1] != IMAGE_CONTAINER_BYTES:
        raise ValueError(f"containers must be [B, {IMAGE_CONTAINER_BYTES}]")
    B = containers.shape[0]
    if out is None:
        out = torch.empty(B, 224, 224, 3, device=dev, dtype=torch.uint8)
    scratch = torch.empty(B * IMAGE_SCRATCH_PER_IMAGE, device=dev, dtype=torch.uint8)
    if err is not None:
        _need(err, "err", torch.int32, dev)
        if err.numel() < B:
            raise ValueError(f"err must have >= {B} elements (one flag per image)")
    rc = lib().mls_image_decode(containers.data_ptr(), out.data_ptr(), scratch.data_ptr(), IMAGE_SCRATCH_PER_IMAGE, B,
                                _ptr(err), stream_ptr(dev))
    check(rc, "mls_image_decode")
    return out


def gpu_sleep(us: int, device=None) -> None:
    """Hold the current stream of ``device`` for ``us`` microseconds (fault injection in tests)."""
    dev = torch.device(device if device is not None else "cuda")
    check(lib().mls_gpu_sleep(int(us), stream_ptr(dev)), "mls_gpu_sleep")


def h2d_pull(src: torch.Tensor, dst: torch.Tensor, blocks: int = 32) -> torch.Tensor:
    """Copy the pinned host tensor ``src`` into the device tensor ``dst`` with a kernel on the current
    stream (zero-copy reads over PCIe; capturable into a hipGraph).  Same byte size, 16-B multiple."""
    if src.is_cuda or not src.is_pinned() or not dst.is_cuda:
        raise ValueError("h2d_pull: src must be pinned host memory and dst a device tensor")
    if not (src.is_contiguous() and dst.is_contiguous()):
        raise ValueError("h2d_pull: contiguous tensors only")
    n = src.numel() * src.element_size()
    if n != dst.numel() * dst.element_size():
        raise ValueError("h2d_pull: size mismatch")
    check(lib().mls_h2d_pull(src.data_ptr(), dst.data_ptr(), n, int(blocks), stream_ptr(dst.device)), "mls_h2d_pull")
    return dst


def h2d_pull_cell(cell: torch.Tensor, nbytes: int, dst: torch.Tensor, blocks: int = 32) -> torch.Tensor:
    """Like :func:`h2d_pull`, but the source address is read when the kernel runs from ``cell`` (a
    pinned host int64 tensor of >= 1 element whose element 0 holds a pinned-buffer address with
    ``nbytes`` readable bytes).  Captured once, a graph then pulls from whichever pinned buffer the
    host wrote into the cell before the replay (engine/worker.py pre-staged batches)."""
    if cell.is_cuda or not cell.is_pinned() or cell.dtype != torch.int64 or not dst.is_cuda:
        raise ValueError("h2d_pull_cell: cell must be a pinned host int64 tensor and dst a device tensor")
    if not dst.is_contiguous() or nbytes != dst.numel() * dst.element_size():
        raise ValueError("h2d_pull_cell: dst must be contiguous and nbytes its byte size")
    check(lib().mls_h2d_pull_cell(cell.data_ptr(), dst.data_ptr(), int(nbytes), int(blocks), stream_ptr(dst.device)),
          "mls_h2d_pull_cell")
    return dst


def d2h_push(src: torch.Tensor, dst: torch.Tensor, blocks: int = 1) -> torch.Tensor:
    """Copy the device tensor ``src`` into the pinned host tensor ``dst`` with a kernel on the current
    stream (stores over PCIe; capturable).  Same byte size, 16-B multiple."""
    if not src.is_cuda or dst.is_cuda or not dst.is_pinned():
        raise ValueError("d2h_push: src must be a device tensor and dst pinned host memory")
    if not (src.is_contiguous() and dst.is_contiguous()):
        raise ValueError("d2h_push: contiguous tensors only")
    n = src.numel() * src.element_size()
    if n != dst.numel() * dst.element_size() or n % 16:
        raise ValueError("d2h_push: sizes must match and be a 16-B multiple")
    check(lib().mls_d2h_push(src.data_ptr(), dst.data_ptr(), n, int(blocks), stream_ptr(src.device)), "mls_d2h_push")
    return dst
