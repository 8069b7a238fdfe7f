"""Tensor-level wrappers over the hand-written CDNA4 kernels (T5).

Every op here runs the native HIP kernel on torch's current stream -- there is no eager
fallback for CUDA tensors (a missing library raises :class:`NativeError`).  The plain-PyTorch
oracles the kernels are tested against live in ``ops.reference``.

Layouts: activations NHWC / row-major ``[rows][features]`` bf16; conv weights
``[Cout][KH][KW][Cin]`` bf16 (see :func:`pack_conv_weight`); per-channel scale / bias fp32.
"""
from __future__ import annotations

import ctypes
import functools
import json
import os
from typing import Dict, List, Optional, Sequence, Tuple

import torch

from . import _lib  # noqa: F401  (re-exported: ops._lib.DEBUG, register_signatures)
from ._lib import NativeError, available, check, lib, stream_ptr

ACT_NONE, ACT_RELU, ACT_GELU, ACT_TANH, ACT_SILU, ACT_SILU_MUL = 0, 1, 2, 3, 4, 5
_ACTS = {None: 0, "none": 0, "relu": 1, "gelu": 2, "tanh": 3, "silu": 4, "silu_mul": 5}

__all__ = [
    "NativeError",
    "available",
    "lib",
    "conv2d_nhwc",
    "gemm",
    "normalize_u8",
    "maxpool2d_nhwc",
    "avgpool_global_nhwc",
    "bn_act",
    "softmax_topk",
    "softmax_rows",
    "pack_conv_weight",
    "conv_out_hw",
    "gemm_heuristic",
]


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


def pack_conv_weight(w_oihw: torch.Tensor, dtype=torch.bfloat16) -> torch.Tensor:
    """OIHW (PyTorch) -> ``[Cout][KH][KW][Cin]``.  Cin == 3 (image stem) is padded to 4 and KW to
    8 so one 16-byte chunk of the K dimension is two 4-channel taps (the kernel's stem mode)."""
    co, ci, kh, kw = w_oihw.shape
    w = w_oihw.permute(0, 2, 3, 1)
    if ci == 3 and kh > 1:
        w = torch.nn.functional.pad(w, (0, 1, 0, 8 - kw))  # Cin 3->4, KW -> 8
    return w.contiguous().to(dtype)


def _workspace_args(ws: Optional[torch.Tensor]):
    if ws is None:
        return None, 0
    return ws.data_ptr(), ws.numel() * ws.element_size()


# conv2d_nhwc ``cfg`` values that select the halo-tiled direct 3x3 kernel (csrc/conv3x3_halo.hip,
# variant 0 / 1) instead of an implicit-GEMM tile config; tuning-table values like any other.
CFG_HALO = 100
CFG_HALO_N32 = 101
CFG_HALO_XL = 102  # 512 output pixels x 64 channels per block, 4 x 4 MFMA tiles per wave
HALO_CFGS = (CFG_HALO, CFG_HALO_N32, CFG_HALO_XL)
# cfg values that select the pipelined halo kernel (csrc/conv3x3_pipe.hip): CFG_PIPE + variant;
# the tuning table's splitk carries the K split, MLS items per block ride in the upper digits of
# splitk (splitk = ks + 16 * (ipb - 1)).
CFG_PIPE = 110
PIPE_VARIANTS = 6
PIPE_CFGS = tuple(range(CFG_PIPE, CFG_PIPE + PIPE_VARIANTS))


def conv2d_nhwc(
    x: torch.Tensor,
    w: torch.Tensor,
    bias: Optional[torch.Tensor] = None,
    *,
    kernel: int,
    stride: int = 1,
    pad: int = 0,
    scale: Optional[torch.Tensor] = None,
    residual: Optional[torch.Tensor] = None,
    act=ACT_NONE,
    out: Optional[torch.Tensor] = None,
    workspace: Optional[torch.Tensor] = None,
    cfg: int = 0,
    splitk: int = 0,
) -> torch.Tensor:
    """``act(conv(x, w) * scale + bias (+ residual))`` with x NHWC bf16 and w packed
    ``[Cout][KH][KW][Cin]`` (stem: ``[Cout][KH][8][4]`` on a pre-padded 4-channel image, pad 0)."""
    dev = x.device
    _need(x, "x", torch.bfloat16, dev)
    _need(w, "w", torch.bfloat16, dev)
    B, H, W, C = x.shape
    cout = w.shape[0]
    kh = kw = kernel
    if C == 4 and kernel > 1:
        if tuple(w.shape) != (cout, kh, 8, 4):
            raise ValueError(f"stem weight must be [Cout,{kh},8,4], got {tuple(w.shape)}")
    elif tuple(w.shape) != (cout, kh, kw, C):
        raise ValueError(f"weight shape {tuple(w.shape)} != [{cout},{kh},{kw},{C}]")
    if cout % 8:
        raise ValueError("Cout must be a multiple of 8")
    ho, wo = conv_out_hw(H, W, kernel, stride, pad)
    if cfg in PIPE_CFGS:
        if kernel != 3 or stride != 1 or pad != 1 or scale is not None or residual is not None:
            raise ValueError("CFG_PIPE: 3x3 / stride 1 / pad 1 convolutions without a scale / residual only")
        ks, ipb = max(1, int(splitk)) % 16 or 1, max(1, int(splitk)) // 16 + 1
        return conv3x3_pipe(x, w, bias, act=act, out=out, variant=cfg - CFG_PIPE, splitk=ks, ipb=ipb,
                            workspace=workspace)
    if cfg in HALO_CFGS:
        if kernel != 3 or stride != 1 or pad != 1 or scale is not None:
            raise ValueError("CFG_HALO: 3x3 / stride 1 / pad 1 convolutions without a scale only")
        return conv3x3_halo(x, w, bias, act=act, residual=residual, out=out, variant=cfg - CFG_HALO,
                            splitk=splitk, workspace=workspace)
    for name, t in (("bias", bias), ("scale", scale)):
        if t is not None:
            _need(t, name, torch.float32, dev)
            if t.numel() != cout:
                raise ValueError(f"{name} must have {cout} elements")
    if residual is not None:
        _need(residual, "residual", torch.bfloat16, dev)
        if tuple(residual.shape) != (B, ho, wo, cout):
            raise ValueError(f"residual shape {tuple(residual.shape)} != {(B, ho, wo, cout)}")
    if out is None:
        out = torch.empty(B, ho, wo, cout, device=dev, dtype=torch.bfloat16)
    else:
        _need(out, "out", torch.bfloat16, dev)
        if tuple(out.shape) != (B, ho, wo, cout):
            raise ValueError("out has wrong shape")
    wsp, wsb = _workspace_args(workspace)
    rc = lib().mls_conv2d(
        x.data_ptr(), w.data_ptr(), _ptr(scale), _ptr(bias), _ptr(residual), out.data_ptr(), wsp, wsb,
        B, H, W, C, cout, kh, kw, stride, pad, _act(act), cfg, splitk, stream_ptr(dev),
    )
    check(rc, "mls_conv2d")
    return out


def conv1x1_dual(y: torch.Tensor, x: torch.Tensor, w_cat: torch.Tensor, bias: Optional[torch.Tensor] = None, *,
                 stride2: int = 1, act=ACT_NONE, out: Optional[torch.Tensor] = None,
                 workspace: Optional[torch.Tensor] = None, cfg: int = 0, splitk: int = 0) -> torch.Tensor:
    """``act(conv1x1(y, W_y) + conv1x1_stride2(x, W_x) + bias)`` as ONE GEMM over the concatenated
    reduction (``w_cat`` = ``[Cout][Cin_y + Cin_x]``): a ResNet bottleneck's last conv fused with its
    downsample projection, so the identity branch is never materialised."""
    dev = y.device
    _need(y, "y", torch.bfloat16, dev)
    _need(x, "x", torch.bfloat16, dev)
    _need(w_cat, "w_cat", torch.bfloat16, dev)
    B, Ho, Wo, C1 = y.shape
    B2, H2, W2, C2 = x.shape
    cout = w_cat.shape[0]
    if B2 != B or tuple(w_cat.shape) != (cout, C1 + C2) or conv_out_hw(H2, W2, 1, stride2, 0) != (Ho, Wo):
        raise ValueError("conv1x1_dual: inconsistent shapes")
    if C1 % 64 or C2 % 8 or cout % 8:
        raise ValueError("conv1x1_dual needs Cin_y % 64 == 0, Cin_x % 8 == 0, Cout % 8 == 0")
    if bias is not None:
        _need(bias, "bias", torch.float32, dev)
    if out is None:
        out = torch.empty(B, Ho, Wo, cout, device=dev, dtype=torch.bfloat16)
    wsp, wsb = _workspace_args(workspace)
    rc = lib().mls_conv2d_dual(y.data_ptr(), x.data_ptr(), w_cat.data_ptr(), _ptr(bias), out.data_ptr(), wsp, wsb,
                               B, Ho, Wo, C1, H2, W2, C2, stride2, cout, _act(act), cfg, splitk, stream_ptr(dev))
    check(rc, "mls_conv2d_dual")
    return out


# (K of the conv3 GEMM, N1, N2) csrc/conv_chain.hip is instantiated for
CHAIN_SHAPES = ((64, 256, 64), (128, 256, 64), (64, 256, 128), (128, 512, 128), (128, 512, 256), (256, 1024, 256))


def set_chain_l2_cw(cw: int) -> None:
    """A/B: output-channel chunk width of the layer2 chain boundaries (64 default, or 32)."""
    lib().mls_chain_set_l2_cw(int(cw))


def conv1x1_chain(a1: torch.Tensor, w3: torch.Tensor, b3: Optional[torch.Tensor], w1: torch.Tensor,
                  b1: Optional[torch.Tensor], *, residual: Optional[torch.Tensor] = None,
                  a2: Optional[torch.Tensor] = None, stride2: int = 1,
                  y_out: Optional[torch.Tensor] = None, t1_out: Optional[torch.Tensor] = None):
    """One bottleneck boundary in one kernel (csrc/conv_chain.hip):
    ``y = relu(conv1x1([a1 | a2 at stride2], w3) + b3 (+ residual))`` and
    ``t1 = relu(conv1x1(y, w1) + b1)``; y never makes an HBM round trip.  Returns ``(y, t1)``.
    ``w3`` is ``[N1][Ka (+ Kb)]`` (the dual concatenation when ``a2`` is given; no residual then),
    ``w1`` ``[N2][N1]``.  Supported (Ka + Kb, N1, N2): CHAIN_SHAPES -- the ResNet-50 layer1,
    layer2 and layer3 boundaries."""
    dev = a1.device
    _need(a1, "a1", torch.bfloat16, dev)
    _need(w3, "w3", torch.bfloat16, dev)
    _need(w1, "w1", torch.bfloat16, dev)
    B, Ho, Wo, Ka = a1.shape
    N1, N2 = w3.shape[0], w1.shape[0]
    if a2 is not None:
        _need(a2, "a2", torch.bfloat16, dev)
        if residual is not None:
            raise ValueError("conv1x1_chain: the dual form has no residual")
        B2, H2, W2, Kb = a2.shape
        if B2 != B or conv_out_hw(H2, W2, 1, stride2, 0) != (Ho, Wo):
            raise ValueError("conv1x1_chain: a2 does not match a1's grid at stride2")
    else:
        H2 = W2 = Kb = 0
    if w3.reshape(N1, -1).shape[1] != Ka + Kb or w1.reshape(N2, -1).shape[1] != N1:
        raise ValueError("conv1x1_chain: weight shapes do not chain")
    if (Ka + Kb, N1, N2) not in CHAIN_SHAPES:
        raise ValueError(f"conv1x1_chain: unsupported shape (K {Ka + Kb}, N1 {N1}, N2 {N2})")
    for name, t, n in (("b3", b3, N1), ("b1", b1, N2)):
        if t is not None:
            _need(t, name, torch.float32, dev)
            if t.numel() != n:
                raise ValueError(f"{name} must have {n} elements")
    if residual is not None:
        _need(residual, "residual", torch.bfloat16, dev)
        if tuple(residual.shape) != (B, Ho, Wo, N1):
            raise ValueError("residual shape mismatch")
    y = torch.empty(B, Ho, Wo, N1, device=dev, dtype=torch.bfloat16) if y_out is None else y_out
    t1 = torch.empty(B, Ho, Wo, N2, device=dev, dtype=torch.bfloat16) if t1_out is None else t1_out
    rc = lib().mls_conv_chain(a1.data_ptr(), _ptr(a2), w3.data_ptr(), _ptr(b3), _ptr(residual), y.data_ptr(),
                              w1.data_ptr(), _ptr(b1), t1.data_ptr(), B, Ho, Wo, Ka, H2, W2, Kb, stride2, N1, N2,
                              stream_ptr(dev))
    check(rc, "mls_conv_chain")
    return y, t1


def gemm(
    a: torch.Tensor,
    w: torch.Tensor,
    bias: Optional[torch.Tensor] = None,
    *,
    scale: Optional[torch.Tensor] = None,
    residual: Optional[torch.Tensor] = None,
    act=ACT_NONE,
    out: Optional[torch.Tensor] = None,
    workspace: Optional[torch.Tensor] = None,
    cfg: int = 0,
    splitk: int = 0,
) -> torch.Tensor:
    """``act(a @ w.T * scale + bias (+ residual))``; a ``[M,K]``, w ``[N,K]`` (nn.Linear layout).
    ``act="silu_mul"``: w rows are gate/up interleaved in groups of 8 (:func:`interleave_gate_up`)
    and the output is ``silu(gate) * up`` of width N/2."""
    dev = a.device
    _need(a, "a", torch.bfloat16, dev)
    _need(w, "w", torch.bfloat16, dev)
    M, K = a.shape
    N, K2 = w.shape
    if K != K2:
        raise ValueError(f"K mismatch {K} vs {K2}")
    if N % 8 or K % 8:
        raise ValueError("N and K must be multiples of 8")
    for name, t in (("bias", bias), ("scale", scale)):
        if t is not None:
            _need(t, name, torch.float32, dev)
            if t.numel() != N:
                raise ValueError(f"{name} must have {N} elements")
    if residual is not None:
        _need(residual, "residual", torch.bfloat16, dev)
        if tuple(residual.shape) != (M, N):
            raise ValueError("residual must be [M, N]")
    n_out = N // 2 if _act(act) == ACT_SILU_MUL else N
    if _act(act) == ACT_SILU_MUL and (N % 16 or scale is not None or residual is not None):
        raise ValueError("silu_mul needs N % 16 == 0 and no scale/residual")
    if out is None:
        out = torch.empty(M, n_out, device=dev, dtype=torch.bfloat16)
    else:
        _need(out, "out", torch.bfloat16, dev)
        if tuple(out.shape) != (M, n_out):
            raise ValueError(f"out must be [M, {n_out}]")
    wsp, wsb = _workspace_args(workspace)
    if M <= 16 and N % 16 == 0 and cfg == 0 and scale is None:
        # decode-shaped: weight-streaming skinny MFMA kernel (splitk <= 0 -> auto K split)
        rc = lib().mls_skinny_gemm(a.data_ptr(), w.data_ptr(), _ptr(bias), _ptr(residual), out.data_ptr(), wsp, wsb,
                                   M, N, K, _act(act), splitk, stream_ptr(dev))
        check(rc, "mls_skinny_gemm")
        return out
    rc = lib().mls_gemm(
        a.data_ptr(), w.data_ptr(), _ptr(scale), _ptr(bias), _ptr(residual), out.data_ptr(), wsp, wsb,
        M, N, K, _act(act), cfg, splitk, stream_ptr(dev),
    )
    check(rc, "mls_gemm")
    return out


GEMM_TILE_CFGS = {1: (256, 256), 2: (256, 128), 3: (128, 128), 4: (128, 128), 5: (128, 256), 6: (256, 256),
                  7: (256, 128), 8: (256, 256), 9: (256, 128), 10: (256, 256), 11: (256, 256), 12: (256, 128),
                  15: (256, 256), 16: (256, 128), 21: (192, 192), 22: (192, 192)}


_SPLIT_COUNTERS: Dict[Tuple[int, int], torch.Tensor] = {}
SPLIT_COUNTER_ELEMS = 1 << 14


def split_counters(workspace: torch.Tensor) -> torch.Tensor:
    """Zeroed int32 arrival counters of the in-launch split-K combine, one set per workspace buffer
    (= per stream: StreamWorkspace), allocated on first use (eager warm-up, before graph capture).
    Each tile's reducer resets its counter, so they stay zero between launches."""
    key = (workspace.device.index or 0, workspace.data_ptr())
    c = _SPLIT_COUNTERS.get(key)
    if c is None:
        c = torch.zeros(SPLIT_COUNTER_ELEMS, device=workspace.device, dtype=torch.int32)
        _SPLIT_COUNTERS[key] = c
    return c


def gemm_tile(a: torch.Tensor, w: torch.Tensor, bias: Optional[torch.Tensor] = None, *, act=ACT_NONE,
              residual: Optional[torch.Tensor] = None, out: Optional[torch.Tensor] = None, cfg: int = 0,
              grid_cap: int = 0, splitk: int = 1, workspace: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Large-M projection on the LDS-DMA MFMA tile kernel (csrc/gemm_tile.hip):
    ``act(a @ w.T + bias) (+ residual)``; SiLU-mul for gate/up interleaved in groups of 8.
    ``K % 64 == 0``, ``N % 16 == 0``; ``cfg`` selects the tile (:data:`GEMM_TILE_CFGS`, 0 = by shape).
    ``splitk > 1`` splits K and combines in the launch through fp32 slabs in ``workspace`` (falls back
    to no split when the workspace is missing or too small, or K does not divide)."""
    dev = a.device
    _need(a, "a", torch.bfloat16, dev)
    _need(w, "w", torch.bfloat16, dev)
    M, K = a.shape
    N, K2 = w.shape
    code = _act(act)
    if K != K2 or K % 64 or N % 16:
        raise ValueError(f"gemm_tile: K ({K} vs {K2}) % 64 == 0 and N ({N}) % 16 == 0")
    if bias is not None:
        _need(bias, "bias", torch.float32, dev)
        if bias.numel() != N:
            raise ValueError(f"bias must have {N} elements")
    if residual is not None:
        if code == ACT_SILU_MUL:
            raise ValueError("silu_mul takes no residual")
        _need(residual, "residual", torch.bfloat16, dev)
        if tuple(residual.shape) != (M, N):
            raise ValueError("residual must be [M, N]")
    n_out = N // 2 if code == ACT_SILU_MUL else N
    if out is None:
        out = torch.empty(M, n_out, device=dev, dtype=torch.bfloat16)
    else:
        _need(out, "out", torch.bfloat16, dev)
        if tuple(out.shape) != (M, n_out):
            raise ValueError(f"out must be [M, {n_out}]")
    sk, ws_ptr, ws_elems, cnt_ptr = 1, None, 0, None
    if splitk > 1 and workspace is not None and (cfg & 0xFF) in GEMM_TILE_CFGS:
        bm, bn = GEMM_TILE_CFGS[cfg & 0xFF]
        bks = 32 if (cfg & 0xFF) in (6, 7) else 64
        tiles = -(-M // bm) * -(-N // bn)
        if (K // bks) % splitk == 0 and tiles * splitk * bm * bn <= workspace.numel() \
                and tiles <= SPLIT_COUNTER_ELEMS and workspace.dtype == torch.float32:
            sk, ws_ptr, ws_elems, cnt_ptr = int(splitk), workspace.data_ptr(), workspace.numel(), \
                split_counters(workspace).data_ptr()
    rc = lib().mls_gemm_tile(a.data_ptr(), w.data_ptr(), _ptr(bias), _ptr(residual), out.data_ptr(), M, N, K, code,
                             n_out, N, int(cfg), int(grid_cap), sk, ws_ptr, ws_elems, cnt_ptr, SPLIT_COUNTER_ELEMS,
                             stream_ptr(dev))
    check(rc, "mls_gemm_tile")
    return out


_TUNED_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "tuned")
def load_blas_tuning(path: Optional[str] = None) -> bool:
    """Make hipBLASLt use the solutions PyTorch TunableOp measured fastest on MI355X for the shapes
    in ``tuned/tunableop_gfx950.csv`` (BERT FFN-up + GELU: 26.4 vs 30.1 us at 4-way concurrency,
    ``profiles/r1_bert_gemm_probe.jsonl``).  Lookup only -- tuning stays off, so nothing is timed or
    written at run time, and untuned shapes keep the library default.  ``MLS_BLAS_TUNING=0``
    disables it; ``MLS_BLAS_TUNING_FILE`` reads another table (A/B).  Returns whether it loaded."""
    if os.environ.get("MLS_BLAS_TUNING", "1") == "0" or not torch.cuda.is_available():
        return False
    from torch.cuda import tunable

    tunable.enable(True)
    tunable.tuning_enable(False)
    path = path or os.environ.get("MLS_BLAS_TUNING_FILE") or os.path.join(_TUNED_DIR, "tunableop_gfx950.csv")
    ok = bool(tunable.read_file(path))
    if not ok:
        tunable.enable(False)
    return ok


def gemm_rmsnorm(x: torch.Tensor, w_folded: torch.Tensor, delta: Optional[torch.Tensor] = None,
                 resid_out: Optional[torch.Tensor] = None, *, act=ACT_NONE, eps: float = 1e-5,
                 workspace: Optional[torch.Tensor] = None, splitk: int = 0) -> torch.Tensor:
    """Decode-shaped (M <= 32) ``act(RMSNorm(x + delta) @ W^T)`` in ONE launch, with the RMSNorm gain
    pre-folded into ``w_folded`` (:func:`fold_norm`); ``x + delta`` is also written to ``resid_out``
    (a buffer distinct from ``x``/``delta``) when given."""
    dev = x.device
    _need(x, "x", torch.bfloat16, dev)
    _need(w_folded, "w", torch.bfloat16, dev)
    M, K = x.shape
    N = w_folded.shape[0]
    if M > 32 or N % 16 or w_folded.shape[1] != K:
        raise ValueError("gemm_rmsnorm: M <= 32, N % 16 == 0, matching K")
    for name, t in (("delta", delta), ("resid_out", resid_out)):
        if t is not None:
            _need(t, name, torch.bfloat16, dev)
            if tuple(t.shape) != (M, K):
                raise ValueError(f"{name} must be [M, K]")
    if resid_out is not None and delta is None:
        raise ValueError("resid_out needs delta")
    code = _act(act)
    out = torch.empty(M, N // 2 if code == ACT_SILU_MUL else N, device=dev, dtype=torch.bfloat16)
    wsp, wsb = _workspace_args(workspace)
    rc = lib().mls_skinny_gemm_norm(x.data_ptr(), _ptr(delta), _ptr(resid_out), w_folded.data_ptr(), None, None,
                                    out.data_ptr(), wsp, wsb, M, N, K, code, splitk, 1, float(eps), stream_ptr(dev))
    check(rc, "mls_skinny_gemm_norm")
    return out


def pack_skinny(w: torch.Tensor) -> torch.Tensor:
    """``w [N, K]`` -> the packed 1 KiB-granule layout of :func:`skinny_packed` (same bytes, flat)."""
    _need(w, "w", torch.bfloat16, w.device)
    N, K = w.shape
    if N % 16 or K % 32:
        raise ValueError("pack_skinny: N % 16 == 0 and K % 32 == 0")
    wp = torch.empty(N * K, device=w.device, dtype=torch.bfloat16)
    check(lib().mls_skinny_pack(w.data_ptr(), wp.data_ptr(), N, K, stream_ptr(w.device)), "mls_skinny_pack")
    return wp


def pack_skinny_reference(w: torch.Tensor) -> torch.Tensor:
    """PyTorch form of the packed layout: ``[N/16][K/32][4][16][8]`` flattened."""
    N, K = w.shape
    return w.reshape(N // 16, 16, K // 32, 4, 8).permute(0, 2, 3, 1, 4).reshape(-1).contiguous()


def skinny_packed(x: torch.Tensor, wp: torch.Tensor, N: int, *, delta: Optional[torch.Tensor] = None,
                  resid_out: Optional[torch.Tensor] = None, norm: bool = False, act=ACT_NONE,
                  bias: Optional[torch.Tensor] = None, residual: Optional[torch.Tensor] = None,
                  eps: float = 1e-5, variant: int = 9, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Decode product (M <= 32) against a :func:`pack_skinny` weight: ``act([RMSNorm](x [+ delta]) @ W^T + b
    [+ residual])``; with ``norm`` the RMSNorm gain must be folded into W (:func:`fold_norm`)."""
    dev = x.device
    _need(x, "x", torch.bfloat16, dev)
    _need(wp, "wp", torch.bfloat16, dev)
    M, K = x.shape
    if M > 32 or N % 16 or K % 32 or wp.numel() != N * K:
        raise ValueError("skinny_packed: M <= 32, N % 16 == 0, K % 32 == 0, wp of N*K elements")
    if resid_out is not None and delta is None:
        raise ValueError("resid_out needs delta")
    if (delta is not None) and not norm:
        raise ValueError("delta exists only with norm")
    for name, t in (("delta", delta), ("resid_out", resid_out)):
        if t is not None:
            _need(t, name, torch.bfloat16, dev)
            if tuple(t.shape) != (M, K):
                raise ValueError(f"{name} must be [M, K]")
    if bias is not None:
        _need(bias, "bias", torch.float32, dev)
    if residual is not None:
        _need(residual, "residual", torch.bfloat16, dev)
        if tuple(residual.shape) != (M, N):
            raise ValueError("residual must be [M, N]")
    code = _act(act)
    n_out = N // 2 if code == ACT_SILU_MUL else N
    if out is None:
        out = torch.empty(M, n_out, device=dev, dtype=torch.bfloat16)
    elif tuple(out.shape) != (M, n_out) or out.dtype != torch.bfloat16 or not out.is_contiguous():
        raise ValueError(f"out must be contiguous bf16 [M, {n_out}]")
    rc = lib().mls_skinny_packed(x.data_ptr(), _ptr(delta), _ptr(resid_out), wp.data_ptr(), _ptr(bias),
                                 _ptr(residual), out.data_ptr(), M, N, K, code, int(norm), float(eps), int(variant),
                                 stream_ptr(dev))
    check(rc, "mls_skinny_packed")
    return out


FP8_MAX = 448.0  # OCP e4m3fn


def pack_skinny_fp8(w: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    """``w [N, K]`` -> (fp8 e4m3 weights in the 1 KiB granule layout of :func:`skinny_fp8`
    (``[N/16][K/64][4][16][2][8]`` bytes, flat uint8), per-row fp32 scales ``max|w[n]| / 448``)."""
    N, K = w.shape
    if N % 16 or K % 64:
        raise ValueError("pack_skinny_fp8: N % 16 == 0 and K % 64 == 0")
    wf = w.float()
    scale = (wf.abs().amax(1) / FP8_MAX).clamp_min(1e-12)
    q = (wf / scale[:, None]).to(torch.float8_e4m3fn)
    q = q.view(N // 16, 16, K // 64, 2, 4, 8).permute(0, 2, 4, 1, 3, 5).contiguous()
    return q.view(torch.uint8).reshape(-1), scale.contiguous()


def fp8_reference(x: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    """fp32 emulation of :func:`skinny_fp8`'s W8A8 product (per-row x scale, per-row w scale)."""
    xf, wf = x.float(), w.float()
    sx = (xf.abs().amax(1, keepdim=True) / FP8_MAX).clamp_min(1e-30)
    sw = (wf.abs().amax(1, keepdim=True) / FP8_MAX).clamp_min(1e-12)
    xq = (xf / sx).to(torch.float8_e4m3fn).float() * sx
    wq = (wf / sw).to(torch.float8_e4m3fn).float() * sw
    return xq @ wq.T


def skinny_fp8(x: torch.Tensor, wq: torch.Tensor, wscale: torch.Tensor, N: int, *,
               delta: Optional[torch.Tensor] = None, resid_out: Optional[torch.Tensor] = None, norm: bool = False,
               act=ACT_NONE, bias: Optional[torch.Tensor] = None, residual: Optional[torch.Tensor] = None,
               eps: float = 1e-5, variant: int = 1) -> torch.Tensor:
    """FP8 (W8A8, e4m3) decode product, M <= 4: ``act([RMSNorm](x [+ delta]) @ W^T + b [+ residual])``
    with W from :func:`pack_skinny_fp8` (the RMSNorm gain folded into W before packing) and the
    activation rows quantised per row inside the kernel.  Half the weight bytes of :func:`skinny_packed`."""
    dev = x.device
    _need(x, "x", torch.bfloat16, dev)
    M, K = x.shape
    if M > 4 or N % 16 or K % 64 or wq.numel() != N * K or M * K * 2 > 65536:
        raise ValueError("skinny_fp8: M <= 4, N % 16 == 0, K % 64 == 0, M * K * 2 <= 64 KiB, wq of N*K bytes")
    _need(wscale, "wscale", torch.float32, dev)
    if resid_out is not None and delta is None:
        raise ValueError("resid_out needs delta")
    if delta is not None and not norm:
        raise ValueError("delta exists only with norm")
    for name, t in (("delta", delta), ("resid_out", resid_out)):
        if t is not None:
            _need(t, name, torch.bfloat16, dev)
            if tuple(t.shape) != (M, K):
                raise ValueError(f"{name} must be [M, K]")
    if bias is not None:
        _need(bias, "bias", torch.float32, dev)
    if residual is not None:
        _need(residual, "residual", torch.bfloat16, dev)
        if tuple(residual.shape) != (M, N):
            raise ValueError("residual must be [M, N]")
    code = _act(act)
    out = torch.empty(M, N // 2 if code == ACT_SILU_MUL else N, device=dev, dtype=torch.bfloat16)
    rc = lib().mls_skinny_fp8(x.data_ptr(), _ptr(delta), _ptr(resid_out), wq.data_ptr(), wscale.data_ptr(),
                              _ptr(bias), _ptr(residual), out.data_ptr(), M, N, K, code, int(norm), float(eps),
                              int(variant), stream_ptr(dev))
    check(rc, "mls_skinny_fp8")
    return out


def fold_norm(w: torch.Tensor, gain: torch.Tensor) -> torch.Tensor:
    """``W[:, k] * gain[k]`` in fp32, rounded once to bf16: RMSNorm(x) @ W^T == rstd * (x @ fold^T)."""
    return (w.float() * gain.float().view(1, -1)).to(w.dtype)


# Large-M projections run on the native LDS-DMA MFMA tile kernel (gemm_tile: csrc/gemm_tile.hip),
# the decode-shaped ones (M <= 32, and 33..TILE_MIN_M - 1 rows) on the skinny / conv_gemm kernels with
# per-shape plans.  hipBLASLt (torch.addmm) is reachable only on request -- impl="blas" or
# MLS_GEMM_IMPL=blas -- as the A/B reference of tools/gemm_tile_probe.py; no default path calls it.
TILE_MIN_M = int(os.environ.get("MLS_TILE_MIN_M", "256"))
BLAS_MIN_M = TILE_MIN_M  # kept for callers that split "large" from "small" token counts
_GEMM_IMPL = os.environ.get("MLS_GEMM_IMPL", "native")
_BF16_BIAS: dict = {}
def _bias_bf16(bias: torch.Tensor) -> torch.Tensor:
    key = (bias.data_ptr(), bias.numel(), bias.device)
    hit = _BF16_BIAS.get(key)
    if hit is None or hit[0] is not bias:
        hit = (bias, bias.to(torch.bfloat16))
        _BF16_BIAS[key] = hit
    return hit[1]


def silu_mul_interleaved(x: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """``[M, 2I]`` gate/up interleaved in groups of 8 -> ``silu(gate) * up`` ``[M, I]``."""
    _need(x, "x", torch.bfloat16, x.device)
    M, N2 = x.shape
    if out is None:
        out = torch.empty(M, N2 // 2, device=x.device, dtype=torch.bfloat16)
    check(lib().mls_silu_mul_interleaved(x.data_ptr(), out.data_ptr(), M, N2 // 2, stream_ptr(x.device)),
          "mls_silu_mul_interleaved")
    return out


@functools.lru_cache(maxsize=None)
def gemm_plan() -> Dict[Tuple[int, int, int], Tuple[int, int]]:
    """Measured per-shape choices for :func:`linear` (``tuned/gemm_plan_gfx950.json``): exact
    ``(M, N, K)`` -> ``(cfg, splitk)`` of the native kernel, cfg 0 = hipBLASLt.  ``MLS_GEMM_PLAN=0``
    disables it."""
    if os.environ.get("MLS_GEMM_PLAN", "1") == "0":
        return {}
    with open(os.path.join(_TUNED_DIR, "gemm_plan_gfx950.json")) as f:
        doc = json.load(f)
    return {(e["M"], e["N"], e["K"]): (int(e["plan"][0]), int(e["plan"][1])) for e in doc["entries"]}


def tile_cfg_for(M: int, N: int, K: int) -> Tuple[int, int]:
    """gemm_tile (config, K splits) for a shape: measured choices first (``tuned/gemm_tile_gfx950.json``),
    else the kernel's own pick (largest tile that still fills the chip), no split."""
    e = gemm_tile_plan().get((M, N, K))
    return e if e is not None else (0, 1)


@functools.lru_cache(maxsize=None)
def gemm_tile_plan() -> Dict[Tuple[int, int, int], Tuple[int, int]]:
    path = os.environ.get("MLS_GEMM_TILE_TABLE") or os.path.join(_TUNED_DIR, "gemm_tile_gfx950.json")
    if os.environ.get("MLS_GEMM_PLAN", "1") == "0" or not os.path.exists(path):
        return {}
    with open(path) as f:
        doc = json.load(f)
    return {(e["M"], e["N"], e["K"]): (int(e["cfg"]), int(e.get("splitk", 1))) for e in doc["entries"]}


def linear(a: torch.Tensor, w: torch.Tensor, bias: Optional[torch.Tensor] = None, *, act=ACT_NONE,
           residual: Optional[torch.Tensor] = None, workspace: Optional[torch.Tensor] = None,
           impl: str = "auto") -> torch.Tensor:
    """Transformer projection ``act(a @ w.T + bias) (+ residual)``, all native: M >= TILE_MIN_M on the
    persistent LDS-DMA tile kernel (:func:`gemm_tile`, bias / GELU / SiLU-mul / residual in its
    epilogue), smaller M on the skinny / conv_gemm kernels (measured per-shape plans in
    ``tuned/gemm_plan_gfx950.json``).  ``impl``: "auto" | "native" | "tile" | "blas" (hipBLASLt, the
    A/B reference only; also ``MLS_GEMM_IMPL=blas``)."""
    code = _act(act)
    M, K = a.shape
    N = w.shape[0]
    if impl == "blas" or (impl == "auto" and _GEMM_IMPL == "blas"):
        return _linear_blas(a, w, bias, code, residual)
    if impl == "tile" or (impl == "auto" and M >= TILE_MIN_M and K % 64 == 0 and N % 16 == 0
                          and a.device.type == "cuda" and a.is_contiguous() and w.is_contiguous()):
        cfg, sk = tile_cfg_for(M, N, K)
        return gemm_tile(a, w, bias, act=code, residual=residual, cfg=cfg, splitk=sk, workspace=workspace)
    plan = gemm_plan().get((M, N, K)) if impl == "auto" else None
    if plan is not None and plan[0] > 0 and not (code == ACT_SILU_MUL and residual is not None):
        return gemm(a, w, bias, act=code, residual=residual, workspace=workspace, cfg=plan[0], splitk=plan[1])
    return gemm(a, w, bias, act=code, residual=residual, workspace=workspace)


def _linear_blas(a, w, bias, code, residual):
    """hipBLASLt through torch (A/B reference; bias / GELU epilogues, SiLU-mul as a native pass)."""
    b16 = _bias_bf16(bias) if bias is not None else None
    if code == ACT_GELU:
        y = torch._addmm_activation(b16 if b16 is not None else torch.zeros(w.shape[0], device=a.device,
                                    dtype=torch.bfloat16), a, w.t(), use_gelu=True)
    elif residual is not None and b16 is None:
        y = torch.addmm(residual, a, w.t())
        residual = None
    elif b16 is not None:
        y = torch.addmm(b16, a, w.t())
    else:
        y = torch.mm(a, w.t())
    if code not in (ACT_NONE, ACT_GELU, ACT_SILU_MUL):
        raise ValueError("blas path: act must be none / gelu / silu_mul")
    if residual is not None:
        y += residual
    if code == ACT_SILU_MUL:
        y = silu_mul_interleaved(y)
    return y


def interleave_gate_up(gate: torch.Tensor, up: torch.Tensor) -> torch.Tensor:
    """``[I, K]`` gate and up projections -> ``[2I, K]`` rows interleaved in groups of 8
    (gate 0-7, up 0-7, gate 8-15, ...), the layout of the fused SiLU-mul GEMM epilogue."""
    I, K = gate.shape
    if I % 8:
        raise ValueError("intermediate size must be a multiple of 8")
    return torch.stack([gate.view(I // 8, 8, K), up.view(I // 8, 8, K)], dim=1).reshape(2 * I, K).contiguous()


def gemm_heuristic(M: int, N: int, K: int) -> Tuple[int, int]:
    cfg, sk = ctypes.c_int(0), ctypes.c_int(0)
    lib().mls_gemm_heuristic(M, N, K, ctypes.byref(cfg), ctypes.byref(sk))
    return cfg.value, sk.value


_MEAN_STD_CACHE = {}


def normalize_u8(images: torch.Tensor, mean, std, pad: int = 0, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """uint8 ``[B,H,W,3]`` -> bf16 ``[B,H+2p,W+2p,4]`` = ((x - mean) / std, 0) with a zero border
    of ``pad`` pixels (the stem conv is then launched with pad 0 on the pre-padded image)."""
    dev = images.device
    _need(images, "images", torch.uint8, dev)
    B, H, W, C = images.shape
    if C != 3:
        raise ValueError("expected 3-channel images")
    shape = (B, H + 2 * pad, W + 2 * pad, 4)
    if out is None:
        out = torch.empty(shape, device=dev, dtype=torch.bfloat16)
    else:
        _need(out, "out", torch.bfloat16, dev)
        if tuple(out.shape) != shape:
            raise ValueError(f"out must be {shape}")
    m = (ctypes.c_float * 3)(*[float(v) for v in mean])
    s = (ctypes.c_float * 3)(*[float(v) for v in std])
    rc = lib().mls_normalize_u8(images.data_ptr(), out.data_ptr(), B, H, W, pad, m, s, stream_ptr(dev))
    check(rc, "mls_normalize_u8")
    return out


def stem_pool_u8(images: torch.Tensor, w: torch.Tensor, bias: torch.Tensor, mean, std,
                 out: Optional[torch.Tensor] = None, conv1_w: Optional[torch.Tensor] = None,
                 conv1_b: Optional[torch.Tensor] = None):
    """ResNet input block in one kernel: uint8 ``[B,224,224,3]`` -> normalise -> 7x7/2 conv
    (packed ``[64,7,8,4]`` weights, BN folded) + bias -> ReLU -> 3x3/2 max pool -> bf16
    ``[B,56,56,64]`` (csrc/stem_pool.hip).  With ``conv1_w`` (``[64, 64]`` or ``[64,1,1,64]``, BN
    folded) / ``conv1_b`` the first bottleneck's 1x1 conv + ReLU runs on each pooled tile in the
    same kernel and ``(pooled, t1)`` is returned."""
    dev = images.device
    _need(images, "images", torch.uint8, dev)
    _need(w, "w", torch.bfloat16, dev)
    _need(bias, "bias", torch.float32, dev)
    B, H, W, C = images.shape
    if C != 3 or H != 224 or W != 224 or tuple(w.shape) != (64, 7, 8, 4) or bias.numel() != 64:
        raise ValueError("stem_pool_u8: 224x224x3 images, [64,7,8,4] weights, 64 biases")
    shape = (B, 56, 56, 64)
    if out is None:
        out = torch.empty(shape, device=dev, dtype=torch.bfloat16)
    else:
        _need(out, "out", torch.bfloat16, dev)
        if tuple(out.shape) != shape:
            raise ValueError(f"out must be {shape}")
    m = (ctypes.c_float * 3)(*[float(v) for v in mean])
    s = (ctypes.c_float * 3)(*[float(v) for v in std])
    if conv1_w is None:
        check(lib().mls_stem_pool(images.data_ptr(), w.data_ptr(), bias.data_ptr(), out.data_ptr(), B, H, W, m, s,
                                  stream_ptr(dev)), "mls_stem_pool")
        return out
    _need(conv1_w, "conv1_w", torch.bfloat16, dev)
    if conv1_w.numel() != 64 * 64 or conv1_w.shape[0] != 64:
        raise ValueError("stem_pool_u8: conv1_w must be [64, 64] (Cout x Cin)")
    if conv1_b is not None:
        _need(conv1_b, "conv1_b", torch.float32, dev)
        if conv1_b.numel() != 64:
            raise ValueError("conv1_b must have 64 elements")
    t1 = torch.empty(shape, device=dev, dtype=torch.bfloat16)
    check(lib().mls_stem_pool_conv1(images.data_ptr(), w.data_ptr(), bias.data_ptr(), out.data_ptr(), B, H, W, m, s,
                                    conv1_w.data_ptr(), _ptr(conv1_b), t1.data_ptr(), stream_ptr(dev)),
          "mls_stem_pool_conv1")
    return out, t1


def conv3x3_halo(x: torch.Tensor, w: torch.Tensor, bias: Optional[torch.Tensor] = None, *, act=ACT_NONE,
                 residual: Optional[torch.Tensor] = None, out: Optional[torch.Tensor] = None,
                 variant: int = 0, splitk: int = 1, workspace: Optional[torch.Tensor] = None) -> torch.Tensor:
    """3x3 / stride 1 / pad 1 NHWC conv on the halo-tiled direct kernel (csrc/conv3x3_halo.hip):
    x ``[B,H,W,Cin]`` bf16, w packed ``[N,3,3,Cin]`` bf16, bias fp32 ``[N]`` -> ``[B,H,W,N]``
    ``act(conv + bias (+ residual))``.  Cin % 32 == 0; ``variant`` 0 = 64 output channels x 8
    waves per block (N % 64 == 0), 1 = 32 x 4 (N % 32 == 0), 2 = the XL tile (512 output pixels
    x 64 channels, 8 waves of 4 x 4 MFMA tiles).  ``splitk`` > 1 splits the input
    channels over that many blocks per tile, reduced in the same launch through fp32 slabs in
    ``workspace`` (>= splitk * B*H*W * N floats; otherwise, or on an uneven split, one slice)."""
    dev = x.device
    _need(x, "x", torch.bfloat16, dev)
    _need(w, "w", torch.bfloat16, dev)
    B, H, W, C = x.shape
    N = w.shape[0]
    if tuple(w.shape) != (N, 3, 3, C) or C % 32 or N % (32 if variant == 1 else 64) or variant not in (0, 1, 2):
        raise ValueError("conv3x3_halo: w must be [N,3,3,Cin], Cin % 32 == 0, N % 64 (variant 1: 32) == 0")
    if bias is not None:
        _need(bias, "bias", torch.float32, dev)
        if bias.numel() != N:
            raise ValueError("bias must have N elements")
    shape = (B, H, W, N)
    if residual is not None:
        _need(residual, "residual", torch.bfloat16, dev)
        if tuple(residual.shape) != shape:
            raise ValueError(f"residual must be {shape}")
    if out is None:
        out = torch.empty(shape, device=dev, dtype=torch.bfloat16)
    else:
        _need(out, "out", torch.bfloat16, dev)
        if tuple(out.shape) != shape:
            raise ValueError(f"out must be {shape}")
    wsp, wsb = _workspace_args(workspace)
    check(lib().mls_conv3x3_halo(x.data_ptr(), w.data_ptr(), _ptr(bias), _ptr(residual), out.data_ptr(), wsp, wsb,
                                 B, H, W, C, N, _act(act), variant, max(1, int(splitk)), stream_ptr(dev)),
          "mls_conv3x3_halo")
    return out


def conv2d_pool(x: torch.Tensor, w: torch.Tensor, bias: Optional[torch.Tensor], pool: torch.Tensor, *, kernel: int,
                stride: int = 1, pad: int = 0, residual: Optional[torch.Tensor] = None, act=ACT_NONE,
                out: Optional[torch.Tensor] = None, pool_only: bool = True, cfg: int = 0) -> Optional[torch.Tensor]:
    """``conv2d_nhwc`` with the global average pool of its output fused into the epilogue (the
    network's last convolution, csrc/conv_gemm.hip ``ConvArgs::pool``): ``pool`` fp32 ``[B, Cout]``
    += the per-image mean of ``act(conv + bias (+ residual))``.  ``pool`` must be zero on entry
    (:func:`fc_head` zeroes it after reading); with ``pool_only`` the output is not written."""
    dev = x.device
    _need(x, "x", torch.bfloat16, dev)
    _need(w, "w", torch.bfloat16, dev)
    _need(pool, "pool", torch.float32, dev)
    B, H, W, C = x.shape
    cout = w.shape[0]
    if tuple(w.shape) != (cout, kernel, kernel, C) or C == 4:
        raise ValueError(f"weight shape {tuple(w.shape)} != [{cout},{kernel},{kernel},{C}]")
    ho, wo = conv_out_hw(H, W, kernel, stride, pad)
    if pool.shape[0] < B or pool.shape[-1] != cout:
        raise ValueError(f"pool must be [>= {B}, {cout}]")
    if bias is not None:
        _need(bias, "bias", torch.float32, dev)
    if residual is not None:
        _need(residual, "residual", torch.bfloat16, dev)
        if tuple(residual.shape) != (B, ho, wo, cout):
            raise ValueError("residual shape mismatch")
    if not pool_only and out is None:
        out = torch.empty(B, ho, wo, cout, device=dev, dtype=torch.bfloat16)
    check(lib().mls_conv2d_pool(x.data_ptr(), w.data_ptr(), None, _ptr(bias), _ptr(residual), _ptr(out),
                                pool.data_ptr(), int(pool_only), B, H, W, C, cout, kernel, kernel, stride, pad,
                                _act(act), int(cfg), stream_ptr(dev)), "mls_conv2d_pool")
    return out


def fc_head(pooled: torch.Tensor, w: torch.Tensor, bias: Optional[torch.Tensor], k: int, *,
            logits: Optional[torch.Tensor] = None, softmax: bool = True, err: Optional[torch.Tensor] = None,
            vals: Optional[torch.Tensor] = None, idx: Optional[torch.Tensor] = None):
    """Classifier head in one launch (csrc/head.hip): ``pooled`` fp32 ``[B, K]`` (the fused average
    pool; ZEROED by this call for the next forward) -> logits = pooled . w^T + bias (fp32, into
    ``logits``) -> (softmax ->) top-``k``.  ``err`` int32 ``[B]``: rows flagged nonzero come back
    with ids -1 and NaN values (an undecodable upload).  Returns (vals fp32 [B,k], ids int32 [B,k],
    logits); with ``k == 0`` only the logits."""
    dev = pooled.device
    _need(pooled, "pooled", torch.float32, dev)
    _need(w, "w", torch.bfloat16, dev)
    B, K = pooled.shape
    N = w.shape[0]
    if w.shape[1] != K:
        raise ValueError("w must be [N, K]")
    if bias is not None:
        _need(bias, "bias", torch.float32, dev)
    if logits is None:
        logits = torch.empty(B, N, device=dev, dtype=torch.float32)
    _need(logits, "logits", torch.float32, dev)
    if logits.numel() < B * N:
        raise ValueError("logits buffer too small")
    if err is not None:
        _need(err, "err", torch.int32, dev)
    if k > 0:
        if vals is None:
            vals = torch.empty(B, k, device=dev, dtype=torch.float32)
        if idx is None:
            idx = torch.empty(B, k, device=dev, dtype=torch.int32)
    check(lib().mls_fc_head(pooled.data_ptr(), w.data_ptr(), _ptr(bias), logits.data_ptr(), _ptr(vals), _ptr(idx),
                            _ptr(err), B, N, K, int(k), int(softmax), stream_ptr(dev)), "mls_fc_head")
    return vals, idx, logits


def conv3x3_pipe(x: torch.Tensor, w: torch.Tensor, bias: Optional[torch.Tensor] = None, *, act=ACT_NONE,
                 out: Optional[torch.Tensor] = None, variant: int = 0, splitk: int = 1, ipb: int = 1,
                 workspace: Optional[torch.Tensor] = None) -> torch.Tensor:
    """3x3 / stride 1 / pad 1 NHWC conv on the pipelined halo kernel (csrc/conv3x3_pipe.hip):
    x ``[B,H,W,Cin]`` bf16, w packed ``[N,3,3,Cin]`` bf16, bias fp32 ``[N]`` -> ``[B,H,W,N]``
    ``act(conv + bias)`` (act: none / ReLU).  ``variant`` picks (channels per item, waves, row
    blocks per wave, ring stages); ``splitk`` > 1 splits the input channels over that many items
    per tile (in-launch reduction through fp32 slabs in ``workspace``, >= splitk * B*H*W*N floats;
    otherwise one slice); ``ipb`` = consecutive items per block."""
    dev = x.device
    _need(x, "x", torch.bfloat16, dev)
    _need(w, "w", torch.bfloat16, dev)
    B, H, W, C = x.shape
    N = w.shape[0]
    if tuple(w.shape) != (N, 3, 3, C) or C % 32 or N % 32 or N > 512 or not 0 <= variant < PIPE_VARIANTS:
        raise ValueError("conv3x3_pipe: w must be [N,3,3,Cin], Cin % 32 == 0, N % 32 == 0, N <= 512")
    if act not in (ACT_NONE, ACT_RELU, "none", "relu"):
        raise ValueError("conv3x3_pipe: act must be none or relu")
    if bias is not None:
        _need(bias, "bias", torch.float32, dev)
        if bias.numel() != N:
            raise ValueError("bias must have N elements")
    shape = (B, H, W, N)
    if out is None:
        out = torch.empty(shape, device=dev, dtype=torch.bfloat16)
    else:
        _need(out, "out", torch.bfloat16, dev)
        if tuple(out.shape) != shape:
            raise ValueError(f"out must be {shape}")
    wsp, wsb = _workspace_args(workspace)
    check(lib().mls_conv3x3_pipe(x.data_ptr(), w.data_ptr(), _ptr(bias), out.data_ptr(), wsp, wsb, B, H, W, C, N,
                                 _act(act), int(variant), max(1, int(splitk)), max(1, int(ipb)), stream_ptr(dev)),
          "mls_conv3x3_pipe")
    return out


def conv3x3_pipe_geometry(B: int, H: int, W: int, variant: int = 0) -> Optional[Tuple[int, int]]:
    """(output rows per item, images per item) of the pipelined kernel's variant, or None."""
    th, nb = ctypes.c_int(0), ctypes.c_int(0)
    rc = lib().mls_conv3x3_pipe_geometry(B, H, W, variant, ctypes.byref(th), ctypes.byref(nb))
    return (th.value, nb.value) if rc == 0 else None


def conv3x3_halo_geometry(B: int, H: int, W: int, variant: int = 0) -> Optional[Tuple[int, int]]:
    """(output rows per tile, images per tile) the halo kernel uses for this shape, or None."""
    th, nb = ctypes.c_int(0), ctypes.c_int(0)
    rc = lib().mls_conv3x3_halo_geometry_v(B, H, W, variant, ctypes.byref(th), ctypes.byref(nb))
    return (th.value, nb.value) if rc == 0 else None


def maxpool2d_nhwc(x: torch.Tensor, k: int = 3, s: int = 2, p: int = 1, out: Optional[torch.Tensor] = None):
    dev = x.device
    _need(x, "x", torch.bfloat16, dev)
    B, H, W, C = x.shape
    ho, wo = conv_out_hw(H, W, k, s, p)
    if out is None:
        out = torch.empty(B, ho, wo, C, device=dev, dtype=torch.bfloat16)
    rc = lib().mls_maxpool2d(x.data_ptr(), out.data_ptr(), B, H, W, C, k, s, p, stream_ptr(dev))
    check(rc, "mls_maxpool2d")
    return out


def avgpool_global_nhwc(x: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    dev = x.device
    _need(x, "x", torch.bfloat16, dev)
    B, H, W, C = x.shape
    if out is None:
        out = torch.empty(B, C, device=dev, dtype=torch.bfloat16)
    rc = lib().mls_avgpool_global(x.data_ptr(), out.data_ptr(), B, H * W, C, stream_ptr(dev))
    check(rc, "mls_avgpool_global")
    return out


def bn_act(x: torch.Tensor, scale: torch.Tensor, bias: torch.Tensor, relu: bool = False, out=None) -> torch.Tensor:
    """Standalone inference BatchNorm over the last (channel) dim (K3 unfused path)."""
    dev = x.device
    _need(x, "x", torch.bfloat16, dev)
    _need(scale, "scale", torch.float32, dev)
    _need(bias, "bias", torch.float32, dev)
    C = x.shape[-1]
    out = torch.empty_like(x) if out is None else out
    rc = lib().mls_bn_act(x.data_ptr(), out.data_ptr(), scale.data_ptr(), bias.data_ptr(), x.numel() // C, C,
                          int(relu), stream_ptr(dev))
    check(rc, "mls_bn_act")
    return out


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


# ------------------------------------------------------------------ transformer ops
def layernorm(x: torch.Tensor, gamma: torch.Tensor, beta: Optional[torch.Tensor] = None, *,
              residual: Optional[torch.Tensor] = None, residual_out: Optional[torch.Tensor] = None,
              eps: float = 1e-5, rms: bool = False, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """``LN(x [+ residual])`` (or RMSNorm with ``rms=True``) over the last dim, bf16.
    ``residual_out`` receives the bf16 sum ``x + residual`` (the pre-norm residual stream)."""
    dev = x.device
    _need(x, "x", torch.bfloat16, dev)
    _need(gamma, "gamma", torch.bfloat16, dev)
    D = x.shape[-1]
    rows = x.numel() // D
    if beta is not None:
        _need(beta, "beta", torch.bfloat16, dev)
    if residual is not None:
        _need(residual, "residual", torch.bfloat16, dev)
    out = torch.empty_like(x) if out is None else out
    rc = lib().mls_layernorm(x.data_ptr(), _ptr(residual), gamma.data_ptr(), _ptr(beta), out.data_ptr(),
                             _ptr(residual_out), rows, D, float(eps), int(rms), stream_ptr(dev))
    check(rc, "mls_layernorm")
    return out


def rmsnorm(x, gamma, *, residual=None, residual_out=None, eps: float = 1e-5, out=None):
    return layernorm(x, gamma, None, residual=residual, residual_out=residual_out, eps=eps, rms=True, out=out)


def embed_layernorm(ids: torch.Tensor, type_ids: Optional[torch.Tensor], word: torch.Tensor, pos: torch.Tensor,
                    typ: torch.Tensor, gamma: torch.Tensor, beta: torch.Tensor, seq_len: int, eps: float = 1e-12,
                    out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """BERT embeddings: ``LN(word[ids] + pos[t % S] + type[type_ids])``; ids int32 ``[T]``."""
    dev = ids.device
    _need(ids, "ids", torch.int32, dev)
    T = ids.numel()
    D = word.shape[1]
    out = torch.empty(T, D, device=dev, dtype=torch.bfloat16) if out is None else out
    rc = lib().mls_embed_ln(ids.data_ptr(), _ptr(type_ids), word.data_ptr(), pos.data_ptr(), typ.data_ptr(),
                            gamma.data_ptr(), beta.data_ptr(), out.data_ptr(), T, seq_len, D, word.shape[0],
                            float(eps), stream_ptr(dev))
    check(rc, "mls_embed_ln")
    return out


def embedding(ids: torch.Tensor, table: torch.Tensor, lo: int = 0, hi: Optional[int] = None,
              out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Row gather; with a vocab shard ``[lo, hi)`` out-of-shard ids give zero rows (TP)."""
    dev = ids.device
    _need(ids, "ids", torch.int32, dev)
    _need(table, "table", torch.bfloat16, dev)
    hi = lo + table.shape[0] if hi is None else hi
    T, D = ids.numel(), table.shape[1]
    out = torch.empty(T, D, device=dev, dtype=torch.bfloat16) if out is None else out
    rc = lib().mls_embedding(ids.data_ptr(), table.data_ptr(), out.data_ptr(), T, D, lo, hi, stream_ptr(dev))
    check(rc, "mls_embedding")
    return out


def rope_(qkv: torch.Tensor, positions: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor, n_rot_heads: int,
          head_dim: int) -> torch.Tensor:
    """In-place rotate-half RoPE on the first ``n_rot_heads`` heads of each row of ``qkv``
    (Q heads then K heads in the fused projection output).  cos/sin fp32 ``[max_pos, D/2]``."""
    dev = qkv.device
    _need(qkv, "qkv", torch.bfloat16, dev)
    _need(positions, "positions", torch.int32, dev)
    T = positions.numel()
    rc = lib().mls_rope(qkv.data_ptr(), positions.data_ptr(), cos.data_ptr(), sin.data_ptr(), T, qkv.shape[-1],
                        n_rot_heads, head_dim, stream_ptr(dev))
    check(rc, "mls_rope")
    return qkv


def rope_kv_(qkv: torch.Tensor, positions: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor, n_q_heads: int,
             n_kv_heads: int, head_dim: int, slots: Optional[torch.Tensor] = None, k_cache=None, v_cache=None,
             lens: Optional[torch.Tensor] = None, seq: int = 1, max_seq: int = 0, hm_rows: int = 0):
    """Fused RoPE (Q and K heads, in place) + KV-cache append in one launch.  Cache slots come from
    ``slots`` (-1 = skip) or, with ``slots=None`` and ``max_seq > 0``, from the token index: token t
    is (batch t // seq, position p) -> slot ``b * max_seq + p``, skipped unless ``p < lens[b]``.
    ``hm_rows = R > 0``: head-major cache ``[slots / R][Hkv][R][D]`` (see :func:`decode_attention`)."""
    dev = qkv.device
    _need(qkv, "qkv", torch.bfloat16, dev)
    _need(positions, "positions", torch.int32, dev)
    T = positions.numel()
    rc = lib().mls_rope_kv(qkv.data_ptr(), positions.data_ptr(), cos.data_ptr(), sin.data_ptr(), T, qkv.shape[-1],
                           n_q_heads, n_kv_heads, head_dim, _ptr(slots), _ptr(k_cache), _ptr(v_cache), _ptr(lens),
                           seq, max_seq, k_cache.numel() // (n_kv_heads * head_dim) if k_cache is not None else 0,
                           cos.shape[0], int(hm_rows), stream_ptr(dev))
    check(rc, "mls_rope_kv")
    return qkv


def kv_append(qkv: torch.Tensor, k_col: int, v_col: int, slots: torch.Tensor, k_cache: torch.Tensor,
              v_cache: torch.Tensor, n_kv_heads: int, head_dim: int, hm_rows: int = 0) -> None:
    """Scatter the K/V heads of each token row of ``qkv`` into cache slot ``slots[t]``
    (``hm_rows`` as in :func:`rope_kv_`)."""
    dev = qkv.device
    _need(slots, "slots", torch.int32, dev)
    T = slots.numel()
    rc = lib().mls_kv_append(qkv.data_ptr(), qkv.shape[-1], k_col, v_col, slots.data_ptr(), k_cache.data_ptr(),
                             v_cache.data_ptr(), T, n_kv_heads, head_dim, int(hm_rows), stream_ptr(dev))
    check(rc, "mls_kv_append")


def flash_attention(qkv: torch.Tensor, batch: int, seq: int, n_q_heads: int, n_kv_heads: int, head_dim: int, *,
                    kv_lens: Optional[torch.Tensor] = None, causal: bool = False, scale: Optional[float] = None,
                    out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Fused attention reading Q/K/V in place from the fused projection ``qkv [B*S, (Hq+2Hkv)*D]``.
    Returns ``[B*S, Hq*D]``."""
    dev = qkv.device
    _need(qkv, "qkv", torch.bfloat16, dev)
    T, W = qkv.shape
    if T != batch * seq or W != (n_q_heads + 2 * n_kv_heads) * head_dim:
        raise ValueError("qkv shape does not match batch/seq/heads")
    if kv_lens is not None:
        _need(kv_lens, "kv_lens", torch.int32, dev)
    out = torch.empty(T, n_q_heads * head_dim, device=dev, dtype=torch.bfloat16) if out is None else out
    scale = head_dim ** -0.5 if scale is None else scale
    base = qkv.data_ptr()
    es = qkv.element_size()
    rc = lib().mls_flash_attention(base, base + n_q_heads * head_dim * es, base + (n_q_heads + n_kv_heads) * head_dim * es,
                                   out.data_ptr(), W, W, W, out.shape[1], batch, seq, n_q_heads, n_kv_heads, head_dim,
                                   _ptr(kv_lens), int(causal), float(scale), stream_ptr(dev))
    check(rc, "mls_flash_attention")
    return out


def decode_attention(q: torch.Tensor, k_cache: torch.Tensor, v_cache: torch.Tensor, lens: torch.Tensor,
                     n_q_heads: int, n_kv_heads: int, head_dim: int, *, chunk: int = 64,
                     scale: Optional[float] = None, workspace: Optional[torch.Tensor] = None,
                     counters: Optional[torch.Tensor] = None, out: Optional[torch.Tensor] = None,
                     positions: Optional[torch.Tensor] = None, cos: Optional[torch.Tensor] = None,
                     sin: Optional[torch.Tensor] = None, max_len: Optional[int] = None,
                     page_table: Optional[torch.Tensor] = None, combine: bool = True, head_major: bool = False,
                     impl: Optional[str] = None):
    """One query token per sequence vs the cache ``[B, max_len, Hkv, D]``; q rows ``[B, >= Hq*D]``
    (head h at column h*D, e.g. the fused QKV row).  Split-KV, combined in the same launch.
    With ``positions``/``cos``/``sin`` (rope mode) q is the raw fused QKV row: RoPE is applied to q
    and to the new K (row ``lens - 1 == positions``), and the new K/V are appended to the cache.
    ``max_len``: a host-side bound on ``lens`` (default: the cache length) -- it sizes the split grid,
    so a tight bound keeps idle split blocks out of short-context launches; keys beyond it are not
    visited, so it must be >= every ``lens[b]``.
    Paged KV (``page_table [B, pages_per_seq]`` int32): the caches are page pools ``[pages, chunk,
    Hkv, D]`` and row ``r`` of sequence ``b`` is row ``r % chunk`` of page ``page_table[b, r // chunk]``.
    ``combine=False``: multi-split rows are left as fp32 partials for the consumer GEMM to merge
    (:func:`skinny_packed_combine`); returns ``(out, DecodePartials)``.
    ``head_major``: caches laid out ``[B, Hkv, max_len, D]`` (paged: ``[pages, Hkv, chunk, D]``) --
    one head's rows contiguous, so each split block streams one run instead of 256-B slices.
    ``impl``: "mfma" (matrix-core kernel: D = 128, chunk 64 / 128, G <= 8), "valu", or "auto"
    (default, env ``MLS_DECODE_ATTN``): the matrix-core kernel wherever it applies."""
    impl = impl or os.environ.get("MLS_DECODE_ATTN", "auto")
    impl_code = {"auto": 0, "valu": 1, "mfma": 2}[impl]
    dev = q.device
    B = lens.numel()
    rows_dim = 2 if head_major else 1
    if page_table is not None:
        _need(page_table, "page_table", torch.int32, dev)
        if page_table.dim() != 2 or page_table.shape[0] < B or k_cache.shape[rows_dim] != chunk:
            raise ValueError("paged decode: page_table [>= B, pages_per_seq], caches [pages, chunk, Hkv, D] "
                             "(head-major: [pages, Hkv, chunk, D])")
        cap = page_table.shape[1] * chunk
        max_len = cap if max_len is None else min(int(max_len), cap)
    else:
        L = k_cache.shape[rows_dim]
        max_len = L if max_len is None else min(int(max_len), L)
    hm_rows = k_cache.shape[2] if head_major else 0
    nsplit = (max_len + chunk - 1) // chunk
    need = B * n_q_heads * nsplit * (head_dim + 2)
    if workspace is None or workspace.numel() < need:
        workspace = torch.empty(need, device=dev, dtype=torch.float32)
    if counters is None or counters.numel() < B * n_kv_heads:
        counters = torch.zeros(B * n_kv_heads, device=dev, dtype=torch.int32)
    ws = workspace[: B * n_q_heads * nsplit * head_dim]
    ws_ml = workspace[B * n_q_heads * nsplit * head_dim: need]
    out = torch.empty(B, n_q_heads * head_dim, device=dev, dtype=torch.bfloat16) if out is None else out
    scale = head_dim ** -0.5 if scale is None else scale
    if positions is not None:
        _need(positions, "positions", torch.int32, dev)
    rc = lib().mls_decode_attention(q.data_ptr(), k_cache.data_ptr(), v_cache.data_ptr(), out.data_ptr(),
                                    ws.data_ptr(), ws_ml.data_ptr(), counters.data_ptr(), q.stride(0), out.stride(0),
                                    k_cache.stride(0), lens.data_ptr(), _ptr(positions), _ptr(cos), _ptr(sin),
                                    cos.shape[0] if cos is not None else 0, B, n_q_heads, n_kv_heads, head_dim, max_len,
                                    chunk, float(scale), _ptr(page_table),
                                    page_table.shape[1] if page_table is not None else 0, int(not combine),
                                    int(hm_rows), impl_code, stream_ptr(dev))
    check(rc, "mls_decode_attention")
    if not combine:
        return out, DecodePartials(ws, ws_ml, nsplit, chunk, lens, n_q_heads, head_dim)
    return out


class DecodePartials:
    """Split-KV decode attention partials left for a consumer to merge (see ``combine=False``)."""

    def __init__(self, ws, ws_ml, nsplit, chunk, lens, n_q_heads, head_dim):
        self.ws, self.ws_ml, self.nsplit, self.chunk = ws, ws_ml, int(nsplit), int(chunk)
        self.lens, self.n_q_heads, self.head_dim = lens, int(n_q_heads), int(head_dim)


def skinny_packed_combine(attn_out: torch.Tensor, parts: DecodePartials, wp: torch.Tensor, N: int, *,
                          bias: Optional[torch.Tensor] = None, residual: Optional[torch.Tensor] = None,
                          variant: int = 9) -> torch.Tensor:
    """``merge(attention partials) @ W^T (+ bias) (+ residual)`` with W packed (:func:`pack_skinny`):
    the o-projection of a decode step that also does the split-KV combine in its prologue (one
    launch instead of two).  ``attn_out``: the attention's direct-written rows ``[M, Hq*D]``."""
    dev = attn_out.device
    _need(attn_out, "attn_out", torch.bfloat16, dev)
    M, K = attn_out.shape
    if M > 4 or K != parts.n_q_heads * parts.head_dim or wp.numel() != N * K or M * K * 2 > 65536:
        raise ValueError("skinny_packed_combine: M <= 4, K == Hq * D, M * K * 2 <= 64 KiB, wp of N*K elements")
    if residual is not None:
        _need(residual, "residual", torch.bfloat16, dev)
        if tuple(residual.shape) != (M, N):
            raise ValueError("residual must be [M, N]")
    if bias is not None:
        _need(bias, "bias", torch.float32, dev)
    out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    rc = lib().mls_skinny_packed_combine(attn_out.data_ptr(), parts.ws.data_ptr(), parts.ws_ml.data_ptr(),
                                         parts.lens.data_ptr(), parts.nsplit, parts.chunk, parts.n_q_heads,
                                         parts.head_dim, wp.data_ptr(), _ptr(bias), _ptr(residual), out.data_ptr(),
                                         M, N, K, ACT_NONE, int(variant), stream_ptr(dev))
    check(rc, "mls_skinny_packed_combine")
    return out


def decode_pick(cand_v: torch.Tensor, cand_i: torch.Tensor, tok: torch.Tensor, pos: torch.Tensor, lens: torch.Tensor,
                step: torch.Tensor, *, topk: Optional[torch.Tensor] = None, temp: Optional[torch.Tensor] = None,
                seed: Optional[torch.Tensor] = None, hist: Optional[torch.Tensor] = None) -> None:
    """X4 merge + next-token pick on device (csrc/decode_pick.hip): ``cand_v`` / ``cand_i`` are the
    all-gathered ``[tp, B, k]`` candidates; per row picks greedily (``topk[b] <= 1``) or samples
    (top-k, temperature, counter-based ``seed`` x step draw -- :func:`models.llama.sample_uniform`),
    then advances ``tok`` / ``pos`` / ``lens`` / ``step`` ``[B]`` in place and records the token in
    ``hist[b, step[b]]``.  Capturable (the TP decode graph ends with it)."""
    dev = cand_v.device
    tp, B, k = cand_v.shape
    _need(cand_v, "cand_v", torch.float32, dev)
    _need(cand_i, "cand_i", torch.int32, dev)
    if tuple(cand_i.shape) != (tp, B, k) or tp * k > 512:
        raise ValueError("cand_i must match cand_v [tp, B, k] with tp * k <= 512")
    for name, t, dt in (("tok", tok, torch.int32), ("pos", pos, torch.int32), ("lens", lens, torch.int32),
                        ("step", step, torch.int32)):
        _need(t, name, dt, dev)
        if t.numel() != B:
            raise ValueError(f"{name} must have {B} elements")
    for name, t, dt in (("topk", topk, torch.int32), ("temp", temp, torch.float32), ("seed", seed, torch.int64)):
        if t is not None:
            _need(t, name, dt, dev)
            if t.numel() != B:
                raise ValueError(f"{name} must have {B} elements")
    cols = 0
    if hist is not None:
        _need(hist, "hist", torch.int32, dev)
        if hist.shape[0] != B:
            raise ValueError("hist must be [B, cols]")
        cols = hist.shape[1]
    rc = lib().mls_decode_pick(cand_v.data_ptr(), cand_i.data_ptr(), tp, B, k, _ptr(topk), _ptr(temp), _ptr(seed),
                               tok.data_ptr(), pos.data_ptr(), lens.data_ptr(), _ptr(hist), cols, step.data_ptr(),
                               stream_ptr(dev))
    check(rc, "mls_decode_pick")


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


MASK_WORDS = 8  # 256 CUs


_MASKED_STREAMS: Dict[tuple, torch.cuda.ExternalStream] = {}
_MASKED_LOCK = __import__("threading").Lock()




def cu_masked_stream(mask: Sequence[int], device=None, key=0) -> torch.cuda.ExternalStream:
    """The HIP stream restricted to the CUs whose bits are set in ``mask`` (``MASK_WORDS`` uint32
    words; csrc/partition.hip) -- one per (device, mask, ``key``), created on first use and kept
    for the process.  Every masked stream holds a hardware queue of its own, so they are pooled:
    engines built one after another reuse them (``key`` tells apart the streams one engine needs
    on the same mask) instead of piling up queues until queue creation fails."""
    import ctypes

    dev = torch.device(device if device is not None else "cuda")
    if dev.index is None:
        dev = torch.device("cuda", torch.cuda.current_device())
    ck = (dev.index, tuple(int(m) & 0xFFFFFFFF for m in mask), key)
    with _MASKED_LOCK:
        st = _MASKED_STREAMS.get(ck)
        if st is None:
            words = (ctypes.c_uint32 * len(mask))(*ck[1])
            out = ctypes.c_void_p()
            with torch.cuda.device(dev):
                check(lib().mls_stream_create_cumask(ctypes.cast(words, ctypes.c_void_p), len(mask),
                                                     ctypes.byref(out)), "mls_stream_create_cumask")
            st = _MASKED_STREAMS[ck] = torch.cuda.ExternalStream(out.value, device=dev)
        return st


def cu_census(stream: torch.cuda.Stream, blocks: int = 2048, spin: int = 64) -> torch.Tensor:
    """(XCC_ID, HW_ID) of the CU each of ``blocks`` blocks ran on, launched on ``stream``: int32 [blocks, 2]."""
    out = torch.full((blocks, 2), -1, device=stream.device, dtype=torch.int32)
    with torch.cuda.stream(stream):
        check(lib().mls_cu_census(out.data_ptr(), blocks, spin, stream.cuda_stream), "mls_cu_census")
    stream.synchronize()
    return out.cpu()


_XCD_MASKS: Dict[int, Optional[List[List[int]]]] = {}


def xcd_cu_masks(device=None) -> Optional[List[List[int]]]:
    """Per XCD, the CU-mask words that select exactly that XCD's CUs, verified on the device with
    :func:`cu_census` (every block of a masked stream must report one XCC id, and the 8 masks 8
    distinct ids).  Logical mask bit ``b`` is tried as XCD ``b % 8`` (round-robin) and as
    ``b // 32`` (contiguous); ``None`` when neither layout verifies."""
    dev = torch.device(device if device is not None else "cuda")
    key = dev.index if dev.index is not None else torch.cuda.current_device()
    if key in _XCD_MASKS:
        return _XCD_MASKS[key]
    ncu = torch.cuda.get_device_properties(dev).multi_processor_count
    result = None
    if ncu == 256:
        for layout in ("roundrobin", "contiguous"):
            masks = []
            for x in range(8):
                bits = [b for b in range(ncu) if (b % 8 if layout == "roundrobin" else b // 32) == x]
                w = [0] * MASK_WORDS
                for b in bits:
                    w[b // 32] |= 1 << (b % 32)
                masks.append(w)
            ids = []
            for w in masks:
                c = cu_census(cu_masked_stream(w, dev, key="census"), blocks=256)
                ids.append(set(c[:, 0].tolist()))
            if all(len(s) == 1 for s in ids) and len(set().union(*ids)) == 8:
                result = masks
                break
    _XCD_MASKS[key] = result
    return result


def census_cus(c: torch.Tensor) -> set:
    """Distinct physical CUs in a :func:`cu_census` result: (XCC, SE, SH, CU) from HW_ID bits 8-15."""
    return {(int(x), (int(h) >> 8) & 0xFF) for x, h in c.tolist()}


def intra_partition_words(parts: int, ncu: int = 256, mode: str = "intra", xccs: int = 8) -> List[List[int]]:
    """The CU-mask words of ``parts`` intra-XCD partitions (pure; verified on the device by
    :func:`partition_masks`).  Mask bit ``b`` is CU ``b // xccs`` of XCC ``b % xccs`` (census:
    profiles/r3_cu_mask_census.txt); an XCC left without a bit runs on ALL its CUs, so every
    partition keeps ``ncu / xccs / parts`` CUs on every XCC: CU ``c`` goes to partition ``c %
    parts`` (``"intra"``) or ``c // (ncu / xccs / parts)`` (``"intra_contig"``)."""
    per_xcc = ncu // xccs
    if parts <= 0 or per_xcc % parts or mode not in ("intra", "intra_contig"):
        raise ValueError(f"{parts} {mode} partitions of {per_xcc} CUs per XCC")
    out = []
    for p in range(parts):
        w = [0] * max(MASK_WORDS, (ncu + 31) // 32)
        for b in range(ncu):
            c = b // xccs
            if (c % parts if mode == "intra" else c // (per_xcc // parts)) == p:
                w[b // 32] |= 1 << (b % 32)
        out.append(w)
    return out


_PARTITION_MASKS: Dict[tuple, Optional[List[List[int]]]] = {}


def partition_masks(parts: int, device=None, mode: str = "xcd") -> Optional[List[List[int]]]:
    """Cached :func:`_partition_masks` (the census verification runs once per device / mode / parts)."""
    dev = torch.device(device if device is not None else "cuda")
    ck = (dev.index if dev.index is not None else torch.cuda.current_device(), parts, mode)
    if ck not in _PARTITION_MASKS:
        _PARTITION_MASKS[ck] = _partition_masks(parts, dev, mode)
    return _PARTITION_MASKS[ck]


def _partition_masks(parts: int, device=None, mode: str = "xcd") -> Optional[List[List[int]]]:
    """``parts`` (1, 2, 4 or 8) CU masks.  ``mode="xcd"``: each the union of 8 / parts whole XCDs
    (needs :func:`xcd_cu_masks`).  ``mode="intra"``: each a 1 / parts share of the CUs of EVERY
    XCD (CU ``c`` of every XCC with ``c % parts == p``; ``"intra_contig"``: ``c // (32 / parts) ==
    p``), verified by census to select disjoint CU sets of the expected size."""
    if parts not in (1, 2, 4, 8):
        raise ValueError("parts must be 1, 2, 4 or 8")
    if mode in ("intra", "intra_contig"):
        dev = torch.device(device if device is not None else "cuda")
        ncu = torch.cuda.get_device_properties(dev).multi_processor_count
        out, seen = [], set()
        for p, w in enumerate(intra_partition_words(parts, ncu, mode)):
            cus = census_cus(cu_census(cu_masked_stream(w, dev, key="census"), blocks=4096))
            if len(cus) > ncu // parts or cus & seen:
                return None
            seen |= cus
            out.append(w)
        return out
    xm = xcd_cu_masks(device)
    if xm is None:
        return None
    per = 8 // parts
    out = []
    for p in range(parts):
        w = [0] * MASK_WORDS
        for x in range(p * per, (p + 1) * per):
            w = [a | b for a, b in zip(w, xm[x])]
        out.append(w)
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
