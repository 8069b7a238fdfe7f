"""Projection dispatch policy (``linear``): which GEMM kernel a transformer projection runs on."""
from __future__ import annotations

import ctypes
import os
from typing import Optional

import torch

from ._core import ACT_GELU, ACT_NONE, ACT_SILU_MUL, _act
from ._lib import check, lib, stream_ptr
from .gemm_ops import _bias_bf16, gemm, gemm_tile, gemm_tile_ln, mgemm, silu_mul_interleaved
from .tables import small_m_plan_for, tile_cfg_for, tile_route_for


# Every projection runs on our own kernels: large M on the LDS-DMA MFMA tile kernel (gemm_tile:
# csrc/gemm_tile.hip) or, for short-M shapes whose tiles cannot fill the chip, the conv_gemm kernel
# with in-launch split-K -- per shape as tuned/gemm_tile_gfx950.json measured -- and the decode-shaped
# ones (M <= 32, and 33..TILE_MIN_M - 1 rows) on the skinny / conv_gemm kernels with per-shape plans.
# No default path calls a library GEMM (round 6 routed the last nine Llama-3-8B TP=1 shapes that still
# went to hipBLASLt to their best native config: profiles/r6_gemm_native_routes_probe.jsonl).
# hipBLASLt (torch.addmm) is reachable only as the explicit A/B arm: MLS_GEMM_IMPL=blas, impl="blas".
TILE_MIN_M = int(os.environ.get("MLS_TILE_MIN_M", "256"))


BLAS_MIN_M = TILE_MIN_M  # kept for callers that split "large" from "small" token counts


_GEMM_IMPL = os.environ.get("MLS_GEMM_IMPL", "auto")  # auto: the table routes; native; blas

# MLS_MGEMM=1: 17..128-row projections with N <= 4096 and K in [4096, 8192) -- Llama-3-8B's o_proj
# in decode at 17-128 slots -- go to the weight-streaming medium-M kernel (csrc/mgemm.hip);
# MLS_MGEMM=all also sends down_proj / qkv shapes.  Off by default.  Alone, with the weights L2-cold
# as in a decode step and the model's workspace (tools/probe/mgemm_probe.py,
# profiles/r6_mgemm_probe_vs_routes.jsonl), us, mgemm vs the table route: o_proj 16.0 / 18.6 vs
# 24.4 / 20.2 at 64 / 128 rows, level at 256; down_proj slower (39.6 / 49.7 / 69.2 vs 34.7 / 41.9 /
# 70.2); qkv level.  Inside the decode step it loses: o_proj routed, decode 32 / 64 / 128 rows
# 4.42-4.45 / 5.01-5.03 / 6.34-6.37 vs 4.36-4.37 / 4.98-4.99 / 6.26-6.27 ms per step
# (profiles/r6_mgemm_o_route_llama_e2e_ab.jsonl); o + down + qkv routed, 64 / 128 / 256 rows 5.38 /
# 6.53 / 8.88 vs 4.97-5.06 / 6.17-6.19 / 8.62 (profiles/r6_mgemm_llama_e2e_ab.jsonl).
_MGEMM = os.environ.get("MLS_MGEMM", "0")


def mgemm_route(M: int, N: int, K: int) -> bool:
    """Whether :func:`linear` sends an ``[M, K] x [N, K]^T`` projection to :func:`mgemm`."""
    if _MGEMM == "0" or not 16 < M <= 256 or N % 64 or K % 256 or K < 4096:
        return False
    if _MGEMM == "all":
        return N <= 4096 or (N <= 8192 and M <= 128)
    return M <= 128 and N <= 4096 and K < 8192


def linear(a: torch.Tensor, w: torch.Tensor, bias: Optional[torch.Tensor] = None, *, act=ACT_NONE,
           residual: Optional[torch.Tensor] = None, workspace: Optional[torch.Tensor] = None,
           impl: str = "auto") -> torch.Tensor:
    """Transformer projection ``act(a @ w.T + bias) (+ residual)``: M >= TILE_MIN_M on the table's
    route -- the persistent LDS-DMA tile kernel (:func:`gemm_tile`, bias / GELU / SiLU-mul / residual
    in its epilogue) or conv_gemm -- smaller M on the skinny / conv_gemm kernels (measured per-shape
    plans in ``tuned/gemm_plan_gfx950.json``).  ``impl``: "auto" / "native" (the same: our kernels) |
    "tile" | "blas" (hipBLASLt, the A/B arm only; also ``MLS_GEMM_IMPL=blas``)."""
    code = _act(act)
    M, K = a.shape
    N = w.shape[0]
    if impl == "blas" or (impl == "auto" and _GEMM_IMPL == "blas"):
        return _linear_blas(a, w, bias, code, residual)
    if (impl in ("auto", "native") and mgemm_route(M, N, K) and a.device.type == "cuda" and a.stride(1) == 1
            and w.is_contiguous() and (residual is None or residual.is_contiguous())
            and code in (ACT_NONE, ACT_SILU_MUL) and not (code == ACT_SILU_MUL and residual is not None)):
        return mgemm(a, w, bias, act=code, residual=residual,
                     workspace=workspace if workspace is not None and workspace.dtype == torch.float32 else None)
    if impl == "tile" or (impl in ("auto", "native") and M >= TILE_MIN_M and K % 64 == 0 and N % 16 == 0
                          and a.device.type == "cuda" and a.is_contiguous() and w.is_contiguous()):
        kind, cfg, sk = tile_route_for(M, N, K) if impl in ("auto", "native") else ("tile",) + tile_cfg_for(M, N, K)
        if kind == "conv":
            return gemm(a, w, bias, act=code, residual=residual, workspace=workspace, cfg=cfg, splitk=sk)
        if kind != "tile":
            cfg, sk = 0, 1  # an unknown route kind (e.g. an old table's "blas"): the tile kernel's own pick
        return gemm_tile(a, w, bias, act=code, residual=residual, cfg=cfg, splitk=sk, workspace=workspace)
    plan = small_m_plan_for(M, N, K) if impl in ("auto", "native") else None
    if plan is not None and plan[0] > 0 and not (code == ACT_SILU_MUL and residual is not None):
        return gemm(a, w, bias, act=code, residual=residual, workspace=workspace, cfg=plan[0], splitk=plan[1])
    return gemm(a, w, bias, act=code, residual=residual, workspace=workspace)


# Llama above 24 tokens per step: a split-K projection whose output only feeds "residual += y;
# x = RMSNorm(residual)" (o_proj, down_proj) leaves its fp32 slabs to one kernel that reduces them,
# adds the residual and normalises (ops mls_gemm_slabs + mls_splitk_add_rmsnorm): one launch instead
# of the reduce + RMSNorm pair.  MLS_FUSE_ADD_NORM=0 turns it off.
_FUSE_ADD_NORM = os.environ.get("MLS_FUSE_ADD_NORM", "1") != "0"
_MLS_UNSUPPORTED = 1002  # csrc/common.h MlsStatus
# the largest row count it takes (the tile route's threshold minus one by default; A/B knob)
_ADD_NORM_MAX_M = int(os.environ.get("MLS_ADD_NORM_MAX_M", str(TILE_MIN_M - 1)))


def linear_add_rmsnorm(a: torch.Tensor, w: torch.Tensor, residual: torch.Tensor, gamma: torch.Tensor, eps: float,
                       workspace: Optional[torch.Tensor]) -> Optional[torch.Tensor]:
    """``residual += a @ w.T`` (in place, rounded to bf16 as :func:`linear` + the residual add would) and
    returns ``RMSNorm(residual) * gamma`` -- bit-identical to :func:`linear` followed by
    ``rmsnorm(y, gamma, residual=residual, residual_out=residual)``, in two launches instead of three.
    Returns None (nothing launched) where the shape is not on a split-K conv_gemm route (24 < M <
    TILE_MIN_M, split > 1, 2048 <= N <= 4096: narrower rows normalise on the wave-per-row kernel,
    whose sum order differs) or the workspace is too small: the caller runs the plain pair."""
    M, K = a.shape
    N = w.shape[0]
    if (not _FUSE_ADD_NORM or _GEMM_IMPL == "blas" or not 24 < M <= _ADD_NORM_MAX_M or N % 8 or K % 8
            or not 2048 <= N <= 4096  # the widths the row-block RMSNorm takes: the same arithmetic
            or workspace is None or workspace.dtype != torch.float32 or not a.is_contiguous()
            or not w.is_contiguous() or not residual.is_contiguous() or tuple(residual.shape) != (M, N)
            or residual.dtype != torch.bfloat16 or gamma.numel() != N):
        return None
    plan = small_m_plan_for(M, N, K)
    cfg, sk = (plan[0], plan[1]) if plan is not None and plan[0] > 0 else (0, 0)
    split = ctypes.c_int(0)
    wsb = workspace.numel() * 4
    dev = a.device
    rc = lib().mls_gemm_slabs(a.data_ptr(), w.data_ptr(), workspace.data_ptr(), wsb, M, N, K, cfg, sk,
                              ctypes.byref(split), stream_ptr(dev))
    if rc == _MLS_UNSUPPORTED:  # this shape would not split -- nothing was launched
        return None
    check(rc, "mls_gemm_slabs")
    out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    rc = lib().mls_splitk_add_rmsnorm(workspace.data_ptr(), wsb, split.value, M, N, residual.data_ptr(),
                                      gamma.data_ptr(), out.data_ptr(), float(eps), stream_ptr(dev))
    check(rc, "mls_splitk_add_rmsnorm")
    return out


def ln_foldable(M: int, N: int, K: int) -> bool:
    """Whether :func:`linear_ln` runs this shape where :func:`linear` would use the tile kernel too
    (large M; K and N multiples of the 128-column statistics blocks) -- callers keep an explicit
    LayerNorm otherwise."""
    return M >= TILE_MIN_M and K % 128 == 0 and N % 128 == 0 and K <= 4096 and _GEMM_IMPL != "blas"


def linear_ln(a: torch.Tensor, w: torch.Tensor, bias: Optional[torch.Tensor] = None, *, act=ACT_NONE,
              fold_c: Optional[torch.Tensor] = None, ln_part: Optional[torch.Tensor] = None,
              residual: Optional[torch.Tensor] = None, ln_g: Optional[torch.Tensor] = None,
              stats_part: Optional[torch.Tensor] = None, eps: float = 1e-12) -> torch.Tensor:
    """A projection with LayerNorm folding (:func:`gemm_tile_ln`) on the tile the table picks for the
    shape (the folding kernels map it to the nearest of theirs)."""
    M, K = a.shape
    N = w.shape[0]
    cfg = tile_cfg_for(M, N, K)[0] if M >= TILE_MIN_M else 0
    return gemm_tile_ln(a, w, bias, act=act, fold_c=fold_c, ln_part=ln_part, residual=residual, ln_g=ln_g,
                        stats_part=stats_part, eps=eps, cfg=cfg)


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
