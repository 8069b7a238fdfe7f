"""GEMM kernels: the conv_gemm-based plain GEMM, the persistent large-M tile GEMM, the skinny (decode) GEMMs."""
from __future__ import annotations

import ctypes
from typing import Dict, Optional, Tuple

import torch

from ._lib import check, lib, stream_ptr
from ._core import ACT_GELU, ACT_NONE, ACT_SILU_MUL, _act, _need, _ptr, _workspace_args


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


def fold_layernorm(w: torch.Tensor, bias: Optional[torch.Tensor], gamma: torch.Tensor, beta: torch.Tensor):
    """Fold a LayerNorm ``(gamma, beta)`` into the projection after it (csrc/gemm_tile.hip, "LayerNorm
    folding"): ``LN(h) @ W.T + b = rstd * (h @ W'.T - mu * c) + b'`` with ``W' = W * gamma`` (bf16),
    ``c = W'.sum(1)`` (fp32 sum of the bf16 ``W'``, so the mean term cancels what the MFMAs add) and
    ``b' = b + W @ beta``.  Returns ``(W', c, b')``."""
    wf = w.float()
    w2 = (wf * gamma.float()[None, :]).to(torch.bfloat16)
    c = w2.float().sum(1).contiguous()
    b2 = wf @ beta.float()
    if bias is not None:
        b2 = b2 + bias.float()
    return w2.contiguous(), c, b2.contiguous()


def ln_partials(M: int, width: int, device) -> torch.Tensor:
    """fp32 buffer for the row statistics a residual :func:`gemm_tile_ln` launch writes
    (``stats_part``) and the next LayerNorm-folding launches read (``ln_part``): per row and 128-column
    block, the sum and sum of squares of the stored bf16 values."""
    return torch.empty(M * (width // 128) * 2, device=device, dtype=torch.float32)


def layernorm_from_partials(h: torch.Tensor, part: torch.Tensor, eps: float = 1e-12):
    """(mean, rstd) per row from :func:`ln_partials` -- the host-side oracle of what the kernels do."""
    M, W = h.shape
    p = part[: M * (W // 128) * 2].view(M, W // 128, 2).double().sum(1)
    mu = p[:, 0] / W
    var = (p[:, 1] / W - mu * mu).clamp_min(0)
    return mu.float(), torch.rsqrt(var + eps).float()


def gemm_tile_ln(a: torch.Tensor, w: torch.Tensor, bias: Optional[torch.Tensor] = None, *, act=ACT_NONE,
                 fold_c: Optional[torch.Tensor] = None, ln_part: Optional[torch.Tensor] = None,
                 residual: Optional[torch.Tensor] = None, ln_g: Optional[torch.Tensor] = None,
                 stats_part: Optional[torch.Tensor] = None, eps: float = 1e-12, cfg: int = 0,
                 out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """The LayerNorm-folding forms of :func:`gemm_tile` (csrc/gemm_tile.hip, "LayerNorm folding").
    Row statistics travel as :func:`ln_partials` buffers:

    * ``fold_c`` given: ``a`` holds the raw pre-LN rows h, ``ln_part`` their partials (width K);
      ``w`` / ``bias`` / ``fold_c`` come from :func:`fold_layernorm`; returns ``act(LN(h) @ W.T + b)``
      (act: none / gelu);
    * ``residual`` given: ``a @ w.T + bias + r`` with ``r = residual``, or ``(residual - mu) * rstd *
      ln_g`` when ``ln_part`` (the residual's partials, width N) and ``ln_g`` (fp32 ``[N]``) are
      given -- that LN's beta must be folded into ``bias``; ``stats_part`` then receives the OUTPUT
      rows' partials (width N)."""
    dev = a.device
    _need(a, "a", torch.bfloat16, dev)
    _need(w, "w", torch.bfloat16, dev)
    M, K = a.shape
    N, K2 = w.shape
    code = _act(act)
    if K != K2 or K % 64 or N % 16:
        raise ValueError("gemm_tile_ln: K % 64 == 0, N % 16 == 0")
    for name, t, n in (("bias", bias, N), ("fold_c", fold_c, N), ("ln_g", ln_g, N),
                       ("ln_part", ln_part, M * ((K if fold_c is not None else N) // 128) * 2),
                       ("stats_part", stats_part, M * (N // 128) * 2)):
        if t is not None:
            _need(t, name, torch.float32, dev)
            if t.numel() < n:
                raise ValueError(f"{name} needs {n} elements")
    if fold_c is not None:
        if ln_part is None or residual is not None or stats_part is not None or code not in (ACT_NONE, ACT_GELU) \
                or K % 256 or K > 1024:
            raise ValueError("folded form: ln_part, no residual / stats_part, act none or gelu, K % 256, K <= 1024")
    else:
        if residual is None or code != ACT_NONE:
            raise ValueError("gemm_tile_ln needs fold_c or a residual (and no activation)")
        _need(residual, "residual", torch.bfloat16, dev)
        if tuple(residual.shape) != (M, N):
            raise ValueError("residual must be [M, N]")
        if ln_part is not None and (ln_g is None or N % 256 or N > 1024):
            raise ValueError("a LayerNorm'd residual needs ln_g and N % 256 == 0, N <= 1024")
        if stats_part is not None and N % 128:
            raise ValueError("stats_part needs N % 128 == 0")
    if out is None:
        out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    else:
        _need(out, "out", torch.bfloat16, dev)
    rc = lib().mls_gemm_tile_ln(a.data_ptr(), w.data_ptr(), _ptr(bias), _ptr(residual), out.data_ptr(), M, N, K,
                                code, int(cfg), _ptr(fold_c), _ptr(ln_part), _ptr(ln_g), _ptr(stats_part),
                                stats_part.numel() if stats_part is not None else 0, float(eps), stream_ptr(dev))
    check(rc, "mls_gemm_tile_ln")
    return out


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


def mgemm(a: torch.Tensor, w: torch.Tensor, bias: Optional[torch.Tensor] = None, *, act=ACT_NONE,
          residual: Optional[torch.Tensor] = None, splitk: int = 0,
          workspace: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Medium-M weight-streaming GEMM (csrc/mgemm.hip): ``act(a @ w.T + bias) (+ residual)`` for
    17..256-row decode batches -- weights straight to registers, activations through an LDS ring.
    a ``[M, K]`` (row stride may exceed K), w ``[N, K]``; N % 64 == 0, K % 256 == 0; ``act="silu_mul"``
    as :func:`gemm`.  ``splitk`` <= 0: the launcher's pick (K slices within one block per CU)."""
    dev = a.device
    _need(w, "w", torch.bfloat16, dev)
    if a.dtype != torch.bfloat16 or a.device != dev or a.dim() != 2 or a.stride(1) != 1:
        raise ValueError("a: bf16 [M, K] with unit column stride")
    M, K = a.shape
    N = w.shape[0]
    if w.shape[1] != K or not 0 < M <= 256 or N % 64 or K % 256:
        raise ValueError(f"mgemm: M {M} (1..256), N {N} (% 64), K {K} (% 256)")
    code = _act(act)
    if bias is not None:
        _need(bias, "bias", torch.float32, dev)
    n_out = N // 2 if code == ACT_SILU_MUL else N
    if residual is not None:
        _need(residual, "residual", torch.bfloat16, dev)
        if code == ACT_SILU_MUL or tuple(residual.shape) != (M, N):
            raise ValueError("residual: [M, N], not with silu_mul")
    out = torch.empty(M, n_out, device=dev, dtype=torch.bfloat16)
    if splitk <= 0:
        splitk = int(lib().mls_mgemm_auto_split(N, K, 0))
    need = splitk * M * N if splitk > 1 else 0
    if need and (workspace is None or workspace.numel() * workspace.element_size() < need * 4):
        workspace = torch.empty(need, device=dev, dtype=torch.float32)
    wsp, wsb = _workspace_args(workspace) if need else (None, 0)
    rc = lib().mls_mgemm(a.data_ptr(), w.data_ptr(), _ptr(bias), _ptr(residual), out.data_ptr(), wsp, wsb,
                         M, N, K, a.stride(0), code, splitk, stream_ptr(dev))
    check(rc, "mls_mgemm")
    return out


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


def skinny_packed_ar(x: torch.Tensor, wp: torch.Tensor, N: int, car, *, variant: int = 9,
                     out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Row-parallel TP projection with its all-reduce fused into the GEMM launch: ``sum over ranks of
    x @ W^T`` (csrc/ar_protocol.h ``ar_fused_tail``: the blocks that complete a 2048-element chunk of
    the output run that chunk's one-shot IPC all-reduce, no separate collective kernel).  ``car``:
    the rank's :class:`parallel.custom_ar.CustomAllReduce`; every rank must make the same call."""
    dev = x.device
    _need(x, "x", torch.bfloat16, dev)
    _need(wp, "wp", torch.bfloat16, dev)
    M, K = x.shape
    if M > 32 or N % 16 or K % 32 or wp.numel() != N * K:
        raise ValueError("skinny_packed_ar: M <= 32, N % 16 == 0, K % 32 == 0, wp of N*K elements")
    if out is None:
        out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    elif tuple(out.shape) != (M, N) or out.dtype != torch.bfloat16 or not out.is_contiguous():
        raise ValueError(f"out must be contiguous bf16 [M, {N}]")
    rc = lib().mls_skinny_packed_ar(x.data_ptr(), None, None, wp.data_ptr(), out.data_ptr(), M, N, K, 0, 0.0,
                                    int(variant), car.ctx_ptr(), stream_ptr(dev))
    check(rc, "mls_skinny_packed_ar")
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
