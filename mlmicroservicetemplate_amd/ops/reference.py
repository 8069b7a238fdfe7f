"""Plain-PyTorch fp32 oracles of every transformer kernel in ``ops`` (device-agnostic: they run
on CPU for the CPU test suite and on GPU as the numerics reference of the HIP kernels)."""
from __future__ import annotations

from typing import Optional, Tuple

import torch
import torch.nn.functional as F


def layernorm(x, gamma, beta=None, residual=None, eps=1e-5, rms=False):
    """Returns (normed, residual_sum) in fp32."""
    h = x.float() + (residual.float() if residual is not None else 0.0)
    hs = h.to(torch.bfloat16).float() if x.dtype == torch.bfloat16 else h
    if rms:
        y = hs * torch.rsqrt(hs.pow(2).mean(-1, keepdim=True) + eps) * gamma.float()
    else:
        y = F.layer_norm(hs, (hs.shape[-1],), gamma.float(), beta.float() if beta is not None else None, eps)
    return y, hs


def rope_tables(max_pos: int, head_dim: int, theta: float = 500000.0, device=None) -> Tuple[torch.Tensor, torch.Tensor]:
    inv = 1.0 / (theta ** (torch.arange(0, head_dim, 2, dtype=torch.float64) / head_dim))
    t = torch.arange(max_pos, dtype=torch.float64)
    ang = torch.outer(t, inv)
    return ang.cos().float().to(device).contiguous(), ang.sin().float().to(device).contiguous()


def rope(x_heads: torch.Tensor, positions: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor) -> torch.Tensor:
    """Rotate-half RoPE on ``[T, H, D]`` (fp32 result)."""
    x = x_heads.float()
    half = x.shape[-1] // 2
    c = cos[positions.long()].unsqueeze(1)
    s = sin[positions.long()].unsqueeze(1)
    x1, x2 = x[..., :half], x[..., half:]
    return torch.cat([x1 * c - x2 * s, x2 * c + x1 * s], dim=-1)


def split_qkv(qkv: torch.Tensor, Hq: int, Hkv: int, D: int):
    T = qkv.shape[0]
    q = qkv[:, : Hq * D].reshape(T, Hq, D)
    k = qkv[:, Hq * D: (Hq + Hkv) * D].reshape(T, Hkv, D)
    v = qkv[:, (Hq + Hkv) * D: (Hq + 2 * Hkv) * D].reshape(T, Hkv, D)
    return q, k, v


def attention(qkv: torch.Tensor, B: int, S: int, Hq: int, Hkv: int, D: int, kv_lens: Optional[torch.Tensor] = None,
              causal: bool = False, scale: Optional[float] = None) -> torch.Tensor:
    """softmax(QK^T*scale + mask) V over the fused projection; returns fp32 ``[B*S, Hq*D]``."""
    scale = D ** -0.5 if scale is None else scale
    q, k, v = split_qkv(qkv.float(), Hq, Hkv, D)
    q = q.view(B, S, Hq, D).transpose(1, 2)
    k = k.view(B, S, Hkv, D).transpose(1, 2).repeat_interleave(Hq // Hkv, dim=1)
    v = v.view(B, S, Hkv, D).transpose(1, 2).repeat_interleave(Hq // Hkv, dim=1)
    s = torch.matmul(q, k.transpose(-1, -2)) * scale
    mask = torch.zeros(B, 1, S, S, dtype=torch.bool, device=qkv.device)
    if kv_lens is not None:
        mask |= (torch.arange(S, device=qkv.device).view(1, 1, 1, S) >= kv_lens.long().view(B, 1, 1, 1))
    if causal:
        mask |= torch.ones(S, S, dtype=torch.bool, device=qkv.device).triu(1).view(1, 1, S, S)
    s = s.masked_fill(mask, float("-inf"))
    p = torch.softmax(s, dim=-1)
    p = torch.nan_to_num(p, nan=0.0)
    o = torch.matmul(p, v)
    return o.transpose(1, 2).reshape(B * S, Hq * D)


def decode_attention(q: torch.Tensor, k_cache: torch.Tensor, v_cache: torch.Tensor, lens: torch.Tensor, Hq: int,
                     Hkv: int, D: int, scale: Optional[float] = None) -> torch.Tensor:
    """q ``[B, >=Hq*D]``, caches ``[B, max_len, Hkv, D]``; returns fp32 ``[B, Hq*D]``."""
    scale = D ** -0.5 if scale is None else scale
    B = lens.numel()
    out = []
    for b in range(B):
        L = int(lens[b])
        qb = q[b, : Hq * D].float().view(Hq, D)
        kb = k_cache[b, :L].float().repeat_interleave(Hq // Hkv, dim=1)  # [L, Hq, D]
        vb = v_cache[b, :L].float().repeat_interleave(Hq // Hkv, dim=1)
        s = torch.einsum("hd,lhd->hl", qb, kb) * scale
        p = torch.softmax(s, dim=-1)
        out.append(torch.einsum("hl,lhd->hd", p, vb).reshape(-1))
    return torch.stack(out)


def gelu(x):
    return F.gelu(x)
