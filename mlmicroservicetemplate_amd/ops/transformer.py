"""Transformer ops: norms, embeddings, RoPE, KV cache writes, flash / decode attention, the on-device token pick."""
from __future__ import annotations

import os
from typing import Optional

import torch

from ._lib import check, lib, stream_ptr
from ._core import ACT_NONE, _need, _ptr


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


def embed_layernorm_packed(x: torch.Tensor, seq_len: int, word: torch.Tensor, pos: torch.Tensor, typ: torch.Tensor,
                           gamma: torch.Tensor, beta: torch.Tensor, eps: float = 1e-12):
    """:func:`embed_layernorm` straight from the engine's packed request rows ``x`` int32
    ``[B, 2S + 1]`` = ids | type ids | length (``models.bert.pack_requests``): no unpacking copies.
    Returns ``(out [B*S, D] bf16, lens [B] int32)`` -- the lengths copied out by the same launch."""
    dev = x.device
    _need(x, "x", torch.int32, dev)
    B, W = x.shape
    S = int(seq_len)
    if W != 2 * S + 1 or not x.is_contiguous():
        raise ValueError("x must be contiguous int32 [B, 2*S + 1]")
    D = word.shape[1]
    out = torch.empty(B * S, D, device=dev, dtype=torch.bfloat16)
    lens = torch.empty(B, device=dev, dtype=torch.int32)
    base = x.data_ptr()
    rc = lib().mls_embed_ln2(base, base + 4 * S, W, base + 8 * S, lens.data_ptr(), word.data_ptr(), pos.data_ptr(),
                             typ.data_ptr(), gamma.data_ptr(), beta.data_ptr(), out.data_ptr(), B * S, S, D,
                             word.shape[0], float(eps), stream_ptr(dev))
    check(rc, "mls_embed_ln2")
    return out, lens


def prefill_slots(pos: torch.Tensor, lens: torch.Tensor, B: int, S: int, slot_ids: Optional[torch.Tensor] = None,
                  table: Optional[torch.Tensor] = None, page_rows: int = 0, max_seq: int = 0) -> torch.Tensor:
    """KV-cache row of every prefill token (int32 ``[B*S]``, -1 = past the sequence's length): batch
    row b = t // S (or ``slot_ids[b]``), position ``pos[t]``; through the page ``table``
    ``[slots][pages]`` (``page_rows`` rows each) or ``slot * max_seq + pos``.  One launch."""
    dev = pos.device
    _need(pos, "pos", torch.int32, dev)
    _need(lens, "lens", torch.int32, dev)
    if slot_ids is not None:
        _need(slot_ids, "slot_ids", torch.int32, dev)
    if table is not None:
        _need(table, "table", torch.int32, dev)
    out = torch.empty(B * S, device=dev, dtype=torch.int32)
    rc = lib().mls_prefill_slots(pos.data_ptr(), lens.data_ptr(), _ptr(slot_ids), _ptr(table),
                                 table.shape[1] if table is not None else 0, page_rows, max_seq, B, S, out.data_ptr(),
                                 stream_ptr(dev))
    check(rc, "mls_prefill_slots")
    return out


def last_rows(x: torch.Tensor, lens: torch.Tensor, B: int, S: int, x2: Optional[torch.Tensor] = None):
    """Row ``b * S + lens[b] - 1`` of ``x`` (and of ``x2``) for every sequence: ``[B, D]`` (pair)."""
    dev = x.device
    _need(x, "x", torch.bfloat16, dev)
    _need(lens, "lens", torch.int32, dev)
    D = x.shape[-1]
    out = torch.empty(B, D, device=dev, dtype=torch.bfloat16)
    out2 = None
    if x2 is not None:
        _need(x2, "x2", torch.bfloat16, dev)
        out2 = torch.empty(B, D, device=dev, dtype=torch.bfloat16)
    rc = lib().mls_last_rows(x.data_ptr(), _ptr(x2), lens.data_ptr(), B, S, D, out.data_ptr(), _ptr(out2),
                             stream_ptr(dev))
    check(rc, "mls_last_rows")
    return out if x2 is None else (out, out2)


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


def flash_attention_rows(q: torch.Tensor, kv: torch.Tensor, batch: int, seq: int, q_rows: int, n_q_heads: int,
                         n_kv_heads: int, head_dim: int, *, kv_lens: Optional[torch.Tensor] = None,
                         causal: bool = False, scale: Optional[float] = None,
                         out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Attention of the first ``q_rows`` positions of every sequence against all of its keys:
    ``q [B*q_rows, >= Hq*D]`` (row-strided), ``kv [B*S, 2*Hkv*D]`` (K then V, e.g. a fused K/V
    projection).  Returns ``[B*q_rows, Hq*D]``.  BERT's last layer runs its [CLS] rows this way
    (``q_rows = 1``: one wave per (sequence, head))."""
    dev = q.device
    if q.dtype != torch.bfloat16:  # row-strided: not _need's contiguity check
        raise TypeError(f"q: expected torch.bfloat16, got {q.dtype}")
    _need(kv, "kv", torch.bfloat16, dev)
    HD, KD = n_q_heads * head_dim, n_kv_heads * head_dim
    if q.dim() != 2 or q.shape[0] != batch * q_rows or q.shape[1] < HD or q.stride(1) != 1:
        raise ValueError("q must be [batch * q_rows, >= Hq*D] with unit column stride")
    if tuple(kv.shape) != (batch * seq, 2 * KD) or not kv.is_contiguous():
        raise ValueError("kv must be a contiguous [batch * seq, 2 * Hkv * D]")
    if not 0 < q_rows <= seq:
        raise ValueError("q_rows must be in 1..seq")
    if kv_lens is not None:
        _need(kv_lens, "kv_lens", torch.int32, dev)
    out = torch.empty(batch * q_rows, HD, device=dev, dtype=torch.bfloat16) if out is None else out
    scale = head_dim ** -0.5 if scale is None else scale
    es = kv.element_size()
    rc = lib().mls_flash_attention_rows(q.data_ptr(), kv.data_ptr(), kv.data_ptr() + KD * es, out.data_ptr(),
                                        q.stride(0), 2 * KD, 2 * KD, out.stride(0), batch, seq, q_rows, n_q_heads,
                                        n_kv_heads, head_dim, _ptr(kv_lens), int(causal), float(scale),
                                        stream_ptr(dev))
    check(rc, "mls_flash_attention_rows")
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


def skinny_packed_combine_ar(attn_out: torch.Tensor, parts: DecodePartials, wp: torch.Tensor, N: int, car, *,
                             variant: int = 9) -> torch.Tensor:
    """:func:`skinny_packed_combine` for a row-parallel TP o-projection with its all-reduce fused into
    the same launch (csrc/ar_protocol.h): the split-KV combine in the prologue, the one-shot IPC
    all-reduce of the output in the epilogue -- one kernel where there were three."""
    dev = attn_out.device
    _need(attn_out, "attn_out", torch.bfloat16, dev)
    M, K = attn_out.shape
    if M > 4 or K != parts.n_q_heads * parts.head_dim or wp.numel() != N * K or M * K * 2 > 65536:
        raise ValueError("skinny_packed_combine_ar: M <= 4, K == Hq * D, M * K * 2 <= 64 KiB, wp of N*K elements")
    out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    rc = lib().mls_skinny_packed_combine_ar(attn_out.data_ptr(), parts.ws.data_ptr(), parts.ws_ml.data_ptr(),
                                            parts.lens.data_ptr(), parts.nsplit, parts.chunk, parts.n_q_heads,
                                            parts.head_dim, wp.data_ptr(), out.data_ptr(), M, N, K, int(variant),
                                            car.ctx_ptr(), stream_ptr(dev))
    check(rc, "mls_skinny_packed_combine_ar")
    return out


def decode_pick(cand_v: torch.Tensor, cand_i: torch.Tensor, tok: torch.Tensor, pos: torch.Tensor, lens: torch.Tensor,
                step: torch.Tensor, *, topk: Optional[torch.Tensor] = None, temp: Optional[torch.Tensor] = None,
                seed: Optional[torch.Tensor] = None, hist: Optional[torch.Tensor] = None,
                rows: Optional[torch.Tensor] = None, active: Optional[torch.Tensor] = None,
                emit: Optional[torch.Tensor] = None) -> None:
    """X4 merge + next-token pick on device (csrc/decode_pick.hip): ``cand_v`` / ``cand_i`` are the
    all-gathered ``[tp, B, k]`` candidates; per row picks greedily (``topk <= 1``) or samples
    (top-k, temperature, counter-based ``seed`` x step draw -- :func:`models.llama.sample_uniform`),
    then advances ``tok`` / ``pos`` / ``lens`` / ``step`` in place and records the token in
    ``hist[., step]``.  Capturable (the TP decode graph ends with it).

    Serving (``models/llama_serving.ContinuousLlama``): the per-sequence state arrays may have more
    rows than ``B`` -- ``rows`` int32 ``[B]`` maps candidate row b to its state row (a prefill of new
    sequences into their slots), ``active`` int32 skips idle state rows, ``emit`` int32 receives
    each picked token at its state row."""
    dev = cand_v.device
    tp, B, k = cand_v.shape
    _need(cand_v, "cand_v", torch.float32, dev)
    _need(cand_i, "cand_i", torch.int32, dev)
    if tuple(cand_i.shape) != (tp, B, k) or tp * k > 512:
        raise ValueError("cand_i must match cand_v [tp, B, k] with tp * k <= 512")
    S = tok.numel()  # state rows
    if rows is None and S != B:
        raise ValueError(f"tok must have {B} elements")
    if rows is not None:
        _need(rows, "rows", torch.int32, dev)
        if rows.numel() != B:
            raise ValueError(f"rows must have {B} elements")
    for name, t, dt in (("tok", tok, torch.int32), ("pos", pos, torch.int32), ("lens", lens, torch.int32),
                        ("step", step, torch.int32)):
        _need(t, name, dt, dev)
        if t.numel() != S:
            raise ValueError(f"{name} must have {S} elements")
    for name, t, dt in (("topk", topk, torch.int32), ("temp", temp, torch.float32), ("seed", seed, torch.int64),
                        ("active", active, torch.int32), ("emit", emit, torch.int32)):
        if t is not None:
            _need(t, name, dt, dev)
            if t.numel() != S:
                raise ValueError(f"{name} must have {S} elements")
    cols = 0
    if hist is not None:
        _need(hist, "hist", torch.int32, dev)
        if hist.shape[0] != S:
            raise ValueError("hist must be [state rows, cols]")
        cols = hist.shape[1]
    rc = lib().mls_decode_pick(cand_v.data_ptr(), cand_i.data_ptr(), tp, B, k, _ptr(topk), _ptr(temp), _ptr(seed),
                               tok.data_ptr(), pos.data_ptr(), lens.data_ptr(), _ptr(hist), cols, step.data_ptr(),
                               _ptr(rows), _ptr(active), _ptr(emit), stream_ptr(dev))
    check(rc, "mls_decode_pick")
