"""BERT-base text classifier (BASELINE.json config 3) -- no reference counterpart (the
reference model is a constant stub, reference ``src/model/model.py:23-31``).

Paths over one parameter set (random init, std 0.02, as BERT's initializer_range):
  * :func:`bert_reference` -- fp32 PyTorch ops; the numerics oracle (runs on CPU too).
  * :class:`BertEager`      -- stock PyTorch-ROCm ops in bf16 (hipBLASLt GEMMs + SDPA):
                               the comparison baseline.
  * :class:`BertFused`      -- our CDNA4 kernels: fused word+pos+type embedding + LN, MFMA
                               GEMMs with bias / GELU / residual epilogues, MFMA flash attention
                               reading Q/K/V in place from the fused QKV projection with a
                               key-padding mask, LN kernels, tanh pooler and softmax/top-k head.

Post-LN encoder (as BERT):  x = LN(x + Attn(x));  x = LN(x + FFN(x)).
"""
from __future__ import annotations

import math
import os
import re
import zlib
from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence, Tuple

import torch
import torch.nn.functional as F


@dataclass
class BertConfig:
    vocab: int = 30522
    hidden: int = 768
    layers: int = 12
    heads: int = 12
    intermediate: int = 3072
    max_pos: int = 512
    type_vocab: int = 2
    eps: float = 1e-12
    num_labels: int = 2

    @property
    def head_dim(self) -> int:
        return self.hidden // self.heads


BERT_BASE = BertConfig()
CLS_ID, SEP_ID, PAD_ID, UNK_ID = 101, 102, 0, 100


_HF_BERT_FIXED = {
    "embeddings.word_embeddings.weight": "emb.word", "embeddings.position_embeddings.weight": "emb.pos",
    "embeddings.token_type_embeddings.weight": "emb.type", "embeddings.LayerNorm.weight": "emb.ln.g",
    "embeddings.LayerNorm.bias": "emb.ln.b", "pooler.dense.weight": "pooler.w", "pooler.dense.bias": "pooler.b",
    "classifier.weight": "cls.w", "classifier.bias": "cls.b",
}
_HF_BERT_LAYER = {
    "attention.self.query": "q", "attention.self.key": "k", "attention.self.value": "v",
    "attention.output.dense": "o", "attention.output.LayerNorm": "ln1", "intermediate.dense": "ffn1",
    "output.dense": "ffn2", "output.LayerNorm": "ln2",
}


def hf_bert_name(k: str) -> Optional[str]:
    """Hugging Face ``BertForSequenceClassification`` key -> this model's name (q/k/v kept apart
    here and fused into ``qkv`` by :func:`_fuse_qkv`)."""
    k = k[5:] if k.startswith("bert.") else k
    k = k.replace("LayerNorm.gamma", "LayerNorm.weight").replace("LayerNorm.beta", "LayerNorm.bias")
    if k.endswith("position_ids"):
        return None
    if k in _HF_BERT_FIXED:
        return _HF_BERT_FIXED[k]
    if k.startswith("encoder.layer."):
        rest = k[len("encoder.layer."):]
        i, sub = rest.split(".", 1)
        mod, leaf = sub.rsplit(".", 1)
        short = _HF_BERT_LAYER.get(mod)
        if short is None:
            return k
        if short.startswith("ln"):
            return f"l{i}.{short}.{'g' if leaf == 'weight' else 'b'}"
        return f"l{i}.{short}.{'w' if leaf == 'weight' else 'b'}"
    return k


def _fuse_qkv(state: Dict[str, torch.Tensor]) -> None:
    i = 0
    while f"l{i}.q.w" in state:
        for leaf in ("w", "b"):
            parts = [state.pop(f"l{i}.{n}.{leaf}") for n in ("q", "k", "v")]
            state[f"l{i}.qkv.{leaf}"] = torch.cat(parts, 0)
        i += 1


def load_bert(path: str, cfg: "BertConfig") -> Dict[str, torch.Tensor]:
    """fp32 parameters from a safetensors checkpoint in this model's names or Hugging Face's."""
    from ..utils.checkpoint import load_validated

    spec = {k: (shape, torch.float32) for k, (shape, _dt) in bert_spec(cfg).items()}
    return load_validated(path, spec, rename=lambda k: k if k in spec else hf_bert_name(k), combine=_fuse_qkv)


def init_bert(cfg: BertConfig = BERT_BASE, seed: int = 0, device="cpu", dtype=torch.float32) -> Dict[str, torch.Tensor]:
    g = torch.Generator(device=device).manual_seed(seed)

    def n(*shape):
        return (torch.randn(*shape, generator=g, device=device) * 0.02).to(dtype)

    def ones(c):
        return (1.0 + 0.1 * torch.randn(c, generator=g, device=device)).to(dtype)

    def small(c):
        return (0.02 * torch.randn(c, generator=g, device=device)).to(dtype)

    H, I = cfg.hidden, cfg.intermediate
    p = {
        "emb.word": n(cfg.vocab, H), "emb.pos": n(cfg.max_pos, H), "emb.type": n(cfg.type_vocab, H),
        "emb.ln.g": ones(H), "emb.ln.b": small(H),
        "pooler.w": n(H, H), "pooler.b": small(H),
        "cls.w": n(cfg.num_labels, H), "cls.b": small(cfg.num_labels),
    }
    for i in range(cfg.layers):
        p.update({
            f"l{i}.qkv.w": n(3 * H, H), f"l{i}.qkv.b": small(3 * H),
            f"l{i}.o.w": n(H, H), f"l{i}.o.b": small(H),
            f"l{i}.ln1.g": ones(H), f"l{i}.ln1.b": small(H),
            f"l{i}.ffn1.w": n(I, H), f"l{i}.ffn1.b": small(I),
            f"l{i}.ffn2.w": n(H, I), f"l{i}.ffn2.b": small(H),
            f"l{i}.ln2.g": ones(H), f"l{i}.ln2.b": small(H),
        })
    return p


def bert_spec(cfg: BertConfig = BERT_BASE) -> Dict[str, Tuple[Tuple[int, ...], torch.dtype]]:
    """Shapes/dtypes of :func:`init_bert` without materialising anything (X1 receivers)."""
    H, I = cfg.hidden, cfg.intermediate
    shapes = {"emb.word": (cfg.vocab, H), "emb.pos": (cfg.max_pos, H), "emb.type": (cfg.type_vocab, H),
              "emb.ln.g": (H,), "emb.ln.b": (H,), "pooler.w": (H, H), "pooler.b": (H,),
              "cls.w": (cfg.num_labels, H), "cls.b": (cfg.num_labels,)}
    for i in range(cfg.layers):
        shapes.update({f"l{i}.qkv.w": (3 * H, H), f"l{i}.qkv.b": (3 * H,), f"l{i}.o.w": (H, H), f"l{i}.o.b": (H,),
                       f"l{i}.ln1.g": (H,), f"l{i}.ln1.b": (H,), f"l{i}.ffn1.w": (I, H), f"l{i}.ffn1.b": (I,),
                       f"l{i}.ffn2.w": (H, I), f"l{i}.ffn2.b": (H,), f"l{i}.ln2.g": (H,), f"l{i}.ln2.b": (H,)})
    return {k: (v, torch.float32) for k, v in shapes.items()}


# ------------------------------------------------------------------------ tokenizer
_WORD = re.compile(r"[A-Za-z0-9]+|[^\sA-Za-z0-9]")


class HashTokenizer:
    """Deterministic offline tokenizer: no vocab file is available in this environment (no
    network), so words are hashed into the WordPiece id range.  With a ``vocab.txt`` the real
    WordPiece tokenizer (``tokenizers`` package) is used instead."""

    def __init__(self, vocab_size: int = 30522, vocab_file: Optional[str] = None, lowercase: bool = True):
        self.vocab_size = vocab_size
        self.lowercase = lowercase
        self._wp = None
        if vocab_file:
            from tokenizers import BertWordPieceTokenizer

            self._wp = BertWordPieceTokenizer(vocab_file, lowercase=lowercase)

    def encode(self, text: str, max_len: int = 512) -> List[int]:
        if self._wp is not None:
            return self._wp.encode(text).ids[:max_len]
        if self.lowercase:
            text = text.lower()
        ids = [CLS_ID]
        span = self.vocab_size - 1000
        for w in _WORD.findall(text):
            ids.append(1000 + zlib.crc32(w.encode("utf-8")) % span)
            if len(ids) >= max_len - 1:
                break
        ids.append(SEP_ID)
        return ids


# ------------------------------------------------------------------------ reference
def bert_reference(p: Dict[str, torch.Tensor], ids: torch.Tensor, type_ids: Optional[torch.Tensor],
                   lens: torch.Tensor, cfg: BertConfig = BERT_BASE) -> torch.Tensor:
    """ids ``[B, S]`` -> fp32 logits ``[B, num_labels]``."""
    B, S = ids.shape
    H, nh, hd = cfg.hidden, cfg.heads, cfg.head_dim
    f = {k: v.float() for k, v in p.items()}
    tt = torch.zeros_like(ids) if type_ids is None else type_ids
    x = f["emb.word"][ids.long()] + f["emb.pos"][:S].unsqueeze(0) + f["emb.type"][tt.long()]
    x = F.layer_norm(x, (H,), f["emb.ln.g"], f["emb.ln.b"], cfg.eps)
    mask = torch.arange(S, device=ids.device).view(1, S) < lens.view(B, 1).long()
    bias = torch.zeros(B, 1, 1, S, device=ids.device).masked_fill(~mask.view(B, 1, 1, S), float("-inf"))
    for i in range(cfg.layers):
        qkv = F.linear(x, f[f"l{i}.qkv.w"], f[f"l{i}.qkv.b"])
        q, k, v = qkv.split(H, dim=-1)
        q = q.view(B, S, nh, hd).transpose(1, 2)
        k = k.view(B, S, nh, hd).transpose(1, 2)
        v = v.view(B, S, nh, hd).transpose(1, 2)
        a = torch.softmax(q @ k.transpose(-1, -2) / math.sqrt(hd) + bias, dim=-1) @ v
        a = a.transpose(1, 2).reshape(B, S, H)
        x = F.layer_norm(x + F.linear(a, f[f"l{i}.o.w"], f[f"l{i}.o.b"]), (H,), f[f"l{i}.ln1.g"], f[f"l{i}.ln1.b"], cfg.eps)
        h = F.gelu(F.linear(x, f[f"l{i}.ffn1.w"], f[f"l{i}.ffn1.b"]))
        x = F.layer_norm(x + F.linear(h, f[f"l{i}.ffn2.w"], f[f"l{i}.ffn2.b"]), (H,), f[f"l{i}.ln2.g"], f[f"l{i}.ln2.b"], cfg.eps)
    pooled = torch.tanh(F.linear(x[:, 0], f["pooler.w"], f["pooler.b"]))
    return F.linear(pooled, f["cls.w"], f["cls.b"])


class BertEager:
    """Stock PyTorch-ROCm bf16 path (comparison baseline)."""

    def __init__(self, p: Dict[str, torch.Tensor], device, cfg: BertConfig = BERT_BASE):
        self.cfg = cfg
        self.p = {k: v.to(device=device, dtype=torch.bfloat16) for k, v in p.items()}

    @torch.no_grad()
    def forward(self, ids: torch.Tensor, type_ids: Optional[torch.Tensor], lens: torch.Tensor) -> torch.Tensor:
        cfg, p = self.cfg, self.p
        B, S = ids.shape
        H, nh, hd = cfg.hidden, cfg.heads, cfg.head_dim
        tt = torch.zeros_like(ids) if type_ids is None else type_ids
        x = p["emb.word"][ids.long()] + p["emb.pos"][:S].unsqueeze(0) + p["emb.type"][tt.long()]
        x = F.layer_norm(x, (H,), p["emb.ln.g"], p["emb.ln.b"], cfg.eps)
        mask = (torch.arange(S, device=ids.device).view(1, S) < lens.view(B, 1).long()).view(B, 1, 1, S)
        for i in range(cfg.layers):
            qkv = F.linear(x, p[f"l{i}.qkv.w"], p[f"l{i}.qkv.b"])
            q, k, v = (t.view(B, S, nh, hd).transpose(1, 2) for t in qkv.split(H, dim=-1))
            a = F.scaled_dot_product_attention(q, k, v, attn_mask=mask)
            a = a.transpose(1, 2).reshape(B, S, H)
            x = F.layer_norm(x + F.linear(a, p[f"l{i}.o.w"], p[f"l{i}.o.b"]), (H,), p[f"l{i}.ln1.g"], p[f"l{i}.ln1.b"], cfg.eps)
            h = F.gelu(F.linear(x, p[f"l{i}.ffn1.w"], p[f"l{i}.ffn1.b"]))
            x = F.layer_norm(x + F.linear(h, p[f"l{i}.ffn2.w"], p[f"l{i}.ffn2.b"]), (H,), p[f"l{i}.ln2.g"], p[f"l{i}.ln2.b"], cfg.eps)
        pooled = torch.tanh(F.linear(x[:, 0], p["pooler.w"], p["pooler.b"]))
        return F.linear(pooled, p["cls.w"], p["cls.b"])

    __call__ = forward




class BertFused:
    """BERT on the CDNA4 kernels; capturable (all shapes static per (batch, seq) bucket)."""

    def __init__(self, p: Dict[str, torch.Tensor], device, cfg: BertConfig = BERT_BASE):
        from .. import ops

        self.ops = ops
        self.cfg = cfg
        self.device = torch.device(device)
        bf = lambda t: t.to(device=self.device, dtype=torch.bfloat16).contiguous()  # noqa: E731
        f32 = lambda t: t.to(device=self.device, dtype=torch.float32).contiguous()  # noqa: E731
        self.w = {}
        for k, v in p.items():
            if k.endswith(".b") and not k.startswith("emb.ln") and ".ln" not in k:
                self.w[k] = f32(v)  # GEMM epilogue biases in fp32
            else:
                self.w[k] = bf(v)
        # classifier padded to a multiple of 8 output columns; padded logits pinned to -1e30
        C = cfg.num_labels
        Cp = (C + 7) // 8 * 8
        self.num_labels = C
        cw = torch.zeros(Cp, cfg.hidden, device=self.device, dtype=torch.bfloat16)
        cw[:C] = self.w["cls.w"]
        cb = torch.full((Cp,), -1e30, device=self.device, dtype=torch.float32)
        cb[:C] = self.w["cls.b"]
        self.cls_w, self.cls_b = cw, cb
        self._ws = ops.StreamWorkspace(16 << 20, self.device)  # per stream: concurrent engine slots
        self._cls_idx: Dict = {}
        # LayerNorm folding (csrc/gemm_tile.hip "LayerNorm folding"): LN1 of layer i folds into its
        # FFN-up projection, LN2 of layer i - 1 into layer i's QKV projection; the residual adds
        # after them normalize their residual operand in the epilogue.  No LN kernel runs between
        # the encoder layers' GEMMs (the last layer, which runs on the [CLS] rows only, keeps them).
        # Folded from the bf16 weights / LN parameters the unfolded path uses; the residual adds that
        # normalize their residual take that LN's beta in their bias.
        self.ln_fold = os.environ.get("MLS_BERT_LN_FOLD", "1") != "0"
        # last layer: Q and attention of the [CLS] rows only (MLS_BERT_CLS_Q=0: all rows, then gather)
        self.cls_q = os.environ.get("MLS_BERT_CLS_Q", "1") != "0"
        self._fold: Dict[str, torch.Tensor] = {}
        if self.ln_fold:
            w, fw = self.w, self._fold
            for i in range(cfg.layers):
                g1, b1 = w[f"l{i}.ln1.g"].float(), w[f"l{i}.ln1.b"].float()
                fw[f"l{i}.ffn1.w"], fw[f"l{i}.ffn1.c"], fw[f"l{i}.ffn1.b"] = \
                    ops.fold_layernorm(w[f"l{i}.ffn1.w"], w[f"l{i}.ffn1.b"], g1, b1)
                fw[f"l{i}.ln1.g"] = g1.contiguous()
                fw[f"l{i}.ffn2.b"] = (w[f"l{i}.ffn2.b"] + b1).contiguous()
                g2, b2 = w[f"l{i}.ln2.g"].float(), w[f"l{i}.ln2.b"].float()
                fw[f"l{i}.ln2.g"] = g2.contiguous()
                if i + 1 < cfg.layers:
                    j = i + 1
                    fw[f"l{j}.qkv.w"], fw[f"l{j}.qkv.c"], fw[f"l{j}.qkv.b"] = \
                        ops.fold_layernorm(w[f"l{j}.qkv.w"], w[f"l{j}.qkv.b"], g2, b2)
                    fw[f"l{j}.o.b"] = (w[f"l{j}.o.b"] + b2).contiguous()

    def forward(self, ids: torch.Tensor, type_ids: Optional[torch.Tensor], lens: torch.Tensor) -> torch.Tensor:
        """ids/type_ids int32 ``[B, S]``, lens int32 ``[B]`` -> bf16 logits ``[B, Cpad]``."""
        ops, cfg, w = self.ops, self.cfg, self.w
        B, S = ids.shape
        ids_f = ids.reshape(-1)
        tt_f = type_ids.reshape(-1) if type_ids is not None else None
        x = ops.embed_layernorm(ids_f, tt_f, w["emb.word"], w["emb.pos"], w["emb.type"], w["emb.ln.g"], w["emb.ln.b"],
                                S, eps=cfg.eps)
        return self._encode(x, lens, B, S)

    __call__ = forward

    def forward_packed(self, x: torch.Tensor, seq_len: int) -> torch.Tensor:
        """The engine's packed request rows ``[B, 2S + 1]`` (ids | type ids | length) -> logits; the
        embedding kernel reads the rows in place and copies the lengths out (no unpacking copies)."""
        ops, cfg, w = self.ops, self.cfg, self.w
        emb, lens = ops.embed_layernorm_packed(x, seq_len, w["emb.word"], w["emb.pos"], w["emb.type"], w["emb.ln.g"],
                                               w["emb.ln.b"], eps=cfg.eps)
        return self._encode(emb, lens, x.shape[0], seq_len)

    def _cls_rows(self, B: int, S: int) -> torch.Tensor:
        """int32 [B] row index of every sequence's first ([CLS]) token (cached: no launch in a graph)."""
        key = (B, S)
        if key not in self._cls_idx:
            self._cls_idx[key] = torch.arange(B, device=self.device, dtype=torch.int32) * S
        return self._cls_idx[key]

    def _encode(self, x: torch.Tensor, lens: torch.Tensor, B: int, S: int) -> torch.Tensor:
        ops, cfg, w = self.ops, self.cfg, self.w
        ws = self._ws.get()
        cls = self._cls_rows(B, S)
        last = cfg.layers - 1
        H, T, eps, fw = cfg.hidden, B * S, cfg.eps, self._fold
        # the LN'd width (hidden) travels as 128-column partials read two per lane: H % 256, H <= 1024
        fold = self.ln_fold and H % 256 == 0 and H <= 1024 and all(ops.ln_foldable(T, n, k) for n, k in (
            (3 * H, H), (H, H), (cfg.intermediate, H), (H, cfg.intermediate)))
        # fold: h = the previous layer's raw pre-LN2 rows (its LN2 output is never formed); part[cur] =
        # the row statistics (partials) of the rows whose LN the next consumer applies, written by the
        # residual projection that produced them (two buffers: a producer reads one, writes the other)
        part = [ops.ln_partials(T, H, x.device) for _ in range(2)] if fold else None
        cur, h = 0, None
        for i in range(cfg.layers):
            # all four projections native (ops.linear: the LDS-DMA tile kernel from TILE_MIN_M tokens,
            # the conv_gemm tiles below); the residual rides in the o / FFN-down epilogues
            if i == last and not self.cls_q:  # A/B arm: full QKV + attention, then the [CLS] rows
                if h is None:
                    qkv = ops.linear(x, w[f"l{i}.qkv.w"], w[f"l{i}.qkv.b"], workspace=ws)
                    x = ops.embedding(cls, x)
                else:
                    qkv = ops.linear_ln(h, fw[f"l{i}.qkv.w"], fw[f"l{i}.qkv.b"], fold_c=fw[f"l{i}.qkv.c"],
                                        ln_part=part[cur], eps=eps)
                    x = ops.layernorm(ops.embedding(cls, h), w[f"l{i - 1}.ln2.g"], w[f"l{i - 1}.ln2.b"], eps=eps)
                    h = None
                a = ops.embedding(cls, ops.flash_attention(qkv, B, S, cfg.heads, cfg.heads, cfg.head_dim,
                                                           kv_lens=lens))
            elif i == last:
                # the classifier reads only the [CLS] rows of the last layer: the keys / values need
                # every token, but the queries and everything after the attention are per token --
                # K / V of all B*S rows (the K / V rows of the QKV projection), Q, attention (one
                # query per sequence) and the rest of the layer on the B [CLS] rows (native row
                # gather) instead of all B*S (~1/12 of the attention and ~6 % of the GEMM FLOPs)
                if h is not None:  # the previous layer's LN2: folded into K / V, explicit on [CLS]
                    x = ops.layernorm(ops.embedding(cls, h), w[f"l{i - 1}.ln2.g"], w[f"l{i - 1}.ln2.b"], eps=eps)
                    kv = ops.linear_ln(h, fw[f"l{i}.qkv.w"][H:], fw[f"l{i}.qkv.b"][H:],
                                       fold_c=fw[f"l{i}.qkv.c"][H:], ln_part=part[cur], eps=eps)
                    h = None
                else:
                    kv = ops.linear(x, w[f"l{i}.qkv.w"][H:], w[f"l{i}.qkv.b"][H:], workspace=ws)
                    x = ops.embedding(cls, x)
                q = ops.linear(x, w[f"l{i}.qkv.w"][:H], w[f"l{i}.qkv.b"][:H], workspace=ws)
                a = ops.flash_attention_rows(q, kv, B, S, 1, cfg.heads, cfg.heads, cfg.head_dim, kv_lens=lens)
            else:
                if h is None:
                    qkv = ops.linear(x, w[f"l{i}.qkv.w"], w[f"l{i}.qkv.b"], workspace=ws)
                else:
                    qkv = ops.linear_ln(h, fw[f"l{i}.qkv.w"], fw[f"l{i}.qkv.b"], fold_c=fw[f"l{i}.qkv.c"],
                                        ln_part=part[cur], eps=eps)
                a = ops.flash_attention(qkv, B, S, cfg.heads, cfg.heads, cfg.head_dim, kv_lens=lens)
            if fold and i < last:
                if h is None:
                    h1 = ops.linear_ln(a, w[f"l{i}.o.w"], w[f"l{i}.o.b"], residual=x, stats_part=part[1 - cur])
                else:
                    h1 = ops.linear_ln(a, w[f"l{i}.o.w"], fw[f"l{i}.o.b"], residual=h, ln_part=part[cur],
                                       ln_g=fw[f"l{i - 1}.ln2.g"], stats_part=part[1 - cur], eps=eps)
                cur = 1 - cur
                f1 = ops.linear_ln(h1, fw[f"l{i}.ffn1.w"], fw[f"l{i}.ffn1.b"], act=ops.ACT_GELU,
                                   fold_c=fw[f"l{i}.ffn1.c"], ln_part=part[cur], eps=eps)
                h = ops.linear_ln(f1, w[f"l{i}.ffn2.w"], fw[f"l{i}.ffn2.b"], residual=h1, ln_part=part[cur],
                                  ln_g=fw[f"l{i}.ln1.g"], stats_part=part[1 - cur], eps=eps)
                cur = 1 - cur
                continue
            hh = ops.linear(a, w[f"l{i}.o.w"], w[f"l{i}.o.b"], residual=x, workspace=ws)
            x = ops.layernorm(hh, w[f"l{i}.ln1.g"], w[f"l{i}.ln1.b"], eps=eps)
            f1 = ops.linear(x, w[f"l{i}.ffn1.w"], w[f"l{i}.ffn1.b"], act=ops.ACT_GELU, workspace=ws)
            hh = ops.linear(f1, w[f"l{i}.ffn2.w"], w[f"l{i}.ffn2.b"], residual=x, workspace=ws)
            x = ops.layernorm(hh, w[f"l{i}.ln2.g"], w[f"l{i}.ln2.b"], eps=eps)
        pooled = ops.gemm(x, w["pooler.w"], w["pooler.b"], act=ops.ACT_TANH, workspace=ws)  # x: the [CLS] rows
        return ops.gemm(pooled, self.cls_w, self.cls_b, workspace=ws)

    def classify(self, ids, type_ids, lens, k: int = 2):
        logits = self.forward(ids, type_ids, lens)
        return self.ops.softmax_topk(logits, min(k, self.num_labels))

    def classify_packed(self, x: torch.Tensor, seq_len: int, k: int = 2):
        return self.ops.softmax_topk(self.forward_packed(x, seq_len), min(k, self.num_labels))


def pack_requests(token_lists: Sequence[Sequence[int]], seq_len: int) -> torch.Tensor:
    """Engine sample layout for one seq bucket: int32 ``[n, 2*S + 1]`` = ids | type ids | length."""
    n = len(token_lists)
    out = torch.zeros(n, 2 * seq_len + 1, dtype=torch.int32)
    for i, t in enumerate(token_lists):
        t = list(t)[:seq_len]
        out[i, : len(t)] = torch.tensor(t, dtype=torch.int32)
        out[i, 2 * seq_len] = len(t)
    return out


def unpack_requests(x: torch.Tensor, seq_len: int):
    ids = x[:, :seq_len].contiguous()
    tt = x[:, seq_len: 2 * seq_len].contiguous()
    lens = x[:, 2 * seq_len].contiguous()
    return ids, tt, lens
