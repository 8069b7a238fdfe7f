"""Llama-3-8B generation with Megatron-style tensor parallelism (BASELINE.json config 5, P3/P6
of SURVEY.md §2.E.3).  No reference counterpart (the reference model is a stub).

Sharding per rank r of ``tp`` (one process per GPU, RCCL over xGMI):
  * column-parallel: fused QKV (``hq = heads/tp`` query heads, ``hkv = kv_heads/tp`` KV heads),
    fused gate/up (``I/tp`` rows each, interleaved for the SiLU-mul epilogue);
  * row-parallel: o_proj and down_proj -> one all-reduce each per layer (X2, 2 x 32 / forward);
  * vocab-parallel embedding (out-of-shard ids give zero rows, then all-reduce, X3) and lm_head
    (each rank takes a local top-k of its 16032-row shard; ranks all-gather only k candidates
    per sequence and merge -- X4 -- instead of gathering 128256 logits).
The residual add is fused into the RMSNorm kernel AFTER the all-reduce (adding the replicated
residual before it would count it ``tp`` times).

Two backends with identical structure and communication:
  * ``reference``: plain PyTorch fp32 math on bf16 weights (runs on CPU with gloo -- the TP
    logic is tested there against TP=1);
  * ``fused``: the CDNA4 kernels (MFMA GEMMs with fused SiLU-mul, RMSNorm+residual, RoPE,
    KV-cache append, MFMA flash-attention prefill, split-KV decode attention, top-k).
Weights are random-init (std 0.02) and generated per tensor from a (seed, name) generator on
the target device, then sliced to the rank's shard -- every rank gets exactly the slice of the
same full model, without any rank materialising the whole 8B model.
"""
from __future__ import annotations

import hashlib
import os
import re
import zlib
from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist
import torch.nn.functional as F

from ..ops import reference as R
from ..utils import tracing

# int32 words of the serving loop's control row (op, admissions, longest prompt, iteration check):
# rank 0's next-iteration header, carried by the decode step's X4 gather (serve_graph)
CTL_WORDS = 4


@dataclass
class LlamaConfig:
    vocab: int = 128256
    hidden: int = 4096
    layers: int = 32
    heads: int = 32
    kv_heads: int = 8
    head_dim: int = 128
    intermediate: int = 14336
    rope_theta: float = 500000.0
    eps: float = 1e-5
    bos_id: int = 128000
    eos_ids: Tuple[int, ...] = (128001, 128009)


LLAMA3_8B = LlamaConfig()


def tiny_config(**kw) -> LlamaConfig:
    base = dict(vocab=2048, hidden=256, layers=2, heads=8, kv_heads=4, head_dim=32, intermediate=512, bos_id=1,
                eos_ids=(2,))
    base.update(kw)
    return LlamaConfig(**base)


@dataclass
class ShardDims:
    tp: int
    rank: int
    hq: int
    hkv: int
    inter: int
    vocab_shard: int
    vocab_lo: int

    @property
    def qkv_rows(self) -> int:
        return 0


def shard_dims(cfg: LlamaConfig, tp: int, rank: int) -> ShardDims:
    if cfg.heads % tp or cfg.intermediate % tp:
        raise ValueError(f"tp={tp} must divide heads and intermediate")
    hkv = cfg.kv_heads // tp if cfg.kv_heads >= tp else 1
    if cfg.kv_heads >= tp and cfg.kv_heads % tp:
        raise ValueError("tp must divide kv_heads (or exceed it)")
    vs = -(-cfg.vocab // tp)
    vs = (vs + 7) // 8 * 8
    return ShardDims(tp, rank, cfg.heads // tp, hkv, cfg.intermediate // tp, vs, rank * vs)


def _gen(seed: int, name: str, device) -> torch.Generator:
    h = int.from_bytes(hashlib.sha256(f"{seed}:{name}".encode()).digest()[:8], "little") & ((1 << 63) - 1)
    g = torch.Generator(device=device)
    g.manual_seed(h)
    return g


def _full(seed, name, shape, device, kind="normal"):
    g = _gen(seed, name, device)
    if kind == "norm":
        return 1.0 + 0.1 * torch.randn(*shape, generator=g, device=device)
    return torch.randn(*shape, generator=g, device=device) * 0.02


class RandomSource:
    """Deterministic random-init weights: every full tensor is generated from (seed, name), so
    any TP shard of it is identical to the same slice at tp=1."""

    def __init__(self, seed: int = 0, device="cpu"):
        self.seed, self.device = seed, device

    def region(self, name: str, shape, kind: str = "normal", rows: Optional[slice] = None,
               cols: Optional[slice] = None) -> torch.Tensor:
        t = _full(self.seed, name, shape, self.device, kind)
        if rows is not None:
            t = t[rows]
        if cols is not None:
            t = t[:, cols]
        return t


def hf_llama_name(name: str) -> str:
    """Canonical name (``l3.q``, ``embed``, ...) -> Hugging Face Llama safetensors key."""
    fixed = {"embed": "model.embed_tokens.weight", "lm_head": "lm_head.weight", "final_norm": "model.norm.weight"}
    if name in fixed:
        return fixed[name]
    layer, part = name[1:].split(".", 1)
    sub = {"q": "self_attn.q_proj", "k": "self_attn.k_proj", "v": "self_attn.v_proj", "o": "self_attn.o_proj",
           "gate": "mlp.gate_proj", "up": "mlp.up_proj", "down": "mlp.down_proj",
           "attn_norm": "input_layernorm", "mlp_norm": "post_attention_layernorm"}[part]
    return f"model.layers.{layer}.{sub}.weight"


class CheckpointSource:
    """Weights from a safetensors file / shard directory, canonical or Hugging Face names.  Each
    TP rank reads only its slice of every matrix (memory-mapped region reads); a checkpoint
    without ``lm_head`` (tied embeddings) reuses ``embed``."""

    def __init__(self, path: str, device="cpu"):
        from ..utils.checkpoint import Checkpoint

        self.ck = Checkpoint(path)
        self.device = device

    def _key(self, name: str) -> str:
        from ..utils.checkpoint import CheckpointError

        for k in (name, hf_llama_name(name)):
            if k in self.ck:
                return k
        if name == "lm_head":
            return self._key("embed")
        raise CheckpointError(f"{self.ck.path}: no tensor for {name!r} (or {hf_llama_name(name)!r})")

    def region(self, name: str, shape, kind: str = "normal", rows: Optional[slice] = None,
               cols: Optional[slice] = None) -> torch.Tensor:
        from ..utils.checkpoint import CheckpointError

        key = self._key(name)
        have = self.ck.shape(key)
        if tuple(have) != tuple(shape):
            raise CheckpointError(f"{self.ck.path}: {key} has shape {tuple(have)}, config expects {tuple(shape)}")
        return self.ck.get_region(key, rows, cols).to(device=self.device, dtype=torch.float32)


def init_llama_shard(cfg: LlamaConfig, tp: int = 1, rank: int = 0, seed: int = 0, device="cpu",
                     dtype=torch.bfloat16, source=None) -> Dict[str, torch.Tensor]:
    """This rank's shard of a Llama: from ``source`` (:class:`CheckpointSource`) or a
    deterministic random init (:class:`RandomSource`, the same full model for every tp)."""
    src = source if source is not None else RandomSource(seed, device)
    sd = shard_dims(cfg, tp, rank)
    H, D = cfg.hidden, cfg.head_dim
    kv_rep = cfg.kv_heads < tp  # more ranks than KV heads: replicate a head over tp/kv_heads ranks
    p: Dict[str, torch.Tensor] = {}

    def vocab_rows(name):
        lo, hi = sd.vocab_lo, min(cfg.vocab, sd.vocab_lo + sd.vocab_shard)
        out = torch.zeros(sd.vocab_shard, H, device=device)
        if hi > lo:
            out[: hi - lo] = src.region(name, (cfg.vocab, H), rows=slice(lo, hi)).to(device)
        return out.to(dtype)

    p["embed"] = vocab_rows("embed")
    p["lm_head"] = vocab_rows("lm_head")
    p["final_norm"] = src.region("final_norm", (H,), "norm").to(device=device, dtype=dtype)
    qs = slice(rank * sd.hq * D, (rank + 1) * sd.hq * D)
    kvh = (rank * cfg.kv_heads) // tp if kv_rep else rank * sd.hkv
    ks = slice(kvh * D, (kvh + sd.hkv) * D)
    sl = slice(rank * sd.inter, (rank + 1) * sd.inter)
    for i in range(cfg.layers):
        q = src.region(f"l{i}.q", (cfg.heads * D, H), rows=qs)
        k = src.region(f"l{i}.k", (cfg.kv_heads * D, H), rows=ks)
        v = src.region(f"l{i}.v", (cfg.kv_heads * D, H), rows=ks)
        p[f"l{i}.qkv"] = torch.cat([q, k, v]).to(device=device, dtype=dtype).contiguous()
        p[f"l{i}.o"] = src.region(f"l{i}.o", (H, cfg.heads * D), cols=qs).to(device=device, dtype=dtype).contiguous()
        p[f"l{i}.gate"] = src.region(f"l{i}.gate", (cfg.intermediate, H), rows=sl).to(device=device,
                                                                                      dtype=dtype).contiguous()
        p[f"l{i}.up"] = src.region(f"l{i}.up", (cfg.intermediate, H), rows=sl).to(device=device,
                                                                                  dtype=dtype).contiguous()
        p[f"l{i}.down"] = src.region(f"l{i}.down", (H, cfg.intermediate), cols=sl).to(device=device,
                                                                                      dtype=dtype).contiguous()
        p[f"l{i}.attn_norm"] = src.region(f"l{i}.attn_norm", (H,), "norm").to(device=device, dtype=dtype)
        p[f"l{i}.mlp_norm"] = src.region(f"l{i}.mlp_norm", (H,), "norm").to(device=device, dtype=dtype)
        del q, k, v
    return p


def full_llama_state(cfg: LlamaConfig, seed: int = 0, dtype=torch.bfloat16) -> Dict[str, torch.Tensor]:
    """The unsharded random-init model under canonical names (what ``export-weights`` writes)."""
    src = RandomSource(seed)
    H, D = cfg.hidden, cfg.head_dim
    out = {"embed": src.region("embed", (cfg.vocab, H)), "lm_head": src.region("lm_head", (cfg.vocab, H)),
           "final_norm": src.region("final_norm", (H,), "norm")}
    for i in range(cfg.layers):
        for n, shp, kind in (("q", (cfg.heads * D, H), "normal"), ("k", (cfg.kv_heads * D, H), "normal"),
                             ("v", (cfg.kv_heads * D, H), "normal"), ("o", (H, cfg.heads * D), "normal"),
                             ("gate", (cfg.intermediate, H), "normal"), ("up", (cfg.intermediate, H), "normal"),
                             ("down", (H, cfg.intermediate), "normal"), ("attn_norm", (H,), "norm"),
                             ("mlp_norm", (H,), "norm")):
            out[f"l{i}.{n}"] = src.region(f"l{i}.{n}", shp, kind)
    return {k: v.to(dtype) for k, v in out.items()}


# --------------------------------------------------------------------------- tokenizer
class LlamaTokenizer:
    """Offline tokenizer: with a ``tokenizer.json`` the real BPE (``tokenizers``) is used;
    otherwise words are hashed into the vocab (synthetic ids) and decoded as ``<id>``."""

    _WORD = re.compile(r"\w+|[^\w\s]")

    def __init__(self, cfg: LlamaConfig, tokenizer_file: Optional[str] = None):
        self.cfg = cfg
        self._tok = None
        if tokenizer_file:
            from tokenizers import Tokenizer

            self._tok = Tokenizer.from_file(tokenizer_file)

    def encode(self, text: str) -> List[int]:
        if self._tok is not None:
            return [self.cfg.bos_id] + self._tok.encode(text).ids
        span = self.cfg.vocab - 1024
        return [self.cfg.bos_id] + [256 + zlib.crc32(w.encode()) % span for w in self._WORD.findall(text)]

    def decode(self, ids: Sequence[int]) -> str:
        if self._tok is not None:
            return self._tok.decode(list(ids))
        return " ".join(f"<{i}>" for i in ids)


# --------------------------------------------------------------------------- comm
class _ARDone:
    """A collective that already completed in stream order (or needed none)."""

    __slots__ = ("t",)

    def __init__(self, t: torch.Tensor):
        self.t = t

    def wait(self) -> torch.Tensor:
        return self.t


class _ARPending:
    """An all-reduce in flight on the backend's own stream (RCCL: ProcessGroupNCCL's NCCL stream,
    ordered after the producer on the current stream); :meth:`wait` orders the current stream
    after it -- the compute between start and wait overlaps the transfer."""

    __slots__ = ("t", "work")

    def __init__(self, t: torch.Tensor, work):
        self.t, self.work = t, work

    def wait(self) -> torch.Tensor:
        with tracing.range("tp.all_reduce_wait"):
            self.work.wait()
        return self.t


class TPComm:
    """Tensor-parallel collectives over a torch.distributed group (RCCL on GPU, gloo on CPU)."""

    def __init__(self, group=None, tp: int = 1, device=None, custom_ar: Optional[bool] = None):
        self.group = group
        self.tp = tp
        self.car = None
        if custom_ar is None:
            # on by default for TP > 1 on GPUs: a start-up self-test against the group's own
            # all-reduce gates it, and it is what lets the TP decode step run as one hipGraph
            custom_ar = os.environ.get("MLS_CUSTOM_AR", "1") == "1"
        if custom_ar and tp > 1 and device is not None and torch.device(device).type == "cuda":
            from ..parallel.custom_ar import CustomAllReduce

            car = CustomAllReduce(group, device)
            self.car = car if car.enabled else None
        # gloo with device tensors (TP rehearsal: several ranks sharing one GPU, where RCCL refuses
        # duplicate devices): stage the collectives through host memory
        self.host_staged = tp > 1 and dist.is_initialized() and dist.get_backend(group) == "gloo"

    def all_reduce_(self, t: torch.Tensor) -> torch.Tensor:
        if self.tp > 1:
            with tracing.range("tp.all_reduce"):
                return self._all_reduce(t)
        return t

    def _all_reduce(self, t: torch.Tensor) -> torch.Tensor:
        if self.car is not None and self.car.eligible(t):
            return self.car.all_reduce_(t)  # one-shot IPC path for small (decode) messages
        if self.host_staged and t.is_cuda:
            h = t.float().cpu()
            dist.all_reduce(h, group=self.group)
            t.copy_(h)
            return t
        dist.all_reduce(t, group=self.group)
        return t

    def all_reduce_start(self, t: torch.Tensor):
        """Start an in-place sum all-reduce and return a handle whose ``wait()`` yields ``t`` reduced.
        Large (prefill) messages go to the backend asynchronously so the caller can run independent
        work in between; the one-shot IPC path (an in-stream kernel) and host-staged gloo
        complete before returning."""
        if self.tp == 1:
            return _ARDone(t)
        with tracing.range("tp.all_reduce"):
            if (self.car is not None and self.car.eligible(t)) or (self.host_staged and t.is_cuda):
                return _ARDone(self._all_reduce(t))
            return _ARPending(t, dist.all_reduce(t, group=self.group, async_op=True))

    def all_gather(self, t: torch.Tensor) -> torch.Tensor:
        if self.tp == 1:
            return t.unsqueeze(0)
        with tracing.range("tp.all_gather"):
            return self._all_gather(t)

    def _all_gather(self, t: torch.Tensor) -> torch.Tensor:
        if self.host_staged and t.is_cuda:
            h = t.contiguous().cpu()
            out = [torch.empty_like(h) for _ in range(self.tp)]
            dist.all_gather(out, h, group=self.group)
            return torch.stack(out).to(t.device)
        out = [torch.empty_like(t) for _ in range(self.tp)]
        dist.all_gather(out, t.contiguous(), group=self.group)
        return torch.stack(out)

    def broadcast_(self, t: torch.Tensor, src: int = 0) -> torch.Tensor:
        if self.tp > 1:
            with tracing.range("tp.broadcast"):
                return self._broadcast(t, src)
        return t

    def _broadcast(self, t: torch.Tensor, src: int) -> torch.Tensor:
        if self.host_staged and t.is_cuda:
            h = t.cpu()
            dist.broadcast(h, src=src, group=self.group)
            t.copy_(h)
            return t
        dist.broadcast(t, src=src, group=self.group)
        return t


class ShardEmulationComm:
    """One TP rank's shard with every collective replaced by a local no-op -- a measurement tool:
    it times exactly the per-rank kernel work of a TP=tp decode / prefill step on one GPU (the
    all-reduce / all-gather cost is measured separately).  Outputs are not the model's."""

    graph_safe = True
    host_staged = False
    car = None

    def __init__(self, tp: int):
        self.tp = tp
        self.group = None

    def all_reduce_(self, t: torch.Tensor) -> torch.Tensor:
        return t

    def all_reduce_start(self, t: torch.Tensor):
        return _ARDone(t)

    def all_gather(self, t: torch.Tensor) -> torch.Tensor:
        return t.unsqueeze(0).expand(self.tp, *t.shape)

    def broadcast_(self, t: torch.Tensor, src: int = 0) -> torch.Tensor:
        return t


@dataclass
class GenParams:
    max_new_tokens: int = 16
    top_k: int = 1  # 1 = greedy
    temperature: float = 1.0
    seed: int = 0


_M64 = (1 << 64) - 1


def _splitmix64(x: int) -> int:
    x = (x + 0x9E3779B97F4A7C15) & _M64
    x = ((x ^ (x >> 30)) * 0xBF58476D1CE4E5B9) & _M64
    x = ((x ^ (x >> 27)) * 0x94D049BB133111EB) & _M64
    return x ^ (x >> 31)


def sample_uniform(seed: int, step: int) -> float:
    """The sampling draw for (request seed, decode step): a counter-based hash, bit-identical to
    the device pick kernel (ops/csrc/decode_pick.hip), independent of the row's batch position."""
    h = _splitmix64(((int(seed) & _M64) * 0x9E3779B97F4A7C15 + int(step)) & _M64)
    return float(h >> 40) / 16777216.0


class TPCommError(RuntimeError):
    """A tensor-parallel collective lost a peer (one-shot all-reduce / all-gather timed out): the
    tokens of the affected generation are not trustworthy and the request fails."""


class LlamaTP:
    """One rank of a tensor-parallel Llama with a KV cache ``[layers][max_batch, max_seq, hkv, D]``
    (or, paged, ``[layers][pages, 64, hkv, D]`` pools addressed through a page table)."""

    def __init__(self, params: Dict[str, torch.Tensor], cfg: LlamaConfig, tp: int = 1, rank: int = 0,
                 comm: Optional[TPComm] = None, backend: str = "reference", device="cpu", max_batch: int = 8,
                 max_seq: int = 1024, top_k_max: int = 50, kv_pages: int = 0):
        """``kv_pages > 0``: paged KV cache -- per layer a pool of ``kv_pages`` pages of 64 rows
        shared by all sequences (:class:`~.kv_pages.PageTable`), instead of ``max_batch x max_seq``."""
        self.cfg = cfg
        self.sd = shard_dims(cfg, tp, rank)
        self.tp, self.rank = tp, rank
        self.comm = comm or TPComm(None, tp)
        # TP prefill: two batch halves interleaved so each o / down all-reduce overlaps the other
        # half's compute (_prefill_overlapped); MLS_TP_OVERLAP=0 runs the plain layer loop
        self.tp_overlap = os.environ.get("MLS_TP_OVERLAP", "1") == "1"
        self.backend = backend
        self.device = torch.device(device)
        self.max_batch, self.max_seq = max_batch, max_seq
        self.top_k_max = top_k_max
        D = cfg.head_dim
        self.p = {k: v.to(self.device) for k, v in params.items()}
        if backend == "fused":
            from .. import ops

            self.ops = ops
            # RMSNorm gains folded into the projections that consume the normalised activations
            for i in range(cfg.layers):
                gu = ops.interleave_gate_up(self.p.pop(f"l{i}.gate"), self.p.pop(f"l{i}.up"))
                mlp_g = self.p.pop(f"l{i}.mlp_norm")
                self.p[f"l{i}.gate_up"] = ops.fold_norm(gu, mlp_g)
                self.p[f"l{i}.qkv"] = ops.fold_norm(self.p[f"l{i}.qkv"], self.p.pop(f"l{i}.attn_norm"))
            self.p["lm_head"] = ops.fold_norm(self.p["lm_head"], self.p.pop("final_norm"))
            # Decode (<= 24 tokens per step) streams a second, granule-packed copy of every projection
            # (ops.pack_skinny: each wave reads contiguous 1 KiB granules, non-temporal): 3.4-4.5 ->
            # 4.6-6.2 TB/s on the Llama-3-8B shapes (profiles/r2_decode_packed_weight_probe.jsonl).
            # Costs one more copy of the weights in HBM (16 GB at 8B / TP = 1 of 288 GB);
            # MLS_PACKED_DECODE=0 turns it off, "auto" packs while the copy stays under 1/4 of the card.
            self.packed: Dict[str, torch.Tensor] = {}
            self.pk_variant = int(os.environ.get("MLS_PACKED_VARIANT", "9"))
            self.pk_fold = os.environ.get("MLS_PACKED_FOLD", "1") == "1"
            # prefill at TP = 1 with the residual add in the o / down GEMM epilogues too (the
            # following RMSNorm then reads one stream and writes one: 64 instead of 128 B per element)
            self.prefill_fold = os.environ.get("MLS_PREFILL_FOLD", "0") == "1"
            self.ar_fuse = os.environ.get("MLS_AR_FUSE", "1") == "1"  # GEMM-fused TP all-reduce (decode)
            self.ar_fused_calls = 0  # projections issued with the fused all-reduce (eager + captured)
            self.fuse_combine = os.environ.get("MLS_FUSE_COMBINE", "1") == "1"
            mode = os.environ.get("MLS_PACKED_DECODE", "auto")
            if self.device.type == "cuda" and mode != "0":
                names = [f"l{i}.{n}" for i in range(cfg.layers) for n in ("qkv", "o", "gate_up", "down")]
                names.append("lm_head")
                names = [n for n in names if self.p[n].shape[0] % 16 == 0 and self.p[n].shape[1] % 32 == 0
                         and self.p[n].numel() * 2 < (1 << 31)]
                total = sum(self.p[n].numel() * 2 for n in names)
                cap = torch.cuda.get_device_properties(self.device).total_memory
                if mode == "1" or total <= cap // 4:
                    self.packed = {n: ops.pack_skinny(self.p[n]) for n in names}
            # Opt-in FP8 decode (MLS_DECODE_FP8=1): W8A8 e4m3 copies of the projections, per-channel
            # weight scales and per-row activation scales (ops.skinny_fp8), for <= 4 tokens per step --
            # half the weight stream (profiles/r2_decode_fp8_weight_probe.jsonl).  Changes numerics
            # (e4m3 has a 3-bit mantissa), so bf16 stays the default.
            self.fp8: Dict[str, Tuple[torch.Tensor, torch.Tensor]] = {}
            if self.device.type == "cuda" and os.environ.get("MLS_DECODE_FP8", "0") == "1":
                names = [f"l{i}.{n}" for i in range(cfg.layers) for n in ("qkv", "o", "gate_up", "down")]
                names.append("lm_head")
                # only matrices of >= 16M weights: below that a decode GEMM is latency-bound and the
                # fp8 prologue (row |max| reduction + requantisation) costs more than the bytes saved
                # -- one emulated TP = 8 rank was 1.13 -> 1.18 ms/token with every projection in fp8
                min_el = int(os.environ.get("MLS_DECODE_FP8_MIN", str(1 << 24)))
                self.fp8 = {n: ops.pack_skinny_fp8(self.p[n]) for n in names
                            if self.p[n].shape[0] % 16 == 0 and self.p[n].shape[1] % 64 == 0
                            and min_el <= self.p[n].numel() < (1 << 31)}
            self.ones = torch.ones(cfg.hidden, device=self.device, dtype=torch.bfloat16)
            self.workspace = torch.empty(32 << 20, device=self.device, dtype=torch.float32)
            self.dec_chunk = int(os.environ.get("MLS_DEC_CHUNK", "0"))  # 0: auto (see _fused_forward)
            self.dec_ws = torch.empty(max_batch * self.sd.hq * (-(-max_seq // 64)) * (D + 2) + 16,
                                      device=self.device, dtype=torch.float32)
            self.dec_cnt = torch.zeros(max_batch * self.sd.hkv, device=self.device, dtype=torch.int32)
        cdt = torch.bfloat16 if backend == "fused" else torch.float32
        # fused: head-major caches ([.., Hkv, rows, D]) -- one head's rows contiguous, so a decode split
        # block streams one 16 KiB run instead of 64 slices of 256 B (MLS_KV_HEAD_MAJOR=0: row-major)
        self.kv_hm = backend == "fused" and os.environ.get("MLS_KV_HEAD_MAJOR", "1") == "1"
        self.pages = None
        if kv_pages > 0:
            from .kv_pages import PageTable

            self.page_rows = 64  # = the decode split: one page per split block
            self.pages = PageTable(kv_pages, self.page_rows, max_batch, -(-max_seq // self.page_rows), self.device)
            shape = ((kv_pages, self.sd.hkv, self.page_rows, D) if self.kv_hm
                     else (kv_pages, self.page_rows, self.sd.hkv, D))
        else:
            shape = (max_batch, self.sd.hkv, max_seq, D) if self.kv_hm else (max_batch, max_seq, self.sd.hkv, D)
        self.kv_hm_rows = 0 if not self.kv_hm else (self.page_rows if kv_pages > 0 else max_seq)
        self.k_cache = [torch.zeros(shape, device=self.device, dtype=cdt) for _ in range(cfg.layers)]
        self.v_cache = [torch.zeros_like(self.k_cache[0]) for _ in range(cfg.layers)]
        self.cos, self.sin = R.rope_tables(max_seq, D, cfg.rope_theta, self.device)
        # hipGraph capture of the decode step (P4): removes ~300 host launches per token.  With
        # tp > 1 the step's collectives are captured too: the one-shot IPC all-reduce is graph-safe
        # (device-side epochs), so with it enabled every decode batch whose messages it takes is
        # captured (see _graph_ok); RCCL collectives inside the graph are opt-in (MLS_TP_GRAPHS=1).
        self._rccl_graphs = (os.environ.get("MLS_TP_GRAPHS", "0") == "1"
                             and not getattr(self.comm, "host_staged", False))
        self.use_graphs = backend == "fused" and self.device.type == "cuda" and (
            tp == 1 or getattr(self.comm, "graph_safe", False) or self._rccl_graphs
            or getattr(self.comm, "car", None) is not None)
        self._graphs: Dict[Tuple[int, int, int], tuple] = {}
        self._dec_ctx: Optional[int] = None  # host bound on decode context (sizes the split grid)
        # device-resident decode loop (X4 on device, _generate_device): per-batch-size static state
        # shared by the captured steps of every context bucket, so switching buckets copies nothing
        self._dev_graphs: Dict[Tuple[int, int, int], torch.cuda.CUDAGraph] = {}
        self._dev_state: Dict[int, Tuple[torch.Tensor, ...]] = {}
        self._serve: Dict[int, Dict[str, torch.Tensor]] = {}
        self.keep_logits = False
        self.last_logits: Optional[torch.Tensor] = None
        self.health_every = int(os.environ.get("MLS_TP_HEALTH_EVERY", "32"))

    # ---------------------------------------------------------------- shared pieces
    @property
    def qkv_width(self) -> int:
        return (self.sd.hq + 2 * self.sd.hkv) * self.cfg.head_dim

    def _embed(self, ids: torch.Tensor) -> torch.Tensor:
        sd = self.sd
        if self.backend == "fused":
            x = self.ops.embedding(ids, self.p["embed"], lo=sd.vocab_lo, hi=sd.vocab_lo + sd.vocab_shard)
        else:
            local = ids.long() - sd.vocab_lo
            ok = (local >= 0) & (local < sd.vocab_shard)
            x = self.p["embed"][local.clamp(0, sd.vocab_shard - 1)].float() * ok.unsqueeze(-1)
        return self.comm.all_reduce_(x)

    def _local_topk(self, logits: torch.Tensor, k: int):
        if self.keep_logits:  # tests: the full (shard-local) last-token logits of the latest step
            self.last_logits = logits
        if self.backend == "fused":  # shard offset + padded-tail mask inside the merge launch
            return self.ops.topk_large(logits, k, lo=self.sd.vocab_lo, valid=self.cfg.vocab - self.sd.vocab_lo)
        else:
            vals, idx = torch.topk(logits.float(), k, dim=-1)
            idx = idx.to(torch.int32)
        # mask rows of the padded vocab tail
        idx = idx + self.sd.vocab_lo
        vals = torch.where(idx < self.cfg.vocab, vals, torch.full_like(vals, float("-inf")))
        return vals, idx

    def _merge_sample(self, vals: torch.Tensor, idx: torch.Tensor, gp: GenParams, step: int) -> torch.Tensor:
        """X4: all-gather the ranks' top-k candidates, merge, pick the next token (identical on
        every rank: same inputs, same counter-based draw -> no broadcast needed)."""
        cv, ci = self.gather_candidates(vals, idx)
        return torch.tensor([self.pick_token(cv[b], ci[b], gp, step) for b in range(cv.shape[0])],
                            dtype=torch.int32, device=vals.device)

    # ---------------------------------------------------------------- reference backend
    def _ref_layer(self, i: int, x: torch.Tensor, B: int, S: int, positions: torch.Tensor, lens: torch.Tensor,
                   slots_b: torch.Tensor, decode: bool) -> torch.Tensor:
        cfg, sd, p = self.cfg, self.sd, self.p
        D = cfg.head_dim
        xn = R.layernorm(x, p[f"l{i}.attn_norm"], None, eps=cfg.eps, rms=True)[0]
        qkv = xn @ p[f"l{i}.qkv"].float().T
        T = qkv.shape[0]
        q = R.rope(qkv[:, : sd.hq * D].view(T, sd.hq, D), positions, self.cos, self.sin)
        k = R.rope(qkv[:, sd.hq * D: (sd.hq + sd.hkv) * D].view(T, sd.hkv, D), positions, self.cos, self.sin)
        v = qkv[:, (sd.hq + sd.hkv) * D:].view(T, sd.hkv, D)
        b_of = torch.arange(B, device=x.device).repeat_interleave(T // B)
        valid = positions < self.max_seq
        if not decode:
            valid = valid & (positions < lens.long()[b_of])
        rows = b_of if slots_b is None else slots_b.long()[b_of]  # batch row -> cache row
        bi, pi = rows[valid], positions[valid].long()
        if self.pages is not None:  # paged: flat pool rows through the page table
            flat = self.pages.rows(bi, pi)
            self.k_cache[i].view(-1, sd.hkv, D)[flat] = k[valid].to(self.k_cache[i].dtype)
            self.v_cache[i].view(-1, sd.hkv, D)[flat] = v[valid].to(self.v_cache[i].dtype)
        else:
            self.k_cache[i][bi, pi] = k[valid].to(self.k_cache[i].dtype)
            self.v_cache[i][bi, pi] = v[valid].to(self.v_cache[i].dtype)
        if decode:
            qrow = q.reshape(B, sd.hq * D)
            if self.pages is not None:  # gather each sequence's pages back into [B, rows, hkv, D]
                table = self.pages.device_table()[:B].long()
                kv = [c[table].reshape(B, -1, sd.hkv, D) for c in (self.k_cache[i], self.v_cache[i])]
                a = R.decode_attention(qrow, kv[0], kv[1], lens, sd.hq, sd.hkv, D)
            else:
                a = R.decode_attention(qrow, self.k_cache[i][:B], self.v_cache[i][:B], lens, sd.hq, sd.hkv, D)
        else:
            qkv_r = torch.cat([q.reshape(T, -1), k.reshape(T, -1), v.reshape(T, -1)], dim=1)
            a = R.attention(qkv_r, B, S, sd.hq, sd.hkv, D, kv_lens=lens, causal=True)
        o = self.comm.all_reduce_(a @ p[f"l{i}.o"].float().T)
        x = x + o
        xn = R.layernorm(x, p[f"l{i}.mlp_norm"], None, eps=cfg.eps, rms=True)[0]
        h = F.silu(xn @ p[f"l{i}.gate"].float().T) * (xn @ p[f"l{i}.up"].float().T)
        d = self.comm.all_reduce_(h @ p[f"l{i}.down"].float().T)
        return x + d

    def _ref_forward(self, ids: torch.Tensor, positions: torch.Tensor, lens: torch.Tensor, B: int, S: int,
                     decode: bool, k: int, slot_ids: Optional[torch.Tensor] = None):
        x = self._embed(ids.reshape(-1))
        for i in range(self.cfg.layers):
            x = self._ref_layer(i, x, B, S, positions.reshape(-1), lens, slot_ids, decode)
        xn = R.layernorm(x, self.p["final_norm"], None, eps=self.cfg.eps, rms=True)[0]
        if not decode:
            last = (torch.arange(B, device=x.device) * S + lens.long() - 1)
            xn = xn[last]
        logits = xn @ self.p["lm_head"].float().T
        return self._local_topk(logits, k)

    # ---------------------------------------------------------------- fused backend
    def _fused_forward(self, ids: torch.Tensor, positions: torch.Tensor, lens: torch.Tensor, B: int, S: int,
                       decode: bool, k: int, slot_ids: Optional[torch.Tensor] = None):
        """Native-kernel forward.  The RMSNorm gains are folded into the following projections, so
        for decode-shaped token counts (<= 16) each pre-norm + residual add rides inside the skinny
        GEMM (``ops.gemm_rmsnorm``: 7 launches per layer); larger counts run a gain-free RMSNorm and
        the library / native GEMM (``ops.linear``)."""
        ops, cfg, sd, p = self.ops, self.cfg, self.sd, self.p
        D, eps = cfg.head_dim, cfg.eps
        ws = self.workspace
        fuse = B * S <= 16
        pos = positions.reshape(-1)
        explicit_slots = None
        if (slot_ids is not None or self.pages is not None) and not decode:
            # prefill into arbitrary cache rows (continuous batching) / through the page table: one
            # native launch (ops.prefill_slots), -1 past each sequence's length
            sid = None if slot_ids is None else slot_ids.to(torch.int32)
            if self.pages is not None:
                explicit_slots = ops.prefill_slots(pos, lens, B, S, sid, table=self.pages.device_table(),
                                                   page_rows=self.pages.page_rows)
            else:
                explicit_slots = ops.prefill_slots(pos, lens, B, S, sid, max_seq=self.max_seq)
        # decode split size: 64 rows measured best from batch 1 to 32, at TP = 1 and on an emulated
        # TP = 8 rank (one KV head).  A single 256-row split per KV head (no combine launch) was
        # 1.6 % slower at batch 1, and one 8-wave block walking a whole <= 1024 context in passes
        # was 26 % slower at TP = 8 (latency-bound on one CU) -- profiles/r1_llama_decode_sweep.jsonl.
        # From batch 32 up the grid is already >= 4k blocks and 128-row splits halve the combine
        # traffic: -3 % step time at batch 128 (profiles/r2_llama8b_decode_chunk_sweep.jsonl).
        dec_chunk = self.dec_chunk if self.dec_chunk > 0 else (128 if B >= 32 else 64)
        r = self._embed(ids.reshape(-1))  # residual stream (bf16)
        delta = None

        T = B * S
        # packed decode GEMMs up to 24 rows: at 25-32 (two 16-row A fragments per weight granule)
        # every column-tile block re-reads A, and the row-major split-K kernel is ahead (batch 24:
        # 4.99 vs 5.36 ms/step, batch 32: 5.75 vs 5.64; profiles/r2_llama8b_decode_packed_ab.jsonl)
        packed = self.packed if T <= 24 else {}

        # TP = 1: the residual add rides in the o / down epilogues (h = r + a Wo^T, r' = h + g Wd^T), so
        # the next pre-norm GEMM reads one activation stream instead of two (r + delta) and writes no
        # residual copy.  With TP > 1 the add has to wait for the all-reduce.
        fold = self.tp == 1 and ((bool(packed) and self.pk_fold) or (not decode and getattr(self, "prefill_fold", False)))
        # decode: the o-projection merges the split-KV partials in its prologue (one launch instead of
        # two) while every block's share of partials is small -- B x local q heads <= 32: one emulated
        # TP = 8 rank 1.166 -> 1.125 ms/token at batch 1, 1.294 -> 1.254 at 4; TP = 1 batch 1 level,
        # batch 4 (128 head rows per block) 3.17 -> 3.37, so off there (profiles/r2_llama8b_fused_combine_ab.jsonl)
        fuse_combine = (decode and self.fuse_combine and "l0.o" in packed and "l0.o" not in self.fp8 and B <= 4
                        and B * sd.hq <= 32 and B * sd.hq * D * 2 <= 65536)

        fp8 = self.fp8 if T <= 4 else {}

        def use_fp8(name, K):
            return name in fp8 and T * K * 2 <= 65536

        # TP > 1 decode: the row-parallel o / down projections run their all-reduce in their own
        # epilogue (ops.skinny_packed_ar / skinny_packed_combine_ar, csrc/ar_protocol.h): one launch
        # per projection + all-reduce instead of two, and each 2048-element chunk of the output is
        # reduced as soon as the blocks producing it finish.  MLS_AR_FUSE=0: separate kernels.
        car = getattr(self.comm, "car", None)
        ar_fuse = (self.tp > 1 and car is not None and getattr(self, "ar_fuse", False) and bool(packed)
                   and car.fusable(T * self.cfg.hidden))

        def row_parallel(x, name):
            """sum over the TP ranks of x @ W_name^T (W row-parallel: each rank holds a K slice)."""
            if ar_fuse and name in packed and not use_fp8(name, x.shape[1]):
                self.ar_fused_calls += 1
                with tracing.range("tp.gemm_all_reduce"):
                    return ops.skinny_packed_ar(x, packed[name], p[name].shape[0], car, variant=self.pk_variant)
            return self.comm.all_reduce_(linear(x, name))

        def linear(x, name, residual=None):
            if use_fp8(name, x.shape[1]):
                q, sc = fp8[name]
                return ops.skinny_fp8(x, q, sc, p[name].shape[0], residual=residual)
            if name in packed:
                return ops.skinny_packed(x, packed[name], p[name].shape[0], residual=residual, variant=self.pk_variant)
            return ops.linear(x, p[name], residual=residual, workspace=ws)

        # TP = 1 above 24 tokens (no packed / fused-norm GEMMs): o_proj and down_proj leave their split-K
        # slabs to one kernel that adds them to the residual stream and normalises it for the next
        # projection (ops.linear_add_rmsnorm) -- one launch instead of reduce + RMSNorm, bit-identical.
        # A projection it cannot take (no split on that shape) runs the plain pair.
        fuse_rn = self.tp == 1 and not packed and not fuse and not fold and getattr(self, "fuse_add_norm", True)
        xn_pending = [None]  # RMSNorm(r) computed by the previous projection's fused reduce

        def proj_add_norm(x, name):
            """r += x @ W_name^T in place, and RMSNorm(r) staged for the next pre_norm; False: not taken."""
            xn = ops.linear_add_rmsnorm(x, p[name], r, self.ones, eps, ws) if fuse_rn else None
            xn_pending[0] = xn
            if xn is not None:
                self.add_norm_fused = getattr(self, "add_norm_fused", 0) + 1
            return xn is not None

        def pre_norm(x, name, d, act=ops.ACT_NONE):
            w = p[name]
            if xn_pending[0] is not None:
                xn, xn_pending[0] = xn_pending[0], None
                return ops.linear(xn, w, act=act, workspace=ws), x
            if use_fp8(name, x.shape[1]):
                q, sc = fp8[name]
                r_new = None if d is None else torch.empty_like(x)
                y = ops.skinny_fp8(x, q, sc, w.shape[0], delta=d, resid_out=r_new, norm=True, act=act, eps=eps)
                return y, (x if d is None else r_new)
            if name in packed:
                r_new = None if d is None else torch.empty_like(x)
                y = ops.skinny_packed(x, packed[name], w.shape[0], delta=d, resid_out=r_new, norm=True, act=act,
                                      eps=eps, variant=self.pk_variant)
                return y, (x if d is None else r_new)
            if fuse:
                r_new = None if d is None else torch.empty_like(x)
                y = ops.gemm_rmsnorm(x, w, d, r_new, act=act, eps=eps, workspace=ws)
                return y, (x if d is None else r_new)
            xn = ops.rmsnorm(x if d is None else d, self.ones, residual=None if d is None else x,
                             residual_out=None if d is None else x, eps=eps)
            return ops.linear(xn, w, act=act, workspace=ws), x

        overlap = (not decode and self.tp > 1 and B >= 2 and T >= 64 and self.tp_overlap
                   and not torch.cuda.is_current_stream_capturing())
        if overlap:
            r, delta = self._prefill_overlapped(r, pos, lens, B, S, explicit_slots, pre_norm, linear)
        for i in range(0 if not overlap else cfg.layers, cfg.layers):
            qkv, r = pre_norm(r, f"l{i}.qkv", delta)
            parts = None
            if decode:  # RoPE + KV append ride inside the decode-attention launch
                kw = dict(workspace=self.dec_ws, counters=self.dec_cnt, positions=pos, cos=self.cos, sin=self.sin,
                          max_len=self._dec_ctx, combine=not fuse_combine, head_major=self.kv_hm)
                if self.pages is not None:
                    a = ops.decode_attention(qkv, self.k_cache[i], self.v_cache[i], lens, sd.hq, sd.hkv, D,
                                             chunk=self.page_rows, page_table=self.pages.dev[:B], **kw)
                else:
                    a = ops.decode_attention(qkv, self.k_cache[i][:B], self.v_cache[i][:B], lens, sd.hq, sd.hkv,
                                             D, chunk=dec_chunk, **kw)
                if fuse_combine:
                    a, parts = a
            else:
                ops.rope_kv_(qkv, pos, self.cos, self.sin, sd.hq, sd.hkv, D, explicit_slots, self.k_cache[i],
                             self.v_cache[i], lens=lens, seq=S, max_seq=self.max_seq, hm_rows=self.kv_hm_rows)
                a = ops.flash_attention(qkv, B, S, sd.hq, sd.hkv, D, kv_lens=lens, causal=True)
            if parts is not None:  # split-KV combine in the o-projection's prologue (one launch, not two)
                o_w = p[f"l{i}.o"]
                if ar_fuse:  # ... and the all-reduce in its epilogue
                    self.ar_fused_calls += 1
                    with tracing.range("tp.gemm_all_reduce"):
                        o = ops.skinny_packed_combine_ar(a, parts, packed[f"l{i}.o"], o_w.shape[0], car,
                                                         variant=self.pk_variant)
                else:
                    o = ops.skinny_packed_combine(a, parts, packed[f"l{i}.o"], o_w.shape[0],
                                                  residual=r if fold else None, variant=self.pk_variant)
                if fold:
                    gu, _ = pre_norm(o, f"l{i}.gate_up", None, act=ops.ACT_SILU_MUL)
                    r = linear(gu, f"l{i}.down", residual=o)
                    continue
                if not ar_fuse:
                    o = self.comm.all_reduce_(o)
                gu, r = pre_norm(r, f"l{i}.gate_up", o, act=ops.ACT_SILU_MUL)
                delta = row_parallel(gu, f"l{i}.down")
                continue
            if fold:
                h = linear(a, f"l{i}.o", residual=r)
                gu, _ = pre_norm(h, f"l{i}.gate_up", None, act=ops.ACT_SILU_MUL)
                r = linear(gu, f"l{i}.down", residual=h)
                continue
            if delta is None and proj_add_norm(a, f"l{i}.o"):
                gu, r = pre_norm(r, f"l{i}.gate_up", None, act=ops.ACT_SILU_MUL)
                if i + 1 < cfg.layers and proj_add_norm(gu, f"l{i}.down"):
                    continue  # delta stays None: the down output is in r, its RMSNorm staged for qkv
                delta = row_parallel(gu, f"l{i}.down")
                continue
            o = row_parallel(a, f"l{i}.o")
            gu, r = pre_norm(r, f"l{i}.gate_up", o, act=ops.ACT_SILU_MUL)
            delta = row_parallel(gu, f"l{i}.down")
        if not decode:  # each sequence's last valid token (one native gather of r and delta)
            if delta is None:
                r = ops.last_rows(r, lens, B, S)
            else:
                r, delta = ops.last_rows(r, lens, B, S, delta)
        if B <= 4 and "lm_head" in self.fp8 and B * r.shape[1] * 2 <= 65536:
            q, sc = self.fp8["lm_head"]
            logits = ops.skinny_fp8(r, q, sc, p["lm_head"].shape[0], delta=delta, norm=True, eps=eps)
        elif B <= 24 and "lm_head" in self.packed:
            logits = ops.skinny_packed(r, self.packed["lm_head"], p["lm_head"].shape[0], delta=delta, norm=True,
                                       eps=eps, variant=self.pk_variant)
        elif B <= 16:
            logits = ops.gemm_rmsnorm(r, p["lm_head"], delta, eps=eps, workspace=ws)
        else:  # 1 GB of weights: the weight-streaming native tile up to 64 rows, the tile GEMM above
            xn = ops.rmsnorm(delta, self.ones, residual=r, eps=eps)
            logits = ops.linear(xn, p["lm_head"], workspace=ws, impl="native" if B <= 64 else "auto")
        return self._local_topk(logits, k)

    def _prefill_overlapped(self, r, pos, lens, B: int, S: int, explicit_slots, pre_norm, linear):
        """TP prefill as two batch halves (micro-batches) interleaved layer by layer so that every
        o / down all-reduce runs while the other half computes:

            half 0: norm+QKV, RoPE/KV, attention, o -> start AR(o0)
            half 1: norm+QKV, RoPE/KV, attention, o -> start AR(o1)     [overlaps AR(o0)]
            half 0: wait AR(o0), norm+gate/up, down -> start AR(d0)     [overlaps AR(o1)]
            half 1: wait AR(o1), norm+gate/up, down -> start AR(d1)     [overlaps AR(d0)]
            next layer, half 0 waits AR(d0)                             [overlaps AR(d1)]

        The residual stream rows of each half are updated in place (views of ``r``); returns the
        full residual and the last layer's all-reduced delta."""
        ops, cfg, sd = self.ops, self.cfg, self.sd
        D = cfg.head_dim
        half = B // 2
        # plain cache: each half runs rope_kv_'s implicit slot mode (token t -> row (t // S) * max_seq
        # + pos) on a view of the caches starting at its first batch row -- no torch-side slot map
        # (the head-major layout groups hm_rows slots, so the offset must be a whole group)
        implicit = explicit_slots is None and (not self.kv_hm_rows or (half * self.max_seq) % self.kv_hm_rows == 0)
        if explicit_slots is None and not implicit:
            explicit_slots = ops.prefill_slots(pos, lens, B, S, max_seq=self.max_seq)
        slot_elems = sd.hkv * D  # cache elements per slot in either layout
        parts = [(0, half), (half, B)]
        res = [r[b0 * S:b1 * S] for b0, b1 in parts]
        dlt = [None, None]
        pend_d = [None, None]
        for i in range(cfg.layers):
            pend_o = [None, None]
            for m, (b0, b1) in enumerate(parts):
                lo, hi = b0 * S, b1 * S
                if pend_d[m] is not None:
                    dlt[m] = pend_d[m].wait()
                qkv, res[m] = pre_norm(res[m], f"l{i}.qkv", dlt[m])
                if implicit:
                    off = b0 * self.max_seq * slot_elems
                    ops.rope_kv_(qkv, pos[lo:hi], self.cos, self.sin, sd.hq, sd.hkv, D, None,
                                 self.k_cache[i].reshape(-1)[off:], self.v_cache[i].reshape(-1)[off:],
                                 lens=lens[b0:b1], seq=S, max_seq=self.max_seq, hm_rows=self.kv_hm_rows)
                else:
                    ops.rope_kv_(qkv, pos[lo:hi], self.cos, self.sin, sd.hq, sd.hkv, D, explicit_slots[lo:hi],
                                 self.k_cache[i], self.v_cache[i], lens=lens[b0:b1], seq=S, max_seq=self.max_seq,
                                 hm_rows=self.kv_hm_rows)
                a = ops.flash_attention(qkv, b1 - b0, S, sd.hq, sd.hkv, D, kv_lens=lens[b0:b1], causal=True)
                pend_o[m] = self.comm.all_reduce_start(linear(a, f"l{i}.o"))
            for m in range(2):
                o = pend_o[m].wait()
                gu, res[m] = pre_norm(res[m], f"l{i}.gate_up", o, act=ops.ACT_SILU_MUL)
                pend_d[m] = self.comm.all_reduce_start(linear(gu, f"l{i}.down"))
        dlt = [p.wait() for p in pend_d]
        if any(x.data_ptr() != y.data_ptr() for x, y in zip(res, (r[:half * S], r[half * S:]))):
            r = torch.cat(res)  # pre_norm handed back new residual tensors instead of the views
        return r, torch.cat(dlt)

    # ---------------------------------------------------------------- public
    @torch.no_grad()
    def step(self, ids: torch.Tensor, positions: torch.Tensor, lens: torch.Tensor, decode: bool, k: int,
             slot_ids: Optional[torch.Tensor] = None):
        """One forward.  ``slot_ids`` (prefill only): cache row of each batch row (default: the
        batch row itself) -- how continuous batching prefills new requests into free slots."""
        B, S = ids.shape
        ids, positions, lens = ids.contiguous(), positions.contiguous(), lens.contiguous()
        if self.pages is not None and not (self.device.type == "cuda" and torch.cuda.is_current_stream_capturing()):
            self.pages.device_table()
        if slot_ids is not None:
            slot_ids = slot_ids.to(self.device).contiguous()
        with tracing.range("llama.decode" if decode else "llama.prefill"):
            if self.backend == "fused":
                return self._fused_forward(ids.to(torch.int32), positions.to(torch.int32), lens.to(torch.int32), B,
                                           S, decode, k, slot_ids)
            return self._ref_forward(ids, positions, lens, B, S, decode, k, slot_ids)

    def gather_candidates(self, vals: torch.Tensor, idx: torch.Tensor):
        """X4 all-gather of every rank's local top-k -> ``[B, tp*k]`` values / ids (host tensors)."""
        allv = self.comm.all_gather(vals)
        alli = self.comm.all_gather(idx)
        B = vals.shape[0]
        return (allv.permute(1, 0, 2).reshape(B, -1).float().cpu(), alli.permute(1, 0, 2).reshape(B, -1).cpu())

    @staticmethod
    def pick_token(cv: torch.Tensor, ci: torch.Tensor, gp: GenParams, step: int) -> int:
        """One row's next token from its merged candidates -- the rule of the device pick kernel
        (ops.decode_pick): greedy = the first maximum; sampled = the ``top_k`` largest (ties in
        candidate order), softmax at ``temperature`` in fp32, the first cumulative weight above
        ``sample_uniform(seed, step)`` of the total."""
        if gp.top_k <= 1:
            return int(ci[int(cv.argmax())])
        k = min(gp.top_k, cv.shape[0], 64)
        v = cv.float()
        order = torch.sort(v, descending=True, stable=True).indices[:k]
        tv = v[order]
        w = torch.exp((tv - tv[0]) / max(gp.temperature, 1e-5))
        cdf = torch.cumsum(w, 0)
        thr = torch.tensor(sample_uniform(gp.seed, step), dtype=torch.float32) * cdf[-1]
        hit = (cdf > thr).nonzero()
        pick = int(hit[0, 0]) if hit.numel() else k - 1
        return int(ci[int(order[pick])])

    def ctx_bucket(self, max_ctx: Optional[int]) -> int:
        """Power-of-two context bound (>= 256, <= max_seq) a decode graph is captured for."""
        if max_ctx is None:
            return self.max_seq
        return min(self.max_seq, max(256, 1 << (max(1, int(max_ctx)) - 1).bit_length()))

    def _graph_ok(self, B: int) -> bool:
        """May the decode step for batch B be captured?  Always at tp == 1 / under a graph-safe
        comm; with the IPC all-reduce only while its B x hidden bf16 messages fit the one-shot
        buffer (larger ones would fall back to an uncapturable collective) unless RCCL capture
        is enabled."""
        if self.tp == 1 or getattr(self.comm, "graph_safe", False) or self._rccl_graphs:
            return True
        car = getattr(self.comm, "car", None)
        if car is None:
            return False
        probe = torch.empty(B * self.cfg.hidden, dtype=torch.bfloat16, device=car.device)
        return car.eligible(probe)  # one-shot or two-shot: both are in-stream kernels

    def _decode_graph(self, B: int, k: int, ctx: int):
        """Captured decode step for batch B and context bound ctx (static token / position / length
        buffers).  The warm-up steps run at position ctx - 1: for a sequence being decoded under
        this bound that row is either the one the step about to replay writes anyway, or a future
        row that will be overwritten before anything reads it -- so graphs can be captured while
        sequences are in flight."""
        key = (B, k, ctx)
        if key in self._graphs:
            return self._graphs[key]
        dev = self.device
        tok = torch.zeros(B, 1, dtype=torch.int32, device=dev)
        pos = torch.full((B, 1), ctx - 1, dtype=torch.int32, device=dev)
        lens = torch.full((B,), ctx, dtype=torch.int32, device=dev)
        self._dec_ctx = ctx
        try:
            side = torch.cuda.Stream(dev)
            side.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(side):
                for _ in range(2):
                    self.step(tok, pos, lens, decode=True, k=k)
            torch.cuda.current_stream(dev).wait_stream(side)
            g = torch.cuda.CUDAGraph()
            # thread_local: the RCCL watchdog thread polls its events while this thread captures
            with torch.cuda.graph(g, capture_error_mode="thread_local"):
                vals, idx = self.step(tok, pos, lens, decode=True, k=k)
        finally:
            self._dec_ctx = None
        self._graphs[key] = (g, tok, pos, lens, vals, idx)
        return self._graphs[key]

    def decode_step(self, tok: torch.Tensor, cur: torch.Tensor, k: int, max_ctx: Optional[int] = None):
        """One decode step: token at position ``cur`` (attending to cur + 1 keys).  ``max_ctx``: a
        host-side bound on cur + 1 (e.g. prompt length + step), used to pick a tight split grid."""
        B = tok.shape[0]
        ctx = self.ctx_bucket(max_ctx)
        if self.use_graphs and self._graph_ok(B):
            g, t_s, p_s, l_s, v_s, i_s = self._decode_graph(B, k, ctx)
            if self.pages is not None:
                self.pages.device_table()  # the graph reads the table buffer in place
            t_s.copy_(tok.view(B, 1))
            p_s.copy_(cur.view(B, 1))
            l_s.copy_(cur.view(B) + 1)
            with tracing.range("llama.decode"):
                g.replay()
            return v_s, i_s
        self._dec_ctx = ctx
        try:
            return self.step(tok.view(B, 1).to(torch.int32), cur.view(B, 1), cur.view(B) + 1, decode=True, k=k)
        finally:
            self._dec_ctx = None

    @torch.no_grad()
    def generate(self, ids: torch.Tensor, lens: torch.Tensor, gp: GenParams) -> torch.Tensor:
        """ids int ``[B, S]`` (right-padded), lens ``[B]`` -> generated ``[B, max_new_tokens]``."""
        B, S = ids.shape
        if B > self.max_batch or S + gp.max_new_tokens > self.max_seq:
            raise ValueError("batch / sequence exceed the KV cache")
        lens_host = lens.detach().to("cpu")
        if lens_host.numel() != B or int(lens_host.min()) < 1 or int(lens_host.max()) > S:
            raise ValueError(f"lens must be in [1, {S}] for each of the {B} sequences")
        dev = self.device
        ids = ids.to(dev)
        lens = lens.to(dev).to(torch.int32)
        k = max(1, min(gp.top_k, self.top_k_max))
        if self._device_loop_ok(B, k):
            return self._generate_device(ids, lens, gp, k)
        assigned = 0
        try:
            if self.pages is not None:  # batch row b = slot b, pages for the prompt + the generation budget
                for b in range(B):
                    self.pages.assign(b, S + gp.max_new_tokens)
                    assigned = b + 1
            pos = torch.arange(S, device=dev, dtype=torch.int32).unsqueeze(0).expand(B, S).contiguous()
            vals, idx = self.step(ids, pos, lens, decode=False, k=k)
            out = []
            tok = self._sample_rows(vals, idx, gp, 0)
            out.append(tok)
            cur = lens.clone()
            for t in range(1, gp.max_new_tokens):
                # the new token sits at position cur; attention covers cur + 1 keys
                vals, idx = self.decode_step(tok.to(dev), cur, k, max_ctx=S + t)
                tok = self._sample_rows(vals, idx, gp, t)
                out.append(tok)
                cur = cur + 1
            return torch.stack(out, dim=1)
        finally:
            if self.pages is not None:  # also on OutOfPages part-way: release exactly the rows assigned
                for b in range(assigned):
                    self.pages.release(b)

    # ---------------------------------------------------------------- device-resident decode loop
    def _gather_pad(self, k: int) -> int:
        return (-2 * k) % 4  # [B, 2k + pad] fp32 rows: a 16-B multiple per row (one-shot all-gather)

    def _device_loop_ok(self, B: int, k: int) -> bool:
        """May generate() run the X4 merge + token pick inside the captured decode step?"""
        if os.environ.get("MLS_DEVICE_PICK", "1") == "0":
            return False
        if not (self.backend == "fused" and self.device.type == "cuda" and self.use_graphs and self._graph_ok(B)):
            return False
        if self.tp * k > 512 or k > 64:
            return False
        if self.tp == 1 or getattr(self.comm, "graph_safe", False):
            return True
        car = getattr(self.comm, "car", None)
        if car is not None:  # + the serving step's control row (serve_graph)
            return (B + 1) * (2 * k + self._gather_pad(k)) * 4 <= car.cap
        return self._rccl_graphs and not getattr(self.comm, "host_staged", False)

    def _gather_dev(self, vals: torch.Tensor, idx: torch.Tensor, ctl: Optional[torch.Tensor] = None):
        """X4 on device: every rank's [B, k] candidates -> ([tp, B, k] f32, [tp, B, k] i32), one
        collective (values and ids packed in one fp32 row); graph-capturable.  ``ctl`` (int32
        [CTL_WORDS], optional): one more row rides the same collective, and the call returns a third
        value, RANK 0's ctl words (int32 [CTL_WORDS]) -- the serving loop's next-iteration header
        (models/llama_serving.py), with no collective of its own."""
        if self.tp == 1:
            if ctl is not None:
                return vals.unsqueeze(0), idx.unsqueeze(0), ctl.clone()
            return vals.unsqueeze(0), idx.unsqueeze(0)
        B, k = vals.shape
        pad = self._gather_pad(k)
        parts = [vals.float(), idx.view(torch.float32)]
        if pad:
            parts.append(torch.zeros(B, pad, device=vals.device, dtype=torch.float32))
        pack = torch.cat(parts, dim=1)
        if ctl is not None:  # W = 2k + pad >= 4 >= CTL_WORDS fp32 columns
            W = pack.shape[1]
            row = torch.zeros(1, W, device=vals.device, dtype=torch.float32)
            row[0, : ctl.numel()] = ctl.view(torch.float32)
            pack = torch.cat([pack, row], dim=0)
        pack = pack.contiguous()
        car = getattr(self.comm, "car", None)
        if car is not None and car.gather_eligible(pack):
            with tracing.range("tp.all_gather"):
                g = car.all_gather(pack)
        elif getattr(self.comm, "graph_safe", False):
            g = self.comm.all_gather(pack)
        else:
            g = torch.empty((self.tp, *pack.shape), device=pack.device, dtype=pack.dtype)
            with tracing.range("tp.all_gather"):
                dist.all_gather_into_tensor(g, pack, group=self.comm.group)
        if ctl is not None:
            c0 = g[0, B, : ctl.numel()].contiguous().view(torch.int32)
            g = g[:, :B]
            return g[..., :k].contiguous(), g[..., k: 2 * k].contiguous().view(torch.int32), c0
        return g[..., :k].contiguous(), g[..., k: 2 * k].contiguous().view(torch.int32)

    def _dev_buffers(self, B: int):
        st = self._dev_state.get(B)
        if st is None:
            dev = self.device
            z = lambda dt: torch.zeros(B, device=dev, dtype=dt)  # noqa: E731
            st = (z(torch.int32), z(torch.int32), z(torch.int32), z(torch.int32),  # tok, pos, lens, step
                  z(torch.int32), torch.ones(B, device=dev, dtype=torch.float32), z(torch.int64),  # topk, temp, seed
                  torch.zeros(B, self.max_seq, device=dev, dtype=torch.int32))  # hist
            self._dev_state[B] = st
        return st

    def _decode_graph_dev(self, B: int, k: int, ctx: int) -> torch.cuda.CUDAGraph:
        """Captured decode step + X4 gather + on-device pick for batch B / context bound ctx: reads
        tok / pos / lens of the shared per-B state and advances them for the next replay."""
        key = (B, k, ctx)
        g = self._dev_graphs.get(key)
        if g is not None:
            return g
        dev = self.device
        tok, pos, lens, step, topk, temp, seed, hist = self._dev_buffers(B)
        # warm-up (kernel selection, workspaces) on scratch inputs at position ctx - 1: that cache row
        # is either the one a replay under this bound writes anyway or a future row rewritten before
        # it is read (see _decode_graph); the shared state is left alone
        t_w = torch.zeros(B, 1, dtype=torch.int32, device=dev)
        p_w = torch.full((B, 1), ctx - 1, dtype=torch.int32, device=dev)
        l_w = torch.full((B,), ctx, dtype=torch.int32, device=dev)
        self._dec_ctx = ctx
        try:
            side = torch.cuda.Stream(dev)
            side.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(side):
                for _ in range(2):
                    v, i = self.step(t_w, p_w, l_w, decode=True, k=k)
                    self._gather_dev(v, i)
            torch.cuda.current_stream(dev).wait_stream(side)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, capture_error_mode="thread_local"):
                v, i = self.step(tok.view(B, 1), pos.view(B, 1), lens, decode=True, k=k)
                cv, ci = self._gather_dev(v, i)
                self.ops.decode_pick(cv, ci, tok, pos, lens, step, topk=topk, temp=temp, seed=seed, hist=hist)
        finally:
            self._dec_ctx = None
        self._dev_graphs[key] = g
        return g

    # ---------------------------------------------------------------- serving (ContinuousLlama) on device
    def serve_state(self, B: int) -> Dict[str, torch.Tensor]:
        """Per-slot device state of the continuous-batching decode loop (models/llama_serving.py):
        ``E`` int32 [2, B] is the one per-iteration read-back -- row 0 the prefill picks of the
        iteration's new sequences, row 1 (= ``tok``, the decode graph's input and output token) the
        decode picks; ``active`` masks idle slots out of the pick (they decode a dummy token into
        their own cache row / the scratch page and keep pos 0).  ``E_all`` = ``E`` followed by
        ``ctl_out`` (int32 [CTL_WORDS]): rank 0's ``ctl_in`` as the decode step's gather carried it
        (the next iteration's header at TP > 1), and ``err_out`` (int32 [1]): this rank's one-shot
        collectives' sticky peer-timeout word after the step -- all read back in the same copy."""
        st = self._serve.get(B)
        if st is None:
            dev = self.device
            z = lambda dt: torch.zeros(B, device=dev, dtype=dt)  # noqa: E731
            E_all = torch.zeros(2 * B + CTL_WORDS + 1, device=dev, dtype=torch.int32)
            E = E_all[: 2 * B].view(2, B)
            st = {"E": E, "E_all": E_all, "ctl_out": E_all[2 * B: 2 * B + CTL_WORDS], "err_out": E_all[2 * B + CTL_WORDS:],
                  "ctl_in": torch.zeros(CTL_WORDS, device=dev, dtype=torch.int32),
                  "tok": E[1], "pos": z(torch.int32), "lens": torch.ones(B, device=dev, dtype=torch.int32),
                  "step": z(torch.int32), "topk": torch.ones(B, device=dev, dtype=torch.int32),
                  "temp": torch.ones(B, device=dev, dtype=torch.float32), "seed": z(torch.int64),
                  "active": z(torch.int32)}
            self._serve[B] = st
        return st

    def serve_graph(self, B: int, k: int, ctx: int) -> torch.cuda.CUDAGraph:
        """Captured serving decode step over all B slots: forward + X4 gather + the on-device pick
        of the ACTIVE slots (``ops.decode_pick(active=...)``), advancing their state in place."""
        key = ("serve", B, k, ctx)
        g = self._dev_graphs.get(key)
        if g is not None:
            return g
        dev = self.device
        st = self.serve_state(B)
        # warm-up on scratch inputs at position ctx - 1 (see _decode_graph): the shared state is not touched
        t_w = torch.zeros(B, 1, dtype=torch.int32, device=dev)
        p_w = torch.full((B, 1), ctx - 1, dtype=torch.int32, device=dev)
        l_w = torch.full((B,), ctx, dtype=torch.int32, device=dev)
        self._dec_ctx = ctx
        try:
            side = torch.cuda.Stream(dev)
            side.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(side):
                for _ in range(2):
                    v, i = self.step(t_w, p_w, l_w, decode=True, k=k)
                    self._gather_dev(v, i)
            torch.cuda.current_stream(dev).wait_stream(side)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, capture_error_mode="thread_local"):
                v, i = self.step(st["tok"].view(B, 1), st["pos"].view(B, 1), st["lens"], decode=True, k=k)
                cv, ci, c0 = self._gather_dev(v, i, ctl=st["ctl_in"])
                st["ctl_out"].copy_(c0)
                car = getattr(self.comm, "car", None)
                if car is not None:  # did a peer wait of this step (or an earlier one) time out?
                    car.error_peek(st["err_out"])
                self.ops.decode_pick(cv, ci, st["tok"], st["pos"], st["lens"], st["step"], topk=st["topk"],
                                     temp=st["temp"], seed=st["seed"], active=st["active"])
        finally:
            self._dec_ctx = None
        self._dev_graphs[key] = g
        return g

    def check_comm_health(self) -> None:
        """Collective (same decode step on every rank): did any one-shot collective lose a peer
        since the last check?  On an error every rank resets the device protocol, drops the IPC
        path (RCCL from now on) and its captured steps, and raises :class:`TPCommError`."""
        car = getattr(self.comm, "car", None)
        if self.tp == 1 or car is None:
            return
        err = car.errors()
        backend = dist.get_backend(self.comm.group)
        flag = torch.tensor([err], dtype=torch.int32, device=self.device if backend == "nccl" else "cpu")
        dist.all_reduce(flag, op=dist.ReduceOp.MAX, group=self.comm.group)
        if int(flag.item()):
            car.reset()
            self.comm.car = None
            self._graphs.clear()
            self._dev_graphs.clear()
            raise TPCommError("a tensor-parallel peer missed a one-shot collective; falling back to RCCL")

    def _generate_device(self, ids: torch.Tensor, lens: torch.Tensor, gp: GenParams, k: int) -> torch.Tensor:
        """generate() with every decode step a graph replay that also merges the ranks' candidates
        and picks the next token on device (X4 + P4): no host round trip until the end (and the
        comm-health check every ``health_every`` steps)."""
        B, S = ids.shape
        dev = self.device
        tok, pos, lens_s, step, topk, temp, seed, hist = self._dev_buffers(B)
        step.zero_()
        topk.fill_(int(gp.top_k))
        temp.fill_(float(gp.temperature))
        seed.fill_(int(gp.seed))
        assigned = 0
        try:
            if self.pages is not None:
                for b in range(B):
                    self.pages.assign(b, S + gp.max_new_tokens)
                    assigned = b + 1
            posp = torch.arange(S, device=dev, dtype=torch.int32).unsqueeze(0).expand(B, S).contiguous()
            vals, idx = self.step(ids, posp, lens, decode=False, k=k)
            cv, ci = self._gather_dev(vals, idx)
            pos.copy_(lens - 1)  # the pick advances them to (lens, lens + 1): the first decode position
            lens_s.copy_(lens)
            self.ops.decode_pick(cv, ci, tok, pos, lens_s, step, topk=topk, temp=temp, seed=seed, hist=hist)
            for t in range(1, gp.max_new_tokens):
                g = self._decode_graph_dev(B, k, self.ctx_bucket(S + t))
                if self.pages is not None:
                    self.pages.device_table()  # the graph reads the table buffer in place
                with tracing.range("llama.decode"):
                    g.replay()
                if self.health_every > 0 and t % self.health_every == 0:
                    self.check_comm_health()
            self.check_comm_health()
            return hist[:, : gp.max_new_tokens].cpu()
        finally:
            if self.pages is not None:
                for b in range(assigned):
                    self.pages.release(b)

    def _sample_rows(self, vals, idx, gp: GenParams, step: int) -> torch.Tensor:
        cv, ci = self.gather_candidates(vals, idx)
        return torch.tensor([self.pick_token(cv[b], ci[b], gp, step) for b in range(cv.shape[0])],
                            dtype=torch.int32)
