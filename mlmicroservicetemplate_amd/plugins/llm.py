"""``llama`` plugin: ``POST /generate`` on Llama-3-8B, tensor-parallel over the node (config 5).

Request: ``{"prompt": str | "input_ids": [int], "max_new_tokens": int, "top_k": int,
"temperature": float, "seed": int}``.  With ``CONTINUOUS_BATCHING`` (default) requests join and
leave the running decode batch at every step (``models/llama_serving.py``); otherwise
concurrent requests are micro-batched (same batcher as ``/predict``), right-padded and generated
together (batched prefill with per-sequence lengths, then lockstep decode steps).

Multi-GPU: rank 0 owns HTTP.  For each batch it broadcasts a small command header and the
token ids to the other ranks (X5); every rank then runs the same TP forward, and the
top-k candidate merge makes the sampled token identical on all ranks, so no per-token
broadcast is needed.  Followers sit in :meth:`follower_loop` until rank 0 sends STOP.
"""
from __future__ import annotations

import logging
import threading
from typing import Any, Dict, List, Tuple

import torch

from ..models.llama_serving import OP_GENERATE, OP_ITER, OP_STOP
from .base import ModelPlugin, PluginContext, register

logger = logging.getLogger("mlsamd.plugin")


@register("llama")
class LlamaPlugin(ModelPlugin):
    name = "llama"
    batched = True
    task = "generate"

    def __init__(self):
        self.model = None
        self.tok = None
        self.ctx = None
        self.comm_dev = None
        self._lock = threading.Lock()

    def init(self, ctx: PluginContext) -> None:
        from ..models import llama

        self.ctx = ctx
        s = ctx.settings
        extra = s.model_yaml() if hasattr(s, "model_yaml") else {}
        size = extra.get("config", "8b")
        cfg = llama.LLAMA3_8B if size == "8b" else llama.tiny_config(**extra.get("overrides", {}))
        tp = ctx.world_size if int(s.TP) > 1 else 1
        if tp > 1 and ctx.world_size != tp:
            raise RuntimeError(f"TP={s.TP} needs WORLD_SIZE={tp}")
        on_gpu = torch.cuda.is_available() and bool(ctx.devices)
        dev = ctx.devices[0] if on_gpu else "cpu"
        backend = s.BACKEND if (on_gpu and s.BACKEND == "fused") else "reference"
        self.comm_dev = torch.device(dev)
        # every TP rank reads just its own slices from the checkpoint (no weight broadcast needed)
        source = llama.CheckpointSource(s.WEIGHTS, device=dev) if s.WEIGHTS else None
        params = llama.init_llama_shard(cfg, tp, ctx.rank, int(s.SEED), device=dev, source=source)
        max_batch, max_seq = int(s.MAX_BATCH) or 32, int(extra.get("max_seq", 2048))
        kv_pages = self._kv_pages(extra.get("kv_pages", 0), cfg, tp, max_batch, max_seq, dev, backend)
        if tp > 1 and kv_pages:  # the scheduler replays rank 0's admissions: every pool must be equal
            from ..parallel import dist as mdist

            kv_pages = int(-mdist.max_over_ranks(-float(kv_pages)))
        self.model = llama.LlamaTP(params, cfg, tp=tp, rank=ctx.rank, comm=llama.TPComm(None, tp, device=dev), backend=backend,
                                   device=dev, max_batch=max_batch, max_seq=max_seq, kv_pages=kv_pages)
        self.tok = llama.LlamaTokenizer(cfg, extra.get("tokenizer_file"))
        self.cfg = cfg
        self.engine = None
        if bool(getattr(s, "CONTINUOUS_BATCHING", True)):
            from ..models.llama_serving import ContinuousLlama

            self.engine = ContinuousLlama(self.model, max_queue=int(s.MAX_QUEUE), channel=self if tp > 1 else None)
            if ctx.rank == 0:
                self.engine.start()
        logger.info("llama ready: tp=%d rank=%d backend=%s device=%s", tp, ctx.rank, backend, dev)

    @staticmethod
    def _kv_pages(spec, cfg, tp, max_batch, max_seq, dev, backend: str = "fused") -> int:
        """MODEL_CONFIG ``kv_pages``: 0 = per-slot caches (``max_batch x max_seq`` rows), N = a
        shared pool of N 64-row pages, ``auto`` = as many pages as half the free HBM holds, capped
        at what ``max_batch`` full-length sequences could use (+ the scratch page).  Under TP the
        ranks then agree on the minimum (rank 0's admissions are replayed on every rank)."""
        if spec in (0, "0", None, ""):
            return 0
        full = max_batch * -(-max_seq // 64) + 1
        if str(spec) != "auto":
            return int(spec)
        from ..models.llama import shard_dims

        elem = 2 if backend == "fused" else 4  # LlamaTP: bf16 caches when fused, fp32 for the reference backend
        page_bytes = cfg.layers * 2 * 64 * shard_dims(cfg, tp, 0).hkv * cfg.head_dim * elem
        if torch.device(dev).type != "cuda":
            return full
        free, _total = torch.cuda.mem_get_info(torch.device(dev))
        return max(2, min(full, int(free * 0.5) // page_bytes))

    # ------------------------------------------------------------------ request path
    def prepare_generate(self, req: dict) -> Tuple[List[int], Any]:
        from ..models.llama import GenParams

        if "input_ids" in req:
            ids = [int(i) for i in req["input_ids"]]
        else:
            ids = self.tok.encode(str(req["prompt"]))
        gp = GenParams(max_new_tokens=int(req.get("max_new_tokens", self.ctx.settings.MAX_NEW_TOKENS)),
                       top_k=int(req.get("top_k", 1)), temperature=float(req.get("temperature", 1.0)),
                       seed=int(req.get("seed", 0)))
        if not ids:
            raise ValueError("empty prompt")
        if gp.max_new_tokens < 1:
            raise ValueError("max_new_tokens must be >= 1")
        return ids, gp

    def submit_generate(self, sample):
        """Continuous batching: enqueue into the scheduler; a concurrent.futures.Future of the
        ``(prompt_len, tokens)`` pair :meth:`finish_generate` formats (None: no engine)."""
        if self.engine is None:
            return None
        ids, gp = sample
        fut = self.engine.submit(ids, gp)
        import concurrent.futures as cf

        out: cf.Future = cf.Future()

        def done(f, n=len(ids)):
            if f.exception() is not None:
                out.set_exception(f.exception())
            else:
                out.set_result((n, f.result()))

        fut.add_done_callback(done)
        return out

    def finish_generate(self, out: Any) -> dict:
        prompt_len, toks = out
        eos = set(self.cfg.eos_ids)
        cut = next((i + 1 for i, t in enumerate(toks) if t in eos), len(toks))
        toks = toks[:cut]
        return {"token_ids": toks, "text": self.tok.decode(toks), "num_tokens": len(toks), "prompt_tokens": prompt_len}

    def replicas(self):
        def run_batch(samples):
            groups: Dict[tuple, List[int]] = {}
            for i, (_ids, gp) in enumerate(samples):
                groups.setdefault((gp.top_k, gp.temperature, gp.seed), []).append(i)
            results: List[Any] = [None] * len(samples)
            for _key, members in groups.items():
                ids_l = [samples[i][0] for i in members]
                gp = samples[members[0]][1]
                from ..models.llama import GenParams

                gpg = GenParams(max(samples[i][1].max_new_tokens for i in members), gp.top_k, gp.temperature, gp.seed)
                toks = self._generate_batch(ids_l, gpg)
                for j, i in enumerate(members):
                    results[i] = (len(ids_l[j]), toks[j][: samples[i][1].max_new_tokens])
            return results

        return [run_batch]

    # ------------------------------------------------------------------ lockstep execution
    def _broadcast_cmd(self, op: int, ids: torch.Tensor = None, lens: torch.Tensor = None, gp=None) -> None:
        import torch.distributed as dist

        if self.model.tp == 1:
            return
        hdr = torch.zeros(7, dtype=torch.int64, device=self.comm_dev)
        if op == OP_GENERATE:
            hdr[:] = torch.tensor([op, ids.shape[0], ids.shape[1], gp.max_new_tokens, gp.top_k,
                                   int(gp.temperature * 1000), gp.seed])
        dist.broadcast(hdr, src=0)
        if op == OP_GENERATE:
            dist.broadcast(ids.to(self.comm_dev), src=0)
            dist.broadcast(lens.to(self.comm_dev), src=0)

    def _generate_batch(self, ids_l: List[List[int]], gp) -> List[List[int]]:
        S = max(len(t) for t in ids_l)
        B = len(ids_l)
        ids = torch.zeros(B, S, dtype=torch.int32)
        for i, t in enumerate(ids_l):
            ids[i, : len(t)] = torch.tensor(t, dtype=torch.int32)
        lens = torch.tensor([len(t) for t in ids_l], dtype=torch.int32)
        with self._lock:
            self._broadcast_cmd(OP_GENERATE, ids, lens, gp)
            out = self.model.generate(ids, lens, gp)
        return out.cpu().tolist()

    # ---- the continuous engine's TP control channel (models/llama_serving.py ContinuousLlama):
    # explicit headers only when no decode step carried one; admissions only when there are any
    def send_header(self, admit) -> None:
        """Rank 0: one iteration's header (None = stop), then its admissions when it has any."""
        import torch.distributed as dist

        hdr = torch.zeros(7, dtype=torch.int64, device=self.comm_dev)
        if admit is None:
            dist.broadcast(hdr, src=0)  # OP_STOP
            return
        n = len(admit)
        S = max((len(a.ids) for a in admit), default=0)
        hdr[:3] = torch.tensor([OP_ITER, n, S])
        dist.broadcast(hdr, src=0)
        if n:
            self.send_admissions(admit)

    def send_admissions(self, admit) -> None:
        """Rank 0: the admitted sequences' slot / length / sampling parameters and prompt ids."""
        import torch.distributed as dist

        n = len(admit)
        S = max(len(a.ids) for a in admit)
        meta = torch.tensor([[a.slot, len(a.ids), a.gp.max_new_tokens, a.gp.top_k, round(a.gp.temperature * 1000),
                              a.gp.seed] for a in admit], dtype=torch.int64, device=self.comm_dev)
        ids = torch.zeros(n, S, dtype=torch.int64, device=self.comm_dev)
        for j, a in enumerate(admit):
            ids[j, : len(a.ids)] = torch.tensor(a.ids, dtype=torch.int64)
        dist.broadcast(meta, src=0)
        dist.broadcast(ids, src=0)

    def recv_header(self):
        """Followers: (op, admissions, longest prompt) of rank 0's explicit header."""
        import torch.distributed as dist

        hdr = torch.zeros(7, dtype=torch.int64, device=self.comm_dev)
        dist.broadcast(hdr, src=0)
        op, n, S = hdr[:3].tolist()
        return op, n, S

    def recv_admissions(self, n: int, S: int):
        """Followers: the ``n`` sequences rank 0 admits this iteration (prompts padded to ``S``)."""
        import torch.distributed as dist

        from ..models.llama import GenParams
        from ..models.llama_serving import _Seq

        meta = torch.zeros(n, 6, dtype=torch.int64, device=self.comm_dev)
        ids = torch.zeros(n, S, dtype=torch.int64, device=self.comm_dev)
        dist.broadcast(meta, src=0)
        dist.broadcast(ids, src=0)
        admit = []
        ids_l = ids.tolist()
        for j, (slot, ln, mnt_j, topk_j, temp_j, seed_j) in enumerate(meta.tolist()):
            seq = _Seq(ids_l[j][:ln], GenParams(mnt_j, topk_j, temp_j / 1000.0, seed_j), None)
            seq.slot = slot
            admit.append(seq)
        return admit

    def _broadcast_iter(self, admit) -> None:
        """Rank 0, continuous mode, one header per iteration (the legacy hook form)."""
        self.send_header(admit)

    def follower_loop(self) -> int:
        """Ranks > 0: execute rank 0's generate commands until STOP."""
        import torch.distributed as dist

        import time

        from ..models.llama import GenParams

        if self.engine is not None:  # continuous batching: the engine's own follow loop (headers
            try:                     # carried by the decode steps where possible)
                return self.engine.follow()
            finally:
                self.follower_stats = dict(self.engine.follower_stats, **self.engine.proto)
        # per-iteration host cost of following (X5): the header broadcast + its host read, and the
        # iteration itself -- in the worker's info dump (tests/llama_tp_worker.py) and /info
        st = self.follower_stats = {"iters": 0, "hdr_s": 0.0, "hdr_max_s": 0.0, "iter_s": 0.0}
        while True:
            t0 = time.perf_counter()
            hdr = torch.zeros(7, dtype=torch.int64, device=self.comm_dev)
            dist.broadcast(hdr, src=0)
            op, B, S, mnt, topk, temp, seed = hdr.tolist()
            dt = time.perf_counter() - t0
            st["hdr_s"] += dt
            st["hdr_max_s"] = max(st["hdr_max_s"], dt)
            if op == OP_STOP:
                logger.info("rank %d: stop", self.ctx.rank)
                return 0
            if op == OP_ITER:  # continuous batching: replay rank 0's iteration
                from ..models.llama_serving import _Seq

                admit = []
                if B:
                    meta = torch.zeros(B, 6, dtype=torch.int64, device=self.comm_dev)
                    ids = torch.zeros(B, S, dtype=torch.int64, device=self.comm_dev)
                    dist.broadcast(meta, src=0)
                    dist.broadcast(ids, src=0)
                    for j, (slot, n, mnt_j, topk_j, temp_j, seed_j) in enumerate(meta.tolist()):
                        seq = _Seq(ids[j, :n].tolist(), GenParams(mnt_j, topk_j, temp_j / 1000.0, seed_j), None)
                        seq.slot = slot
                        admit.append(seq)
                t1 = time.perf_counter()
                self.engine.run_iteration(admit)  # same failure handling / health checks as rank 0
                st["iter_s"] += time.perf_counter() - t1
                st["iters"] += 1
                continue
            ids = torch.zeros(B, S, dtype=torch.int32, device=self.comm_dev)
            lens = torch.zeros(B, dtype=torch.int32, device=self.comm_dev)
            dist.broadcast(ids, src=0)
            dist.broadcast(lens, src=0)
            self.model.generate(ids, lens, GenParams(mnt, topk, temp / 1000.0, seed))

    def close(self) -> None:
        if self.engine is not None and self.ctx.rank == 0:
            self.engine.stop()  # in TP mode its scheduler announces STOP to the followers
            if self.model.tp > 1:
                return
        if self.model is not None and self.model.tp > 1 and self.ctx.rank == 0:
            try:
                self._broadcast_cmd(OP_STOP)
            except Exception as e:  # followers may already be gone
                logger.warning("stop broadcast failed: %s", e)

    def describe(self) -> dict:
        d = super().describe()
        if self.model is not None:
            d.update({"tp": self.model.tp, "backend": self.model.backend, "max_batch": self.model.max_batch,
                      "max_seq": self.model.max_seq})
        return d
