"""``bert`` plugin: BERT-base text classifier with dynamic request batching (config 3).

``POST /predict`` takes the text as multipart field ``text`` (or a JSON body
``{"text": ...}``).  Requests are tokenised on the CPU pool, micro-batched, padded to the
smallest sequence bucket (32/64/128/256/512) that holds the longest request of the batch and
run through one engine per sequence bucket (each with its own batch-bucket hipGraphs).
"""
from __future__ import annotations

import logging
import os
from typing import Any, List


from ..api.multipart import Part
from .base import ModelPlugin, PluginContext, register

logger = logging.getLogger("mlsamd.plugin")

SEQ_BUCKETS = (32, 64, 128, 256, 512)


@register("bert")
class BertPlugin(ModelPlugin):
    name = "bert"
    batched = True
    task = "text"
    form_field = "text"

    def __init__(self):
        self.engines = {}  # device -> {seq bucket: GpuEngine}
        self.labels: List[str] = []
        self.tokenizer = None
        self.max_seq = 128
        self.cfg = None

    def configure(self, settings) -> None:
        """Labels, ``max_seq`` and the tokenizer from MODEL_CONFIG -- everything the native front
        end's packed-row geometry depends on, without touching the GPU."""
        from ..models import bert

        extra = settings.model_yaml() if hasattr(settings, "model_yaml") else {}
        self.cfg = bert.BertConfig(num_labels=int(extra.get("num_labels", 2)))
        self.labels = list(extra.get("labels", [f"label_{i}" for i in range(self.cfg.num_labels)]))
        self.max_seq = int(extra.get("max_seq", 128))
        self.tokenizer = bert.HashTokenizer(self.cfg.vocab, extra.get("vocab_file"))

    def init(self, ctx: PluginContext) -> None:
        import torch

        from ..engine.worker import GpuEngine
        from ..models import bert
        from ..parallel import dist as mdist

        s = ctx.settings
        self.configure(s)
        cfg = self.cfg
        devices = ctx.devices or (["cuda:0"] if torch.cuda.is_available() else [])
        if not devices:
            raise RuntimeError("bert plugin needs a GPU")
        params = None
        if ctx.rank == 0:
            params = bert.load_bert(s.WEIGHTS, cfg) if s.WEIGHTS else bert.init_bert(cfg, int(s.SEED))
        if ctx.world_size > 1:
            spec = bert.bert_spec(cfg)
            params = mdist.broadcast_state(params, src=0, device=torch.device(devices[0]), spec=spec)
        if not int(s.MAX_BATCH):
            # auto: 128 rows per batch -- over HTTP at 256 connections 37.8k req/s at p50 6.5 ms vs
            # 29.5k at 8.4 ms with a cap of 32 (profiles/r2_http_bert_max_batch_32_vs_128.jsonl);
            # the batcher still sends smaller batches whenever fewer requests are waiting
            s.MAX_BATCH = 128
            s.GRAPH_BUCKETS = sorted(set(list(s.GRAPH_BUCKETS) + [64, 128]))
        buckets = [b for b in s.GRAPH_BUCKETS if b <= s.MAX_BATCH]
        seqs = [q for q in SEQ_BUCKETS if q <= self.max_seq] or [self.max_seq]
        for dev in devices:
            if s.BACKEND == "fused":
                model = bert.BertFused(params, dev, cfg)
            else:
                model = bert.BertEager(params, dev, cfg)
            per = {}
            for S in seqs:
                def fwd(x, S=S, model=model):
                    if s.BACKEND == "fused":  # the packed rows straight into the embedding kernel
                        return model.classify_packed(x, S, min(int(s.TOPK), cfg.num_labels))
                    ids, tt, lens = bert.unpack_requests(x, S)
                    logits = model(ids, tt, lens)
                    v, i = torch.topk(torch.softmax(logits.float(), -1), min(int(s.TOPK), cfg.num_labels), dim=-1)
                    return v, i.to(torch.int32)

                eng = GpuEngine(fwd, dev, (2 * S + 1,), torch.int32, buckets=buckets, inflight=int(s.INFLIGHT),
                                use_graphs=bool(s.USE_GRAPHS), name=f"bert.s{S}.{dev}",
                                concurrent=bool(s.CONCURRENT_SLOTS),
                                # unpartitioned: CU-masked halves win the engine bench at B=32
                                # (30.4k vs 28.2k seq/s, B=128 level) but lose over HTTP with the
                                # per-sequence-bucket engines sharing the masked streams (18.8k vs
                                # 24.1k req/s at 64 connections, 30.9k vs 32.5k at 256;
                                # profiles/r3_bert_cu_partition_ab.jsonl); MLS_CU_PARTITION opts in
                                cu_partitions=None)
                eng.warmup(capture=bool(s.USE_GRAPHS))
                per[S] = eng
            self.engines[dev] = per
        logger.info("bert ready on %s (seq buckets %s, batch buckets %s)", devices, seqs, buckets)

    def preprocess(self, part: Part) -> Any:
        text = part.data.decode("utf-8", errors="replace")
        return self.tokenizer.encode(text, self.max_seq)

    # --- native front end: one fixed-size packed row per request at the largest seq bucket ---
    def _native_seq(self) -> int:
        return max(q for q in SEQ_BUCKETS if q <= self.max_seq) if self.max_seq >= SEQ_BUCKETS[0] else self.max_seq

    def native_spec(self) -> dict:
        # raw_samples False: a packed row is only ever built here, never taken from a client body
        spec = {"sample_bytes": (2 * self._native_seq() + 1) * 4, "result": "topk", "raw_samples": False}
        if self.tokenizer is None:
            raise RuntimeError("BertPlugin.native_spec() before configure(settings)")
        if os.environ.get("MLS_NATIVE_TOKENIZER", "1") == "1" and self.tokenizer._wp is None:
            # ASCII texts hash-tokenised on the C++ I/O threads (no Python per request; others go to
            # the Python decode threads): 25.0k / 29.2k req/s vs 17.2-19.6k / 20.0-20.7k with Python
            # tokenisation at 64 / 256 connections (profiles/r2_http_bert_tokenizer_ab_fixed.jsonl).
            # MLS_NATIVE_TOKENIZER=0 turns it off.
            from ..models import bert

            spec["text_hash"] = [self.tokenizer.vocab_size, self.max_seq, self._native_seq(), bert.CLS_ID, bert.SEP_ID]
        return spec

    def native_preprocess(self, part: Part):
        """Tokenise straight into the engine row layout (ids | type ids | length, int32)."""
        import numpy as np

        S = self._native_seq()
        ids = self.preprocess(part)[:S]
        row = np.zeros(2 * S + 1, dtype=np.int32)
        row[: len(ids)] = ids
        row[2 * S] = len(ids)
        return row

    def native_replicas(self):
        from ..frontend.native import EngineReplica

        S = self._native_seq()
        return [EngineReplica(per[S]) for per in self.engines.values()]

    def replica_probes(self):
        return [lambda per=per: all(e.healthy for e in per.values()) for per in self.engines.values()]

    def replicas(self):
        from ..models import bert

        out = []
        for dev, per in self.engines.items():
            seqs = sorted(per)

            def run_batch(samples, per=per, seqs=seqs):
                longest = max(len(t) for t in samples)
                S = next((q for q in seqs if q >= longest), seqs[-1])
                packed = bert.pack_requests(samples, S).numpy()
                vals, idx = per[S].run(packed)
                return [(vals[i], idx[i]) for i in range(len(samples))]

            out.append(run_batch)
        return out

    def postprocess(self, out: Any) -> dict:
        # same body as the native front end's C++ top-k reply (classes in probability order)
        from .builtin import topk_result

        return topk_result(self.labels, *out)

    def describe(self) -> dict:
        d = super().describe()
        d["engines"] = {dev: {S: e.stats() for S, e in per.items()} for dev, per in self.engines.items()}
        return d
