"""Throughput of the BERT (config 3) and Llama-3-8B (config 5) paths on one MI355X.

bert : sequences/s at (batch, seq) through the GpuEngine (hipGraph per bucket), fused kernels
       vs stock PyTorch-ROCm (hipBLASLt + SDPA) on the same random weights.
llama: TP=1 (all of Llama-3-8B on one GPU): prefill tokens/s and decode ms/step at several
       batch sizes with the fused kernels.
One JSON line per measurement.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _warm(step, ms):
    """Run ``step`` until ``ms`` of load have passed (the GPU's clocks ramp up over tens of ms of
    load after idling: bench.py's warmup floor, docs/PERF_NOTES.md round 6)."""
    t = time.perf_counter()
    while (time.perf_counter() - t) * 1e3 < ms:
        step()
    torch.cuda.synchronize()


def _closed_loop(eng, x, n):
    pend = []
    for _ in range(n):
        pend.append(eng.submit(x))
        if len(pend) >= eng.inflight:
            pend.pop(0).wait()
    for t in pend:
        t.wait()


def bench_bert(args):
    from mlmicroservicetemplate_amd.engine.worker import GpuEngine
    from mlmicroservicetemplate_amd.models import bert

    dev = torch.device("cuda:0")
    cfg = bert.BertConfig()
    p = bert.init_bert(cfg, 0)
    models = {"fused": lambda: bert.BertFused(p, dev, cfg), "eager": lambda: bert.BertEager(p, dev, cfg)}
    models = {k: v() for k, v in models.items() if k in args.backends}
    for S in args.seqs:
        for B in args.batches:
            rng = np.random.default_rng(0)
            toks = [list(rng.integers(1000, 30000, S)) for _ in range(B)]
            packed = bert.pack_requests(toks, S).numpy()
            for name, model in models.items():
                def fwd(x, model=model, S=S, name=name):
                    if name == "fused":  # the serving path (plugins/text_classifier.py): packed rows, fused top-k
                        return model.classify_packed(x, S, 2)
                    ids, tt, lens = bert.unpack_requests(x, S)
                    logits = model(ids, tt, lens)
                    v, i = torch.topk(torch.softmax(logits.float(), -1), 2, dim=-1)
                    return v, i.to(torch.int32)

                eng = GpuEngine(fwd, dev, (2 * S + 1,), torch.int32, buckets=[B], inflight=args.inflight, concurrent=True,
                                cu_partitions=args.cu_partition)
                eng.warmup(capture=True)
                for _ in range(5):
                    eng.run(packed)
                _warm(lambda: _closed_loop(eng, packed, 2 * eng.inflight), args.warm_ms)
                n = args.steps
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                pend = []
                for _ in range(n):
                    pend.append(eng.submit(packed))
                    if len(pend) >= eng.inflight:  # a partitioned engine may hold fewer slots
                        pend.pop(0).wait()
                for t in pend:
                    t.wait()
                dt = (time.perf_counter() - t0) / n
                print(json.dumps({"bench": "bert-base", "backend": name, "batch": B, "seq": S, "inflight": eng.inflight,
                                  "cu_partitions": eng.cu_partitions,
                                  "ms_per_batch": round(dt * 1e3, 3), "seq_per_s": round(B / dt, 1),
                                  "tokens_per_s": round(B * S / dt, 1)}), flush=True)
                del eng


def bench_llama(args):
    """``--emulate-tp N``: rank 0's shard of a TP=N model with the collectives stubbed out
    (:class:`ShardEmulationComm`) -- the per-rank kernel time of config 5 on one GPU."""
    from mlmicroservicetemplate_amd.models.llama import LLAMA3_8B, LlamaTP, ShardEmulationComm, init_llama_shard

    dev = torch.device("cuda:0")
    t0 = time.time()
    tp = args.emulate_tp
    p = init_llama_shard(LLAMA3_8B, tp, 0, seed=0, device=dev)
    comm = ShardEmulationComm(tp) if tp > 1 else None
    m = LlamaTP(p, LLAMA3_8B, tp=tp, rank=0, comm=comm, backend="fused", device=dev, max_batch=max(args.batches),
                max_seq=2048, kv_pages=args.kv_pages)
    if m.pages is not None and args.shuffle_pages:  # pages scattered as in a long-running server
        import random

        random.Random(0).shuffle(m.pages._free)
    print(json.dumps({"bench": "llama3-8b", "tp": tp, "collectives": "stubbed" if tp > 1 else "none",
                      "skinny_max_split": args.skinny_max_split, "kv_pages": args.kv_pages,
                      "init_s": round(time.time() - t0, 1)}), flush=True)
    for B in args.batches:
        S = args.prompt
        if m.pages is not None:
            m.pages.reset()
            for b in range(B):
                m.pages.assign(b, S + 1)
        ids = torch.randint(1000, 100000, (B, S), device=dev, dtype=torch.int32)
        lens = torch.full((B,), S, device=dev, dtype=torch.int32)
        pos = torch.arange(S, device=dev, dtype=torch.int32).unsqueeze(0).expand(B, S).contiguous()
        for _ in range(2):
            m.step(ids, pos, lens, decode=False, k=1)
        _warm(lambda: (m.step(ids, pos, lens, decode=False, k=1), torch.cuda.synchronize()), args.warm_ms)
        t1 = time.perf_counter()
        for _ in range(3):
            m.step(ids, pos, lens, decode=False, k=1)
        torch.cuda.synchronize()
        pre = (time.perf_counter() - t1) / 3
        tok = torch.randint(1000, 100000, (B, 1), device=dev, dtype=torch.int32)
        cur = lens.view(B, 1).clone()
        for _ in range(3):
            m.decode_step(tok, cur, 1, max_ctx=S + 1)
        _warm(lambda: (m.decode_step(tok, cur, 1, max_ctx=S + 1), torch.cuda.synchronize()), args.warm_ms)
        t2 = time.perf_counter()
        n = args.steps
        for _ in range(n):
            m.decode_step(tok, cur, 1, max_ctx=S + 1)
        torch.cuda.synchronize()
        dec = (time.perf_counter() - t2) / n
        print(json.dumps({"bench": "llama3-8b", "tp": tp, "batch": B, "prompt": S, "kv_pages": args.kv_pages,
                          "prefill_ms": round(pre * 1e3, 2), "prefill_tok_s": round(B * S / pre, 1),
                          "decode_ms_per_step": round(dec * 1e3, 3), "decode_tok_s": round(B / dec, 1)}), flush=True)


def bench_llama_serve(args):
    """Continuous batching throughput: ``--requests`` generate requests (prompt ``--prompt``,
    ``--new`` tokens each) submitted at once to a ``max_batch = batches[0]`` engine."""
    from mlmicroservicetemplate_amd.models.llama import LLAMA3_8B, GenParams, LlamaTP, init_llama_shard
    from mlmicroservicetemplate_amd.models.llama_serving import ContinuousLlama

    dev = torch.device("cuda:0")
    B = args.batches[0]
    p = init_llama_shard(LLAMA3_8B, 1, 0, seed=0, device=dev)
    m = LlamaTP(p, LLAMA3_8B, backend="fused", device=dev, max_batch=B, max_seq=2048, kv_pages=args.kv_pages)
    eng = ContinuousLlama(m).start()
    rng = np.random.default_rng(0)
    warm = [eng.submit(rng.integers(1000, 100000, args.prompt).tolist(), GenParams(4)) for _ in range(B)]
    [f.result() for f in warm]
    t0 = time.perf_counter()
    futs = [eng.submit(rng.integers(1000, 100000, args.prompt).tolist(), GenParams(args.new))
            for _ in range(args.requests)]
    lat = []
    for f in futs:
        f.result()
        lat.append(time.perf_counter() - t0)
    dt = time.perf_counter() - t0
    toks = sum(len(f.result()) for f in futs)
    eng.stop()
    print(json.dumps({"bench": "llama3-8b-continuous", "max_batch": B, "kv_pages": args.kv_pages, "requests": args.requests,
                      "prompt": args.prompt, "new_tokens": args.new, "tokens_per_s": round(toks / dt, 1),
                      "requests_per_s": round(args.requests / dt, 2), "p50_latency_s": round(float(np.median(lat)), 3),
                      "iterations": eng.iterations}), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("which", choices=["bert", "llama", "llama-serve"])
    ap.add_argument("--requests", type=int, default=128)
    ap.add_argument("--new", type=int, default=64)
    ap.add_argument("--batches", type=int, nargs="+", default=[1, 8, 32])
    ap.add_argument("--seqs", type=int, nargs="+", default=[128])
    ap.add_argument("--prompt", type=int, default=512)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warm-ms", type=float, default=200.0, help="untimed load before each timed window (0 = off)")
    ap.add_argument("--inflight", type=int, default=5, help="bert: batches in flight (co-running engine slots)")
    ap.add_argument("--backends", nargs="+", default=["fused", "eager"], help="bert: which implementations")
    ap.add_argument("--emulate-tp", type=int, default=1)
    ap.add_argument("--cu-partition", type=int, default=0,
                    help="bert: CU-masked partitions for the engine slots (engine/worker.py; 0 = off)")
    ap.add_argument("--skinny-max-split", type=int, default=0)
    ap.add_argument("--kv-pages", type=int, default=0, help="llama: paged KV pool of N 64-row pages (0: per-slot)")
    ap.add_argument("--shuffle-pages", action="store_true", help="llama: hand out pages in random order")
    args = ap.parse_args()
    if args.skinny_max_split:
        from mlmicroservicetemplate_amd.ops import _lib

        _lib.lib().mls_skinny_set_max_split(args.skinny_max_split)
    {"bert": bench_bert, "llama": bench_llama, "llama-serve": bench_llama_serve}[args.which](args)


if __name__ == "__main__":
    main()
