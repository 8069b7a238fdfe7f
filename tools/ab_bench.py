"""Interleaved A/B of ResNet-50 engine variants in ONE process (cdna_hip_programming.md §5.4 rule
24: separate invocations add cross-process / cross-box variance that looks like a kernel
property).  Each variant gets its own fused model + GpuEngine (hipGraphs captured per variant);
rounds alternate A, B, A, B, ... and the per-variant median / min of ms per batch are reported.

    python tools/ab_bench.py --variants chain=1 chain=0 --rounds 6 --steps 100

A variant is ``attr=value[,attr=value]`` applied to the ResNet50Fused instance before capture
(e.g. ``chain=0``), or ``env:NAME=value`` exported while that variant's model is built.
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from mlmicroservicetemplate_amd.engine.worker import GpuEngine  # noqa: E402
from mlmicroservicetemplate_amd.models.resnet import ResNet50Fused, init_resnet50  # noqa: E402
from mlmicroservicetemplate_amd.ops import autotune  # noqa: E402


def build(spec: str, params, dev, batch: int, inflight: int):
    env_saved = {}
    attrs = {}
    for kv in spec.split(","):
        k, v = kv.split("=", 1)
        if k.startswith("env:"):
            name = k[4:]
            env_saved[name] = os.environ.get(name)
            os.environ[name] = v
        else:
            attrs[k] = v
    try:
        model = ResNet50Fused(params, dev, max_batch=batch, tuning=autotune.load_tuning("resnet50", batch))
        for k, v in attrs.items():
            cur = getattr(model, k)
            if k == "chain_skip":  # '+'-separated block names whose boundary is NOT chained
                setattr(model, k, set(v.split("+")))
            else:
                setattr(model, k, type(cur)(int(v)) if isinstance(cur, (bool, int)) else type(cur)(v))
        eng = GpuEngine(lambda x: model.classify(x, 5), dev, (224, 224, 3), torch.uint8, buckets=[batch],
                        inflight=inflight, name=f"ab.{spec}", concurrent=True)
        eng.warmup(capture=True)
    finally:
        for k, v in env_saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    return eng


def run(eng, pool, steps: int, inflight: int) -> float:
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    pending = []
    for i in range(steps):
        pending.append(eng.submit(pool[i % len(pool)]))
        if len(pending) >= inflight:
            pending.pop(0).wait()
    for t in pending:
        t.wait()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) * 1e3 / steps


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", nargs="+", required=True)
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--inflight", type=int, default=5)
    ap.add_argument("--tag", default="")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    params = init_resnet50(0)
    engines = {v: build(v, params, dev, args.batch, args.inflight) for v in args.variants}
    rng = np.random.default_rng(0)
    pool = [[rng.integers(0, 256, (224, 224, 3), dtype=np.uint8) for _ in range(args.batch)] for _ in range(4)]
    for eng in engines.values():
        run(eng, pool, 20, args.inflight)
    res = {v: [] for v in args.variants}
    for r in range(args.rounds):
        order = args.variants if r % 2 == 0 else list(reversed(args.variants))
        for v in order:
            res[v].append(run(engines[v], pool, args.steps, args.inflight))
    for v, ms in res.items():
        med = statistics.median(ms)
        print(json.dumps({"tool": "ab_bench", "tag": args.tag, "variant": v, "batch": args.batch,
                          "inflight": args.inflight, "steps": args.steps, "rounds": args.rounds,
                          "ms_per_batch_median": round(med, 4), "ms_per_batch_min": round(min(ms), 4),
                          "req_per_s_median": round(args.batch / med * 1e3, 1),
                          "ms_all": [round(x, 4) for x in ms]}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
