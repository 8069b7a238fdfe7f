"""Batch-size planning for ``MAX_BATCH=0`` (auto): SURVEY.md §2.E.3 P1 -- the micro-batcher's cap
is derived from the GPU's free HBM (288 GB on MI355X) divided by the measured per-sample
activation bytes of every in-flight slot, and from the latency SLO.

On MI355X the HBM bound is rarely the binding one (ResNet-50 needs a few MB of activations per
image, so 288 GB would allow tens of thousands per batch): the latency budget ``LATENCY_SLO_MS``
for one batch's GPU time, and the graph-bucket ceiling ``MAX_BATCH_CAP``, usually are.  The plan
reports which limit bound it.
"""
from __future__ import annotations

import time
from dataclasses import asdict, dataclass
from typing import Callable, List, Optional


@dataclass
class CapacityPlan:
    max_batch: int
    limit: str  # "hbm" | "slo" | "cap"
    per_sample_bytes: float
    free_bytes: float
    per_sample_ms: float
    fixed_ms: float
    slots: int

    def to_dict(self) -> dict:
        return asdict(self)


def pow2_floor(n: int) -> int:
    return 1 << (max(1, int(n)).bit_length() - 1)


def buckets_up_to(n: int) -> List[int]:
    """Powers of two up to ``n`` (plus ``n`` itself): the graph buckets of a planned cap."""
    out, b = [], 1
    while b < n:
        out.append(b)
        b *= 2
    out.append(n)
    return out


def plan_batch(per_sample_bytes: float, free_bytes: float, fraction: float, slots: int, per_sample_ms: float,
               fixed_ms: float, slo_ms: float, hard_cap: int) -> CapacityPlan:
    """Largest power-of-two batch that (a) fits ``slots`` copies of its activations in
    ``fraction`` of the free HBM and (b) keeps one batch's GPU time (``fixed_ms + b *
    per_sample_ms``) within ``slo_ms``; at most ``hard_cap``, at least 1."""
    slots = max(1, int(slots))
    by_hbm = int(fraction * free_bytes / (slots * max(per_sample_bytes, 1.0)))
    by_slo = int((slo_ms - fixed_ms) / per_sample_ms) if per_sample_ms > 0 else int(hard_cap)
    cands = {"hbm": by_hbm, "slo": by_slo, "cap": int(hard_cap)}
    limit = min(cands, key=lambda k: cands[k])
    n = max(1, pow2_floor(max(1, cands[limit])))
    return CapacityPlan(max_batch=n, limit=limit, per_sample_bytes=float(per_sample_bytes),
                        free_bytes=float(free_bytes), per_sample_ms=float(per_sample_ms), fixed_ms=float(fixed_ms),
                        slots=slots)


def measure_forward(fwd: Callable, make_input: Callable[[int], object], device, b1: int = 8, b2: int = 32,
                    iters: int = 3):
    """(bytes per sample, ms per sample, fixed ms) of ``fwd`` from two batch sizes: peak
    allocator growth and eager wall time (synchronised), differenced so constant costs cancel."""
    import torch

    def one(b):
        x = make_input(b)
        fwd(x)  # warm (kernel loads, workspaces)
        torch.cuda.synchronize(device)
        torch.cuda.reset_peak_memory_stats(device)
        base = torch.cuda.memory_allocated(device)
        t0 = time.perf_counter()
        out = None
        for _ in range(iters):
            out = fwd(x)
        torch.cuda.synchronize(device)
        dt = (time.perf_counter() - t0) / iters * 1e3
        peak = torch.cuda.max_memory_allocated(device) - base
        del out
        return float(peak), dt

    m1, t1 = one(b1)
    m2, t2 = one(b2)
    per_bytes = max((m2 - m1) / (b2 - b1), m2 / b2 * 0.5, 1.0)
    per_ms = max((t2 - t1) / (b2 - b1), 1e-4)
    fixed = max(t1 - per_ms * b1, 0.0)
    return per_bytes, per_ms, fixed


def plan_for_device(fwd: Callable, make_input: Callable[[int], object], device, settings,
                    slots: Optional[int] = None) -> CapacityPlan:
    import torch

    per_bytes, per_ms, fixed = measure_forward(fwd, make_input, device)
    free, _total = torch.cuda.mem_get_info(device)
    return plan_batch(per_bytes, free, float(settings.HBM_FRACTION), slots or int(settings.INFLIGHT), per_ms, fixed,
                      float(settings.LATENCY_SLO_MS), int(settings.MAX_BATCH_CAP))
