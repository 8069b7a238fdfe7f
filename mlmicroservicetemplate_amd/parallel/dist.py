"""Process-group bootstrap and the X1 / X5 / X6 collectives of SURVEY.md §2.E.2.

One process per GPU (torchrun or our own launcher sets RANK / LOCAL_RANK / WORLD_SIZE /
MASTER_ADDR / MASTER_PORT).  On ROCm the ``"nccl"`` backend *is* RCCL, which runs over xGMI
between the GPUs of a node; ``gloo`` is used for CPU tests.

X1 (weight broadcast for DP replicas) flattens every tensor of one dtype into ONE contiguous
buffer and broadcasts that: one large message instead of ~270 small ones, which is what a
point-to-point xGMI ring wants (per-message latency dominates small broadcasts; bandwidth is
per link).  Rank 0 builds/loads weights; the others receive them -- no rank re-initialises.
"""
from __future__ import annotations

import datetime
import os
from dataclasses import dataclass
from typing import Dict, List, Optional, Tuple

import torch
import torch.distributed as dist

from ..utils import tracing


@dataclass
class DistInfo:
    rank: int = 0
    world_size: int = 1
    local_rank: int = 0
    backend: str = "none"

    @property
    def is_distributed(self) -> bool:
        return self.world_size > 1

    @property
    def is_main(self) -> bool:
        return self.rank == 0


def env_info() -> DistInfo:
    return DistInfo(
        rank=int(os.environ.get("RANK", 0)),
        world_size=int(os.environ.get("WORLD_SIZE", 1)),
        local_rank=int(os.environ.get("LOCAL_RANK", 0)),
    )


def init_distributed(backend: Optional[str] = None, timeout_s: float = 600.0, device_id: Optional[int] = None,
                     force: bool = False) -> DistInfo:
    """Initialise the default process group from the environment.  World size 1 is a no-op
    unless ``force`` (or ``MLS_DIST_FORCE=1``): then a one-rank group is created too, which is how
    the RCCL code paths (device-tensor broadcast / all-reduce / barrier) run on a one-GPU box."""
    info = env_info()
    force = force or os.environ.get("MLS_DIST_FORCE", "0") == "1"
    if info.world_size <= 1 and not force:
        return info
    if dist.is_initialized():
        info.backend = dist.get_backend()
        return info
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    if "MASTER_PORT" not in os.environ:
        if info.world_size > 1:
            raise RuntimeError("MASTER_PORT must be set for a multi-rank process group")
        from .launch import free_port

        os.environ["MASTER_PORT"] = str(free_port())
    # dmabuf IPC only on this pool's host driver (RCCL / tensor sharing across processes)
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    if backend is None:  # MLS_DIST_BACKEND=gloo: rehearse several ranks on one GPU (RCCL refuses that)
        backend = os.environ.get("MLS_DIST_BACKEND") or ("nccl" if torch.cuda.is_available() else "gloo")
    kwargs = {}
    if backend == "nccl":
        dev = info.local_rank if device_id is None else device_id
        torch.cuda.set_device(dev)
        kwargs["device_id"] = torch.device("cuda", dev)
    elif torch.cuda.is_available():
        torch.cuda.set_device(info.local_rank % max(1, torch.cuda.device_count()))
    dist.init_process_group(backend=backend, rank=info.rank, world_size=info.world_size,
                            timeout=datetime.timedelta(seconds=timeout_s), **kwargs)
    info.backend = backend
    return info


def destroy() -> None:
    if dist.is_initialized():
        dist.destroy_process_group()


def barrier(group=None) -> None:
    if dist.is_initialized():
        with tracing.range("dist.barrier"):
            _barrier(group)


def _barrier(group=None) -> None:
    if dist.get_backend(group) == "nccl":
        dist.barrier(group=group, device_ids=[torch.cuda.current_device()])
    else:
        dist.barrier(group=group)


def _group_by_dtype(tensors: Dict[str, torch.Tensor]) -> Dict[torch.dtype, List[str]]:
    out: Dict[torch.dtype, List[str]] = {}
    for k in sorted(tensors):
        out.setdefault(tensors[k].dtype, []).append(k)
    return out


def broadcast_state(
    state: Optional[Dict[str, torch.Tensor]],
    src: int = 0,
    device: Optional[torch.device] = None,
    group=None,
    spec: Optional[Dict[str, Tuple[Tuple[int, ...], torch.dtype]]] = None,
) -> Dict[str, torch.Tensor]:
    """X1: broadcast a name->tensor dict from ``src``.  Non-src ranks pass ``state=None`` plus the
    ``spec`` (shapes/dtypes, known from the architecture) -- or ``spec=None`` to receive it via
    a small object broadcast first.  Returns tensors on ``device`` on every rank."""
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    if not dist.is_initialized():
        assert state is not None
        return {k: v.to(device) if device is not None else v for k, v in state.items()}
    with tracing.range("dist.broadcast"):
        return _broadcast_state(state, src, device, group, spec, rank)


def _broadcast_state(state, src, device, group, spec, rank) -> Dict[str, torch.Tensor]:
    backend = dist.get_backend(group)
    comm_dev = torch.device("cuda", torch.cuda.current_device()) if backend == "nccl" else torch.device("cpu")
    if spec is None:
        obj = [{k: (tuple(v.shape), v.dtype) for k, v in state.items()} if rank == src else None]
        dist.broadcast_object_list(obj, src=src, group=group)
        spec = obj[0]
    out: Dict[str, torch.Tensor] = {}
    groups = _group_by_dtype({k: torch.empty(0, dtype=d) for k, (_s, d) in spec.items()})
    for dtype, names in groups.items():
        numels = [int(torch.Size(spec[n][0]).numel()) for n in names]
        total = sum(numels)
        if rank == src:
            flat = torch.cat([state[n].reshape(-1).to(comm_dev, dtype) for n in names])
        else:
            flat = torch.empty(total, dtype=dtype, device=comm_dev)
        dist.broadcast(flat, src=src, group=group)
        off = 0
        for n, ne in zip(names, numels):
            t = flat[off: off + ne].view(spec[n][0])
            out[n] = t.to(device) if device is not None and t.device != device else t.clone()
            off += ne
    return out


def all_reduce_health(ok: bool, group=None) -> bool:
    """X6: every rank reports readiness; True only if all are ready (gates ``/status``)."""
    if not dist.is_initialized():
        return ok
    backend = dist.get_backend(group)
    dev = torch.device("cuda", torch.cuda.current_device()) if backend == "nccl" else torch.device("cpu")
    t = torch.tensor([1 if ok else 0], dtype=torch.int32, device=dev)
    with tracing.range("dist.health"):
        dist.all_reduce(t, op=dist.ReduceOp.MIN, group=group)
    return bool(t.item())


def max_over_ranks(value: float, group=None) -> float:
    if not dist.is_initialized():
        return value
    backend = dist.get_backend(group)
    dev = torch.device("cuda", torch.cuda.current_device()) if backend == "nccl" else torch.device("cpu")
    t = torch.tensor([value], dtype=torch.float64, device=dev)
    with tracing.range("dist.max"):
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return float(t.item())


def gather_objects(obj, group=None) -> list:
    """Every rank's ``obj`` (picklable), in rank order, on every rank; ``[obj]`` without a group."""
    if not dist.is_initialized():
        return [obj]
    out = [None] * dist.get_world_size(group)
    with tracing.range("dist.gather_objects"):
        dist.all_gather_object(out, obj, group=group)
    return out


def all_ranks_true(flag: bool, group=None) -> bool:
    """True only if ``flag`` holds on every rank (a capability every rank must agree on)."""
    return all(bool(x) for x in gather_objects(bool(flag), group))


def group_description(group=None) -> dict:
    """The process group as it was formed: backend and world size (``none`` / 1 without one)."""
    if not dist.is_initialized():
        return {"dist_backend": "none", "dist_world": 1}
    return {"dist_backend": str(dist.get_backend(group)), "dist_world": int(dist.get_world_size(group))}


def merge_rank_configs(per_rank: List[dict]) -> dict:
    """Fold per-rank config dicts into one: a key every rank agrees on keeps its value, a key the
    ranks disagree on becomes ``"mixed"`` with the per-rank values under ``<key>_per_rank``;
    ``ranks_consistent`` says whether all agreed."""
    merged: dict = {}
    consistent = True
    keys = sorted({k for d in per_rank for k in d})
    for k in keys:
        vals = [d.get(k) for d in per_rank]
        if all(v == vals[0] for v in vals):
            merged[k] = vals[0]
        else:
            consistent = False
            merged[k] = "mixed"
            merged[f"{k}_per_rank"] = vals
    merged["ranks_consistent"] = consistent
    return merged
