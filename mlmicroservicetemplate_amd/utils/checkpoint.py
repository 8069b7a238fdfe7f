"""Weights on disk: safetensors only -- nothing executable is ever unpickled.

The reference has no checkpointing: its ``init()`` is merely documented as the place to "fetch
all needed files" (reference ``src/model/model.py:7-10``, ``README.md:103-104``).  Here every
model family can start from random init (the benchmarks) or from a ``.safetensors`` file /
directory of shards (``WEIGHTS=...``):

* :class:`Checkpoint` opens a file or a directory of ``*.safetensors`` shards lazily (memory-
  mapped; a tensor, or a row/column slice of it, is read only when asked for -- a TP rank reads
  just its shard of each Llama matrix instead of the whole 16 GB);
* :func:`load_validated` reads a whole state dict, renaming foreign layouts (torchvision
  ResNet-50, HF BERT / Llama names) and checking every name, shape and dtype against the
  model's spec, so a wrong file fails at load time with a precise message instead of
  producing garbage predictions;
* :func:`save_state` writes one (used by ``python -m mlmicroservicetemplate_amd export-weights``).
"""
from __future__ import annotations

import glob
import os
from typing import Callable, Dict, Iterable, Optional, Tuple

import torch

Spec = Dict[str, Tuple[Tuple[int, ...], torch.dtype]]


class CheckpointError(ValueError):
    pass


def save_state(path: str, state: Dict[str, torch.Tensor], metadata: Optional[Dict[str, str]] = None) -> None:
    from safetensors.torch import save_file

    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    save_file({k: v.detach().to("cpu").contiguous() for k, v in state.items()}, path, metadata=metadata)


class Checkpoint:
    """Lazy view of a ``.safetensors`` file or a directory of shards."""

    def __init__(self, path: str):
        from safetensors import safe_open

        if os.path.isdir(path):
            files = sorted(glob.glob(os.path.join(path, "*.safetensors")))
        else:
            files = [path]
        if not files or not all(os.path.isfile(f) for f in files):
            raise CheckpointError(f"no .safetensors file at {path!r}")
        self.path = path
        self._handles = [safe_open(f, framework="pt", device="cpu") for f in files]
        self._where: Dict[str, int] = {}
        for i, h in enumerate(self._handles):
            for k in h.keys():
                if k in self._where:
                    raise CheckpointError(f"tensor {k!r} appears in two shards")
                self._where[k] = i

    def keys(self) -> Iterable[str]:
        return self._where.keys()

    def __contains__(self, name: str) -> bool:
        return name in self._where

    def _h(self, name: str):
        if name not in self._where:
            raise CheckpointError(f"{self.path}: missing tensor {name!r}")
        return self._handles[self._where[name]]

    def shape(self, name: str) -> Tuple[int, ...]:
        return tuple(self._h(name).get_slice(name).get_shape())

    def get(self, name: str) -> torch.Tensor:
        return self._h(name).get_tensor(name)

    def get_region(self, name: str, rows: Optional[slice] = None, cols: Optional[slice] = None) -> torch.Tensor:
        """``tensor[rows, cols]`` reading only that region from disk."""
        sl = self._h(name).get_slice(name)
        nd = len(sl.get_shape())
        if nd == 1:
            return sl[rows if rows is not None else slice(None)]
        return sl[rows if rows is not None else slice(None), cols if cols is not None else slice(None)]


def load_validated(path: str, spec: Spec, rename: Optional[Callable[[str], Optional[str]]] = None,
                   strict: bool = True, combine: Optional[Callable[[Dict[str, torch.Tensor]], None]] = None
                   ) -> Dict[str, torch.Tensor]:
    """Read every tensor, map its name through ``rename`` (None = drop it, e.g. BN step counters),
    let ``combine`` fuse renamed parts in place (e.g. q/k/v -> qkv), then check the result against
    ``spec`` (name -> (shape, dtype); values are cast to the spec dtype).  ``strict``: missing or
    unexpected tensors are errors; otherwise missing ones are simply absent from the result."""
    ck = Checkpoint(path)
    out: Dict[str, torch.Tensor] = {}
    for k in ck.keys():
        name = rename(k) if rename is not None else k
        if name is None:
            continue
        if name in out:
            raise CheckpointError(f"two tensors map to {name!r}")
        out[name] = ck.get(k)
    if combine is not None:
        combine(out)
    problems = []
    for name, t in list(out.items()):
        if name not in spec:
            if strict:
                problems.append(f"unexpected tensor {name!r}")
            out.pop(name)
            continue
        shape, dtype = spec[name]
        if tuple(t.shape) != tuple(shape):
            problems.append(f"{name}: shape {tuple(t.shape)} != expected {tuple(shape)}")
            continue
        out[name] = t.to(dtype)
    if strict:
        problems += [f"missing tensor {n!r}" for n in spec if n not in out]
    if problems:
        head = "; ".join(problems[:8]) + (f" (+{len(problems) - 8} more)" if len(problems) > 8 else "")
        raise CheckpointError(f"{path}: {head}")
    return out


def spec_of(state: Dict[str, torch.Tensor]) -> Spec:
    return {k: (tuple(v.shape), v.dtype) for k, v in state.items()}
