"""Model plugin contract (T2; reference ``src/model/model.py``).

The reference contract is two module functions (reference ``model.py:6-21``,
``README.md:97-111``):

    init()                 -- run once at startup, off the request path; fetch files here
    predict(image_file)    -- image_file is an upload (``.file`` is file-like), returns a dict

That contract is kept verbatim (:class:`ModulePlugin` wraps any module exposing it, and the
default ``stub`` plugin reproduces the reference stub).  GPU models add a *batched tensor
contract* so requests can be micro-batched onto the MI355X engines:

    preprocess(part) -> sample        per request, on a CPU thread (decode / tokenise)
    replicas()       -> [run_batch]   one callable per GPU replica: list[sample] -> list[out]
    postprocess(out) -> dict          per request, JSON-serialisable

and LLM plugins add ``generate(request_dict) -> dict`` for ``POST /generate``.
"""
from __future__ import annotations

import importlib
import logging
from dataclasses import dataclass, field
from typing import Any, Callable, Dict, List, Optional, Sequence

from ..api.multipart import Part

logger = logging.getLogger("mlsamd.plugin")

RunBatch = Callable[[List[Any]], Sequence[Any]]


@dataclass
class PluginContext:
    settings: Any
    rank: int = 0
    world_size: int = 1
    local_rank: int = 0
    devices: List[str] = field(default_factory=list)  # devices this process drives
    extra: Dict[str, Any] = field(default_factory=dict)


def default_devices(settings, world_size: int = 1, local_rank: int = 0) -> List[str]:
    """The devices a process drives: its own GPU when it is one rank of several, else the first
    ``GPUS`` GPUs; none for CPU models (stub / identity / user modules) or ``GPUS=0``."""
    try:
        import torch

        ngpu = torch.cuda.device_count()
    except Exception:
        ngpu = 0
    model = str(getattr(settings, "MODEL", ""))
    if not ngpu or int(getattr(settings, "GPUS", 1)) <= 0 or model in ("stub", "identity", "toy_classifier") or "." in model:
        return []
    import os

    if os.environ.get("MLS_DEVICE"):  # a launcher-assigned GPU (several workers per GPU)
        return [f"cuda:{int(os.environ['MLS_DEVICE'])}"]
    if world_size > 1:
        return [f"cuda:{local_rank}"]
    return [f"cuda:{i}" for i in range(min(int(settings.GPUS), ngpu))]


class ModelPlugin:
    name: str = "plugin"
    batched: bool = False
    task: str = "image"  # image | text | generate | echo
    form_field: str = "image_file"  # multipart field /predict reads (reference main.py:120)

    def configure(self, settings) -> None:
        """Derive request geometry (sample shapes, tokenizer, labels) from the settings alone --
        cheap, no GPU.  Called before :meth:`native_spec` and again at the start of :meth:`init`,
        so the front end's row layout and the engines always agree."""

    def init(self, ctx: PluginContext) -> None:
        """Load / build weights; may take long (runs on a background thread)."""

    # --- reference (unbatched) contract ---
    def predict(self, upload) -> dict:  # pragma: no cover - abstract
        raise NotImplementedError

    # --- batched contract ---
    def preprocess(self, part: Part) -> Any:
        raise NotImplementedError

    def replicas(self) -> List[RunBatch]:
        raise NotImplementedError

    def postprocess(self, out: Any) -> dict:
        return out

    # --- /generate ---
    def generate(self, request: dict) -> dict:
        raise NotImplementedError(f"model {self.name!r} does not support /generate")

    # --- native front end (FRONTEND=native, frontend/native.py) ---
    def native_spec(self) -> Optional[dict]:
        """``{"sample_bytes": int, "result": "topk" | "json"}`` when every request is one
        fixed-size sample the C++ batcher can pack; ``None`` = Python front end only."""
        return None

    def native_replicas(self) -> List[Any]:
        """After ``init``: one replica per engine, with ``acquire / release / buffer / run``
        (``frontend.native.EngineReplica`` / ``HostReplica``)."""
        raise NotImplementedError

    # --- hot weight reload (POST /admin/reload, parallel/reload.py) ---
    def reload_spec(self) -> Optional[Dict[str, tuple]]:
        """``{name: (shape, dtype)}`` of the parameters ``load_params`` returns (what non-source
        ranks receive in the X1 broadcast); ``None`` = reload unsupported."""
        return None

    def load_params(self, weights: Optional[str], seed: Optional[int]) -> Dict[str, Any]:
        """Rank 0 side: parameters from a safetensors path, or random ones from ``seed``."""
        raise NotImplementedError

    def apply_params(self, params: Dict[str, Any]) -> None:
        """Every rank: swap the serving weights (quiescing the engines; in place for graphs)."""
        raise NotImplementedError

    def replica_probes(self) -> List[Optional[Callable[[], bool]]]:
        """Optional per-replica health probes for the watchdog (same order as :meth:`replicas`)."""
        return []

    def describe(self) -> dict:
        return {"name": self.name, "task": self.task, "batched": self.batched}

    def close(self) -> None:
        pass


class ModulePlugin(ModelPlugin):
    """Adapter for a reference-style module with ``init()`` / ``predict(image_file)``."""

    def __init__(self, module_path: str):
        self.module_path = module_path
        self.module = importlib.import_module(module_path)
        self.name = getattr(self.module, "NAME", module_path)
        if not callable(getattr(self.module, "predict", None)):
            raise TypeError(f"{module_path} has no predict(image_file)")

    def init(self, ctx: PluginContext) -> None:
        fn = getattr(self.module, "init", None)
        if callable(fn):
            fn()

    def predict(self, upload) -> dict:
        return self.module.predict(upload)


_REGISTRY: Dict[str, Callable[[], ModelPlugin]] = {}


def register(name: str):
    def deco(factory):
        _REGISTRY[name] = factory
        return factory

    return deco


def available_plugins() -> List[str]:
    _load_builtin()
    return sorted(_REGISTRY)


def _load_builtin() -> None:
    # import for registration side effects
    from . import builtin  # noqa: F401


def load_plugin(spec: str) -> ModelPlugin:
    """``spec`` is a registered name (stub, identity, resnet50, bert, llama, ...) or a dotted
    module path exposing the reference ``init()`` / ``predict(image_file)`` contract, or
    ``module:Class`` naming a :class:`ModelPlugin` subclass."""
    _load_builtin()
    if spec in _REGISTRY:
        return _REGISTRY[spec]()
    if ":" in spec:
        mod, cls = spec.split(":", 1)
        obj = getattr(importlib.import_module(mod), cls)
        return obj()
    return ModulePlugin(spec)
