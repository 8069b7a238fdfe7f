"""Built-in plugins: ``stub`` (reference parity), ``identity`` (config 1, CPU echo) and
``resnet50`` (configs 2 and 4).  ``bert`` and ``llama`` register from their own modules."""
from __future__ import annotations

import io
import logging
import time
import zlib
from typing import Any, List

import numpy as np

from ..api.multipart import Part
from .base import ModelPlugin, PluginContext, register

logger = logging.getLogger("mlsamd.plugin")


@register("stub")
class StubPlugin(ModelPlugin):
    """The reference stub model (reference ``src/model/model.py:6-31``): ``init`` sleeps
    (1 s there; ``STUB_INIT_S`` here), ``predict`` opens the upload with PIL -- which only parses
    the header, so a non-image raises (HTTP 500) -- and returns a constant result."""

    name = "stub"
    RESULT = {"classes": ["isGreen", "isRed"], "result": {"isGreen": 0, "isRed": 1}}

    def __init__(self, init_seconds: float = 1.0):
        self.init_seconds = init_seconds

    def init(self, ctx: PluginContext) -> None:
        secs = getattr(ctx.settings, "STUB_INIT_S", None)
        time.sleep(self.init_seconds if secs is None else float(secs))

    def predict(self, upload) -> dict:
        from PIL import Image

        Image.open(upload.file)  # header parse only, as the reference does
        return {"classes": list(self.RESULT["classes"]), "result": dict(self.RESULT["result"])}


@register("identity")
class IdentityPlugin(ModelPlugin):
    """Config 1: echo model on CPU through the full batched path (parser -> batcher ->
    run_batch -> postprocess).  Returns size and crc32 of the upload, so a client can verify
    the bytes made it through unchanged."""

    name = "identity"
    batched = True
    task = "echo"

    def init(self, ctx: PluginContext) -> None:
        self.ctx = ctx

    def preprocess(self, part: Part) -> Any:
        return part.data

    def replicas(self):
        def run_batch(samples: List[bytes]):
            return [{"bytes": len(s), "crc32": zlib.crc32(s) & 0xFFFFFFFF, "batch": len(samples)} for s in samples]

        return [run_batch]

    def postprocess(self, out: Any) -> dict:
        return {"classes": ["bytes", "crc32"], "result": {"bytes": out["bytes"], "crc32": out["crc32"]},
                "batch_size": out["batch"]}


RAW_CONTENT_TYPES = ("application/octet-stream", "application/x-rgb8")
IMAGE_CONTAINER_BYTES = 64 + 224 * 224 * 3  # frontend/csrc/jpeg_coefs.h


def image_container(data: bytes, content_type: str = "") -> np.ndarray:
    """Upload bytes -> GPU image container (``frontend/csrc/jpeg_coefs.h``) as a uint8 row: raw RGB8
    wrapped, baseline JPEGs Huffman-decoded by the C++ decoder, anything else decoded by PIL
    (:func:`decode_image`) and wrapped.  ``ops.image_decode`` turns a batch of them into pixels."""
    from ..frontend.native import load_extension

    ext = load_extension()
    n = 224 * 224 * 3
    if len(data) == n and (not content_type or content_type.split(";")[0].strip() in RAW_CONTENT_TYPES):
        return np.frombuffer(ext.raw_container(data), dtype=np.uint8)
    if data[:2] == b"\xff\xd8":
        c = ext.jpeg_container(data)
        if isinstance(c, bytes):
            return np.frombuffer(c, dtype=np.uint8)
    return np.frombuffer(ext.raw_container(decode_image(data, content_type).tobytes()), dtype=np.uint8)


def decode_image(data: bytes, content_type: str = "", size: int = 224, resize: int = 256) -> np.ndarray:
    """Bytes -> uint8 HWC RGB ``[size, size, 3]``: raw RGB8 of exactly that size passes through;
    otherwise PIL decode (JPEG DCT-domain downscale via ``draft``), shorter side -> ``resize``,
    centre crop ``size``."""
    n = size * size * 3
    if len(data) == n and (not content_type or content_type.split(";")[0].strip() in RAW_CONTENT_TYPES):
        return np.frombuffer(data, dtype=np.uint8).reshape(size, size, 3)
    from PIL import Image

    img = Image.open(io.BytesIO(data))
    if img.format == "JPEG":
        img.draft("RGB", (resize, resize))
    img = img.convert("RGB")
    w, h = img.size
    s = resize / min(w, h)
    nw, nh = max(size, round(w * s)), max(size, round(h * s))
    img = img.resize((nw, nh), Image.BILINEAR)
    left, top = (nw - size) // 2, (nh - size) // 2
    img = img.crop((left, top, left + size, top + size))
    return np.asarray(img, dtype=np.uint8)


@register("resnet50")
class ResNet50Plugin(ModelPlugin):
    """ResNet-50 image classifier (configs 2 and 4).  One GPU engine per device this process
    drives; each engine replays hipGraphs of the fused CDNA4 kernels (``BACKEND=fused``) or of
    stock PyTorch ops (``BACKEND=eager``, the comparison baseline)."""

    name = "resnet50"
    batched = True
    task = "image"

    def __init__(self):
        self.engines = []
        self.models = []
        self.labels: List[str] = []
        self.topk = 5

    def init(self, ctx: PluginContext) -> None:
        import torch

        from ..engine.worker import GpuEngine
        from ..models import resnet
        from ..parallel import dist as mdist

        s = ctx.settings
        self.topk = int(s.TOPK)
        self.labels = [f"class_{i}" for i in range(resnet.NUM_CLASSES)]
        devices = ctx.devices or (["cuda:0"] if torch.cuda.is_available() else [])
        if not devices:
            raise RuntimeError("resnet50 plugin needs a GPU (use MODEL=identity or stub on CPU)")
        # X1: rank 0 builds (or loads) the weights, every other rank receives them over RCCL
        params = None
        if ctx.rank == 0:
            params = resnet.load_resnet50(s.WEIGHTS) if s.WEIGHTS else resnet.init_resnet50(int(s.SEED))
        if ctx.world_size > 1:
            spec = {k: (tuple(v.shape), v.dtype) for k, v in resnet.init_resnet50_spec().items()}
            params = mdist.broadcast_state(params, src=0, device=torch.device(devices[0]), spec=spec)
        # GPU image decode: engine rows are image containers, the graph starts with ops.image_decode
        self.containers = bool(s.GPU_IMAGE_DECODE) and s.BACKEND == "fused"
        if int(s.MAX_BATCH) == 0:  # auto: plan from free HBM and the latency SLO (scheduler/capacity.py)
            self.plan_batch(s, devices[0], params)
        buckets = [b for b in s.GRAPH_BUCKETS if b <= s.MAX_BATCH]
        shape = (IMAGE_CONTAINER_BYTES,) if self.containers else (224, 224, 3)
        for dev in devices:
            serial = not bool(s.CONCURRENT_SLOTS) or int(s.INFLIGHT) <= 1
            fwd = self._build_forward(s.BACKEND, dev, max(buckets), params, serial=serial)
            if self.containers:
                from .. import ops

                model = self.models[-1]

                def fwd(x, model=model, k=self.topk):
                    # per-image decode flags ride into the fused head: an unusable container comes
                    # back as ids -1 (the request fails) instead of a black image's top-5
                    err = torch.empty(x.shape[0], dtype=torch.int32, device=x.device)
                    return model.classify(ops.image_decode(x, err=err), k, err=err)
            eng = GpuEngine(fwd, dev, shape, torch.uint8, buckets=buckets, inflight=int(s.INFLIGHT),
                            use_graphs=bool(s.USE_GRAPHS), name=f"resnet50.{dev}",
                            concurrent=bool(s.CONCURRENT_SLOTS), cu_partitions=int(s.CU_PARTITION))
            eng.warmup(capture=bool(s.USE_GRAPHS))
            self.engines.append(eng)
        logger.info("resnet50 ready on %s (backend=%s buckets=%s)", devices, s.BACKEND, buckets)

    def plan_batch(self, s, dev: str, params) -> None:
        """MAX_BATCH=0: measure this model's per-image activation bytes and time on ``dev`` and set
        MAX_BATCH + GRAPH_BUCKETS from free HBM (all in-flight slots) and LATENCY_SLO_MS."""
        import torch

        from ..models import resnet
        from ..scheduler.capacity import buckets_up_to, plan_for_device

        fused = s.BACKEND == "fused"
        probe = resnet.ResNet50Fused(params, dev, max_batch=32) if fused else resnet.ResNet50Eager(params, dev)
        gen = torch.Generator(device="cpu").manual_seed(0)

        containers = getattr(self, "containers", False)

        def make(b):
            imgs = torch.randint(0, 256, (b, 224, 224, 3), dtype=torch.uint8, generator=gen)
            if containers:  # the served rows: image containers (their decode scratch counts too)
                from ..frontend.native import load_extension

                ext = load_extension()
                rows = [np.frombuffer(ext.raw_container(im.numpy().tobytes()), dtype=np.uint8) for im in imgs]
                return torch.from_numpy(np.stack(rows)).to(dev)
            return imgs.to(dev)

        def fwd(x):
            if containers:
                from .. import ops

                err = torch.empty(x.shape[0], dtype=torch.int32, device=x.device)
                return probe.classify(ops.image_decode(x, err=err), self.topk, err=err)
            return probe.classify(x, self.topk) if fused else probe(x)

        with torch.no_grad():
            plan = plan_for_device(fwd, make, torch.device(dev), s)
        del probe
        torch.cuda.empty_cache()
        self.capacity_plan = plan
        s.MAX_BATCH = plan.max_batch
        s.GRAPH_BUCKETS = buckets_up_to(plan.max_batch)
        logger.info("auto batch: %d (bound by %s; %.1f MB/image, %.4f ms/image, %.1f GB free)", plan.max_batch,
                    plan.limit, plan.per_sample_bytes / 1e6, plan.per_sample_ms, plan.free_bytes / 1e9)

    def _build_forward(self, backend: str, dev: str, max_batch: int, params, serial: bool = False):
        import torch

        from ..models import resnet

        k = self.topk
        if backend == "fused":
            from ..ops import autotune

            tuning = autotune.load_tuning("resnet50", max_batch, regime="serial" if serial else "concurrent")
            model = resnet.ResNet50Fused(params, dev, max_batch=max_batch, tuning=tuning)
            self.models.append(model)
            return lambda x: model.classify(x, k)
        if backend == "eager":
            model = resnet.ResNet50Eager(params, dev)
            self.models.append(model)

            def fwd(x):
                v, i = torch.topk(torch.softmax(model(x).float(), -1), k, dim=-1)
                return v, i.to(torch.int32)

            return fwd
        raise ValueError(f"unknown BACKEND {backend}")

    def preprocess(self, part: Part) -> Any:
        if getattr(self, "containers", False):
            return image_container(part.data, part.content_type or "")
        return decode_image(part.data, part.content_type or "")

    def replica_probes(self):
        return [lambda e=e: e.healthy for e in self.engines]

    def replicas(self):
        out = []
        for eng in self.engines:
            def run_batch(samples, eng=eng):
                vals, idx = eng.run(samples)
                return [(vals[i], idx[i]) for i in range(len(samples))]

            out.append(run_batch)
        return out

    def postprocess(self, out: Any) -> dict:
        vals, idx = out
        if len(idx) and int(idx[0]) < 0:  # ops.image_decode flagged the container (fused head: ids -1)
            raise ValueError("undecodable image")
        return topk_result(self.labels, vals, idx)

    def configure(self, settings) -> None:
        # known before init(): the native front end sizes its rows from native_spec()
        self.containers = bool(settings.GPU_IMAGE_DECODE) and settings.BACKEND == "fused"

    def native_spec(self) -> dict:
        if getattr(self, "containers", False):
            return {"sample_bytes": IMAGE_CONTAINER_BYTES, "result": "topk", "image_container": True}
        return {"sample_bytes": 224 * 224 * 3, "result": "topk"}

    def reload_spec(self):
        from ..models import resnet

        return {k: (tuple(v.shape), v.dtype) for k, v in resnet.init_resnet50_spec().items()}

    def load_params(self, weights, seed):
        from ..models import resnet

        return resnet.load_resnet50(weights) if weights else resnet.init_resnet50(int(seed))

    def apply_params(self, params) -> None:
        for eng, model in zip(self.engines, self.models):
            with eng.quiesce():
                model.update_params(params)

    def native_replicas(self):
        from ..frontend.native import EngineReplica

        return [EngineReplica(e) for e in self.engines]

    def describe(self) -> dict:
        d = super().describe()
        d["engines"] = [e.stats() for e in self.engines]
        plan = getattr(self, "capacity_plan", None)
        if plan is not None:
            d["capacity_plan"] = plan.to_dict()
        return d


def topk_result(labels: List[str], vals, idx) -> dict:
    """Classifier result dict (``classes`` + ``result`` map, the reference stub's shape,
    reference ``model.py:31``) from one row of top-k probabilities / class ids."""
    names = [labels[int(i)] if 0 <= int(i) < len(labels) else f"class_{int(i)}" for i in idx]
    return {"classes": names, "result": {n: float(v) for n, v in zip(names, vals)}}


@register("toy_classifier")
class ToyClassifierPlugin(ModelPlugin):
    """A CPU image classifier on tiny fixed-shape inputs (``TOY_SIZE``²x3 uint8 -> 10 classes,
    fixed random linear layer + softmax + top-k): the batched fixed-shape serving path of
    configs 2/4 -- either front end, micro-batching, raw and decoded uploads -- without a GPU."""

    name = "toy_classifier"
    batched = True
    task = "image"
    NUM_CLASSES = 10

    def __init__(self, size: int = 8):
        self.size = size
        self.labels = [f"class_{i}" for i in range(self.NUM_CLASSES)]
        self.topk = 5
        self.w = None
        self.max_batch = 32
        self.inflight = 2

    def init(self, ctx: PluginContext) -> None:
        s = ctx.settings
        self.topk = min(int(s.TOPK), self.NUM_CLASSES)
        self.max_batch = int(s.MAX_BATCH)
        self.inflight = int(s.INFLIGHT)
        rng = np.random.default_rng(int(s.SEED))
        self.w = (rng.standard_normal((self.NUM_CLASSES, self.size * self.size * 3)) / 8).astype(np.float32)

    def scores(self, x: np.ndarray):
        """uint8 ``[n, size, size, 3]`` -> (probs fp32 ``[n, k]``, ids int32 ``[n, k]``)."""
        logits = (x.reshape(len(x), -1).astype(np.float32) / 255.0) @ self.w.T
        p = np.exp(logits - logits.max(1, keepdims=True))
        p /= p.sum(1, keepdims=True)
        idx = np.argsort(-p, axis=1, kind="stable")[:, : self.topk].astype(np.int32)
        return np.take_along_axis(p, idx, 1).astype(np.float32), idx

    def preprocess(self, part: Part) -> Any:
        return decode_image(part.data, part.content_type or "", size=self.size, resize=self.size)

    def replicas(self):
        def run_batch(samples):
            v, i = self.scores(np.stack(samples))
            return [(v[j], i[j]) for j in range(len(samples))]

        return [run_batch]

    def postprocess(self, out: Any) -> dict:
        vals, idx = out
        if len(idx) and int(idx[0]) < 0:  # ops.image_decode flagged the container (fused head: ids -1)
            raise ValueError("undecodable image")
        return topk_result(self.labels, vals, idx)

    def native_spec(self) -> dict:
        return {"sample_bytes": self.size * self.size * 3, "result": "topk"}

    def reload_spec(self):
        import torch

        return {"w": ((self.NUM_CLASSES, self.size * self.size * 3), torch.float32)}

    def load_params(self, weights, seed):
        import torch

        if weights:
            from ..utils.checkpoint import load_validated

            return load_validated(weights, self.reload_spec())
        rng = np.random.default_rng(int(seed))
        w = (rng.standard_normal((self.NUM_CLASSES, self.size * self.size * 3)) / 8).astype(np.float32)
        return {"w": torch.from_numpy(w)}

    def apply_params(self, params) -> None:
        self.w = params["w"].detach().cpu().float().numpy().copy()  # one reference swap: batches see old or new

    def native_replicas(self):
        from ..frontend.native import HostReplica

        return [HostReplica(self.scores, (self.size, self.size, 3), self.max_batch, self.inflight)]


def _register_optional() -> None:
    # GPU model families living in their own modules register themselves on import
    for mod in ("text_classifier", "llm"):
        try:
            __import__(f"{__package__}.{mod}")
        except ImportError as e:  # module not present yet
            logger.debug("plugin module %s unavailable: %s", mod, e)


_register_optional()
