"""Native front end (``FRONTEND=native``): C++ HTTP/1.1 server + C++ dynamic batcher, Python
entered once per batch.

Layout of one serving process::

    epoll I/O threads (C++, csrc/httpfront.cpp)
        accept / parse HTTP + multipart / answer GET / and /status / 422 / 503 ...
        raw fixed-shape sample -> pending queue (C++)
    dispatcher threads (Python, one per in-flight engine slot; GIL released while waiting)
        slot = replica.acquire(); (id, n) = srv.next_batch(slot's pinned buffer)   # C++ memcpy
        vals, idx = replica.run(slot, n)          # H2D -> hipGraph replay -> D2H (GpuEngine)
        srv.complete_topk(id, vals, idx)          # C++ formats + writes the n responses
    decode threads (Python): JPEG / PNG uploads -> plugin.preprocess -> srv.submit_sample
    request threads (Python): /health, /info, /metrics, legacy ?filename= -> srv.respond

The reference runs ``predict`` inline on uvicorn's event loop (reference
``src/server/main.py:119-140``); the FastAPI app (:mod:`..api.app`) keeps that surface in Python
and tops out near 1k ResNet uploads/s per process.  This path serves the same wire contract
(status codes and bodies of C3/C5/C14/C15, CORS C2) with no per-request Python.

Plugins opt in with ``native_spec()`` (sample size + result kind) and ``native_replicas()``
(objects with ``acquire / release / buffer / run`` -- :class:`EngineReplica` wraps a
:class:`~..engine.worker.GpuEngine`, :class:`HostReplica` a CPU function).
"""
from __future__ import annotations

import importlib.util
import json
import logging
import os
import queue
import signal
import threading
import time
from typing import Any, Callable, List, Optional, Sequence, Tuple
from urllib.parse import parse_qs

import numpy as np

from .. import discovery
from ..utils import tracing
from ..api.multipart import MultipartError, Part, parse_multipart
from ..api.state import ServiceState
from . import build as fbuild

logger = logging.getLogger("mlsamd.frontend")

_EXT = None


def load_extension():
    """Import the in-tree ``_httpfront`` module; build it first if it is missing or stale (a
    host-only C++ build, seconds).  No fallback: FRONTEND=native without it is an error."""
    global _EXT
    if _EXT is None:
        path = fbuild.build()[0]
        spec = importlib.util.spec_from_file_location("_httpfront", path)
        mod = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(mod)
        _EXT = mod
    return _EXT


# --------------------------------------------------------------------------------- replicas
class HostReplica:
    """A CPU "engine": ``fn(batch[n, *shape]) -> (vals [n, k], idx [n, k])`` over ``inflight``
    reusable host buffers."""

    def __init__(self, fn: Callable[[np.ndarray], Any], sample_shape: Sequence[int], max_batch: int,
                 inflight: int = 2, dtype=np.uint8):
        self.fn = fn
        self.max_batch = int(max_batch)
        self.inflight = max(1, int(inflight))
        self.healthy = True
        self._free: "queue.Queue[np.ndarray]" = queue.Queue()
        for _ in range(self.inflight):
            self._free.put(np.zeros((self.max_batch, *sample_shape), dtype=dtype))

    def acquire(self, timeout: Optional[float] = None):
        try:
            return self._free.get(timeout=timeout)
        except queue.Empty:
            return None

    def release(self, slot) -> None:
        self._free.put(slot)

    @staticmethod
    def buffer(slot) -> np.ndarray:
        return slot

    def run(self, slot, n: int):
        try:
            with tracing.range("native.handoff"):
                return self.fn(slot[:n])
        finally:
            self.release(slot)


class EngineReplica:
    """:class:`~..engine.worker.GpuEngine` adapter: the batch lands straight in a slot's pinned
    host buffer, then one H2D + hipGraph replay + D2H."""

    def __init__(self, engine):
        self.engine = engine
        self.max_batch = engine.max_batch
        self.inflight = engine.inflight

    @property
    def healthy(self) -> bool:
        return self.engine.healthy

    def acquire(self, timeout: Optional[float] = None):
        return self.engine.acquire(timeout)

    def release(self, slot) -> None:
        self.engine.release(slot)

    def buffer(self, slot) -> np.ndarray:
        return self.engine.host_buffer(slot)

    def run(self, slot, n: int):
        with tracing.range("native.handoff"):
            t = self.engine.launch(slot, n)
        return t.wait()


# --------------------------------------------------------------------------------- service
class NativeService:
    """One serving process on the native front end.  ``start()`` begins serving immediately
    (``/`` and ``/status`` answer during init) and runs ``plugin.init`` on a background thread;
    ``stop()`` drains and joins everything."""

    def __init__(self, settings, plugin, ctx, host: str = "0.0.0.0", port: Optional[int] = None,
                 listen_fd: Optional[int] = None):
        if hasattr(plugin, "configure"):  # row geometry from the settings, before init() runs
            plugin.configure(settings)
        spec = plugin.native_spec() if hasattr(plugin, "native_spec") else None
        if not spec:
            raise ValueError(f"model {plugin.name!r} has no native front-end support (use FRONTEND=python)")
        self.settings = settings
        self.plugin = plugin
        self.ctx = ctx
        self.spec = spec
        self.result_kind = spec.get("result", "topk")
        self.state = ServiceState(pool_workers=int(settings.POOL_WORKERS))
        ext = load_extension()
        self.srv = ext.Server(
            host=host, port=int(settings.PORT if port is None else port),
            listen_fd=-1 if listen_fd is None else int(listen_fd),
            io_threads=int(settings.IO_THREADS), sample_bytes=int(spec["sample_bytes"]),
            max_batch=int(settings.MAX_BATCH) or 32,  # wake-up hint only: batches are sized by the replica
            max_wait_us=int(settings.MAX_WAIT_US),
            max_queue=int(settings.MAX_QUEUE), max_upload=int(settings.MAX_UPLOAD_BYTES),
            form_field=plugin.form_field, cors_origins=list(settings.CORS_ORIGINS),
            request_timeout_s=float(settings.REQUEST_TIMEOUT_S), python_decode=True,
            raw_samples=bool(spec.get("raw_samples", True)), text_hash=list(spec.get("text_hash", [])),
            image_container=bool(spec.get("image_container", False)))
        self.replicas: List[Any] = []
        self.reloader = None  # parallel.reload.ReloadCoordinator, after init
        self._stop = threading.Event()
        self._threads: List[threading.Thread] = []
        self._live_dispatchers = 0
        self._lock = threading.Lock()
        self.t_start = time.time()

    @property
    def port(self) -> int:
        return self.srv.port

    # ---------------------------------------------------------------- lifecycle
    def start(self, auto_init: bool = True) -> "NativeService":
        self.srv.start()
        for i in range(max(1, int(self.settings.DECODE_WORKERS))):
            self._spawn(self._decode_loop, f"decode{i}")
        for i in range(2):
            self._spawn(self._request_loop, f"req{i}")
        if auto_init:
            self.state.pool.submit(self._init)
        logger.info("native front end listening on port %d (%d I/O threads)", self.port, int(self.settings.IO_THREADS))
        return self

    def _spawn(self, fn, name: str, *args) -> None:
        t = threading.Thread(target=fn, args=args, name=f"mls-native-{name}", daemon=True)
        t.start()
        self._threads.append(t)

    def _init(self) -> None:
        """Reference ``init_model_helper`` (main.py:77-82): init, ready, then register."""
        self.state.mark_init_started()
        try:
            if not self.ctx.extra.get("preinitialized"):  # a respawned replica ran init before listening
                self.plugin.init(self.ctx)
            if self.ctx.world_size > 1:
                from ..parallel import dist as mdist

                if not mdist.all_reduce_health(True):
                    raise RuntimeError("another rank failed to initialise")
            if self.plugin.reload_spec() is not None:
                from ..parallel.reload import ReloadCoordinator

                self.reloader = ReloadCoordinator(self.plugin, self.ctx, self.settings)
            self.replicas = list(self.plugin.native_replicas())
            labels = getattr(self.plugin, "labels", None)
            if labels:
                self.srv.set_labels([str(x) for x in labels])
            import gc

            gc.collect()
            gc.freeze()  # long-lived model / engine objects leave the collected generations
            for ri, rep in enumerate(self.replicas):
                for si in range(max(1, int(getattr(rep, "inflight", 1)))):
                    with self._lock:
                        self._live_dispatchers += 1
                    self._spawn(self._dispatch, f"r{ri}s{si}", rep)
        except BaseException as e:  # reported by /status, not swallowed (reference C6 defect)
            logger.exception("model init failed")
            self.state.mark_failed(e)
            self.srv.set_ready(False, self.state.init_error or "init failed")
            return
        self.state.mark_ready()
        self.srv.set_ready(True)
        from ..parallel.launch import mark_replica_ready

        mark_replica_ready(self.ctx.rank)
        if self.ctx.rank == 0:
            discovery.start_heartbeat(self.state, self.settings)

    def stop(self) -> None:
        self.state.ready_to_predict = False
        self.srv.set_ready(False)
        self._stop.set()
        self.state.shutdown.set()
        self.srv.stop()
        for t in self._threads:
            t.join(timeout=10)
        self.state.pool.shutdown(wait=True)
        if self.reloader is not None:
            self.reloader.close()
        self.plugin.close()

    def serve_forever(self) -> int:
        """Serve until SIGINT / SIGTERM (main thread only)."""
        self.start()
        for sig in (signal.SIGINT, signal.SIGTERM):
            signal.signal(sig, lambda *_: self._stop.set())
        self._stop.wait()
        logger.info("native front end shutting down")
        self.stop()
        return 0

    # ---------------------------------------------------------------- workers
    def _dispatch(self, rep) -> None:
        srv = self.srv
        try:
            while not self._stop.is_set() and rep.healthy:
                slot = rep.acquire(0.2)
                if slot is None:
                    continue
                try:
                    got = srv.next_batch(rep.buffer(slot), rep.max_batch, 200)
                except BaseException:
                    rep.release(slot)
                    raise
                if got is None:
                    rep.release(slot)
                    continue
                bid, n = got
                try:
                    out = rep.run(slot, n)  # releases the slot
                except Exception as e:
                    logger.exception("batch of %d failed", n)
                    srv.fail_batch(bid, 500, f"{type(e).__name__}: {e}")
                    continue
                if self.result_kind == "topk":
                    srv.complete_topk(bid, out[0], out[1])
                else:
                    srv.complete_json(bid, [json.dumps(self.plugin.postprocess(o)) for o in out])
        finally:
            with self._lock:
                self._live_dispatchers -= 1
                dead = self._live_dispatchers == 0 and not self._stop.is_set()
            if dead:
                logger.error("no healthy replica left; /status reports not ready")
                self.srv.set_ready(False, "no healthy replica")

    def _decode_loop(self) -> None:
        srv, plugin = self.srv, self.plugin
        # plugins whose Python-path sample differs from the engine row (bert: token list vs the
        # packed ids | type ids | length row) provide native_preprocess
        prep = getattr(plugin, "native_preprocess", None) or plugin.preprocess
        while not self._stop.is_set():
            item = srv.next_decode(200)
            if item is None:
                continue
            token, data, ctype = item
            try:
                arr = prep(Part(name=plugin.form_field, data=data, content_type=ctype))
                srv.submit_sample(token, np.ascontiguousarray(arr))
            except Exception as e:  # undecodable upload: 500, as PIL's error was in the reference
                srv.respond(token, 500, _json({"status": "failure", "detail": f"{type(e).__name__}: {e}"}))

    def _request_loop(self) -> None:
        while not self._stop.is_set():
            item = self.srv.next_request(200)
            if item is None:
                continue
            token, method, path, query, headers, body = item
            try:
                self._handle(token, method, path, query, headers, body)
            except Exception as e:
                logger.exception("%s %s failed", method, path)
                self.srv.respond(token, 500, _json({"status": "failure", "detail": f"{type(e).__name__}: {e}"}))

    # ---------------------------------------------------------------- Python-served routes
    KNOWN = {"/": "GET", "/status": "GET", "/predict": "POST", "/health": "GET", "/info": "GET", "/metrics": "GET",
             "/admin/reload": "POST"}

    def _handle(self, token, method: str, path: str, query: str, headers: dict, body: bytes) -> None:
        srv = self.srv
        if path == "/health" and method == "GET":
            srv.respond(token, 200, _json(self.health()))
        elif path == "/info" and method == "GET":
            srv.respond(token, 200, _json({"settings": self.settings.to_dict(), "model": self.plugin.describe(),
                                           "rank": self.ctx.rank, "world_size": self.ctx.world_size,
                                           "frontend": "native"}))
        elif path == "/metrics" and method == "GET":
            srv.respond(token, 200, self.metrics_text().encode(), "text/plain; version=0.0.4; charset=utf-8")
        elif path == "/predict" and method == "POST":
            self._legacy_predict(token, query, headers, body)
        elif path == "/admin/reload" and method == "POST":
            from ..parallel.reload import handle_reload_request

            if not self.state.ready_to_predict:
                srv.respond(token, 503, _json({"status": "failure", "detail": "Model is not ready to receive predictions."}))
                return
            try:
                payload = json.loads(body or b"null")
            except ValueError:
                payload = None
            code, out = handle_reload_request(self.reloader, self.settings, headers, payload)
            srv.respond(token, code, _json(out))
        elif path in self.KNOWN:
            srv.respond(token, 405, _json({"detail": "Method Not Allowed"}), headers=[("allow", self.KNOWN[path])])
        else:
            srv.respond(token, 404, _json({"detail": "Not Found"}))

    def _legacy_predict(self, token, query: str, headers: dict, body: bytes) -> None:
        """``?filename=`` / JSON / urlencoded ``filename`` -> ``IMAGE_DIR/<filename>`` (old-rev
        main.pyc@L119-152); everything else without the upload field is a 422 as in FastAPI."""
        srv, plugin = self.srv, self.plugin
        ctype = headers.get("content-type", "").lower()
        prep = getattr(plugin, "native_preprocess", None) or plugin.preprocess
        if getattr(plugin, "task", "") == "text":  # JSON / urlencoded text field (the bert plugin)
            text = None
            try:
                if ctype.startswith("application/json"):
                    payload = json.loads(body or b"null")
                    if isinstance(payload, dict) and isinstance(payload.get(plugin.form_field), str):
                        text = payload[plugin.form_field]
                elif ctype.startswith("application/x-www-form-urlencoded"):
                    text = (parse_qs(body.decode("utf-8", "replace")).get(plugin.form_field) or [None])[0]
            except ValueError:
                text = None
            if text is not None:
                if not self.state.ready_to_predict:
                    srv.respond(token, 503, _json({"status": "failure",
                                                   "detail": "Model is not ready to receive predictions."}))
                    return
                arr = prep(Part(name=plugin.form_field, data=text.encode("utf-8")))
                srv.submit_sample(token, np.ascontiguousarray(arr))
                return
        filename = (parse_qs(query).get("filename") or [None])[0]
        try:
            if filename is None and ctype.startswith("application/json"):
                payload = json.loads(body or b"null")
                if isinstance(payload, dict):
                    filename = payload.get("filename")
            elif filename is None and ctype.startswith("application/x-www-form-urlencoded"):
                filename = (parse_qs(body.decode("utf-8", "replace")).get("filename") or [None])[0]
            elif filename is None and ctype.startswith("multipart/form-data"):
                fields = parse_multipart(body, headers.get("content-type", ""))
                if fields.get("filename"):
                    filename = fields["filename"][0].text()
        except (ValueError, MultipartError):
            filename = None
        if filename is None:
            srv.respond(token, 422, _json({"detail": [{"type": "missing", "loc": ["body", plugin.form_field],
                                                       "msg": "Field required", "input": None}]}))
            return
        if not self.state.ready_to_predict:
            srv.respond(token, 503, _json({"status": "failure", "detail": "Model is not ready to receive predictions."}))
            return
        base = os.path.realpath(self.settings.IMAGE_DIR)
        p = os.path.realpath(os.path.join(base, str(filename)))
        if not p.startswith(base + os.sep) or not os.path.isfile(p):
            srv.respond(token, 400, _json({"status": "failure", "detail":
                                           f"Invalid file name provided: [{filename}]. Unable to find image on server."}))
            return
        with open(p, "rb") as f:
            data = f.read()
        arr = prep(Part(name=plugin.form_field, data=data, filename=os.path.basename(p)))
        srv.submit_sample(token, np.ascontiguousarray(arr))

    def health(self) -> dict:
        return {"status": "ok", "ready": self.state.ready_to_predict, "connected": self.state.connected,
                "init_error": self.state.init_error, "model": self.plugin.name, "frontend": "native",
                "replicas": [{"healthy": bool(r.healthy), "inflight": int(getattr(r, "inflight", 1))}
                             for r in self.replicas],
                "native": dict(self.srv.stats()), "pid": os.getpid(),
                "worker": int(os.environ.get("MLS_WORKER_INDEX", "0")), "devices": list(self.ctx.devices)}

    def metrics_text(self) -> str:
        s = dict(self.srv.stats())
        lines = []

        def metric(name, kind, help_, samples):
            lines.append(f"# HELP {name} {help_}")
            lines.append(f"# TYPE {name} {kind}")
            for labels, v in samples:
                lab = "{" + ",".join(f'{k}="{val}"' for k, val in labels.items()) + "}" if labels else ""
                lines.append(f"{name}{lab} {v}")

        metric("mls_native_requests_total", "counter", "HTTP requests parsed by the native front end",
               [({}, s.get("requests", 0))])
        metric("mls_native_responses_total", "counter", "HTTP responses by status code",
               [({"code": k[len("status_"):]}, v) for k, v in sorted(s.items()) if k.startswith("status_")])
        metric("mls_batches_total", "counter", "batches run", [({}, s.get("batches", 0))])
        metric("mls_batch_samples_total", "counter", "samples run in batches", [({}, s.get("samples", 0))])
        metric("mls_queue_depth", "gauge", "samples waiting for a batch", [({}, s.get("queue_depth", 0))])
        metric("mls_overload_rejections_total", "counter", "requests rejected by admission control",
               [({}, s.get("rejected_overload", 0))])
        metric("mls_open_connections", "gauge", "open client connections", [({}, s.get("connections_open", 0))])
        metric("mls_ready", "gauge", "1 when the model is ready", [({}, 1 if self.state.ready_to_predict else 0)])
        return "\n".join(lines) + "\n"


def _json(obj) -> bytes:
    return json.dumps(obj).encode()


def supports_native(plugin, settings=None) -> bool:
    if settings is not None and hasattr(plugin, "configure"):
        plugin.configure(settings)
    return bool(getattr(plugin, "native_spec", None) and plugin.native_spec())
