"""ASGI app (T1): the reference's REST surface plus the GPU serving routes.

Reference parity (reference ``src/server/main.py``):
  * ``GET /``        -> 200 ``["MLMicroserviceTemplate is Running!"]``            (main.py:52-58)
  * ``GET /status``  -> 503 not-ready body / 200 ready body                        (main.py:101-116)
  * ``POST /predict`` multipart field ``image_file``: missing -> 422 (validation runs before
    the readiness check), not ready -> 503, model error -> 500, else
    ``{"status": "success", "result": <model dict>}``                              (main.py:119-140)
  * legacy ``POST /predict?filename=`` reads ``IMAGE_DIR/<filename>``; missing file -> 400
    ``Invalid file name provided: [...]``                                          (old-rev main.pyc@L119-152)
  * CORS for the five localhost origins with credentials                           (main.py:21-38)
  * startup: ``init()`` on a background thread, ready flag, then the registration
    heartbeat; shutdown: not-ready, stop heartbeat, join the pool                  (main.py:61-98)

Additions: ``GET /health`` (liveness + detail), ``GET /metrics`` (Prometheus),
``POST /generate`` (LLM plugins), ``GET /info``.  ``init()`` failures are reported by
``/status`` (503 with the error) instead of being swallowed.  Requests to a batched plugin go
through the dynamic micro-batcher; decode/tokenise runs on a thread pool so the event loop
never blocks (the reference ran ``predict`` on the loop).
"""
from __future__ import annotations

import asyncio
import contextlib
import json
import logging
import os
import time
from typing import Optional

from fastapi import FastAPI, Request, status
from fastapi.exceptions import RequestValidationError
from fastapi.middleware.cors import CORSMiddleware
from starlette.concurrency import run_in_threadpool
from starlette.responses import JSONResponse, Response

from .. import discovery
from ..config import Settings, load_dotenv
from ..plugins.base import ModelPlugin, PluginContext, default_devices, load_plugin
from ..scheduler.batcher import BatcherClosed, DynamicBatcher, QueueFull, ReplicaRouter
from ..scheduler.watchdog import ReplicaWatchdog
from ..utils.metrics import CONTENT_TYPE_LATEST, Metrics, gpu_memory_collector
from .multipart import MultipartError, Part, parse_multipart
from .state import OverloadedException, PredictionException, ServiceState

logger = logging.getLogger("api")

ROOT_MESSAGE = "MLMicroserviceTemplate is Running!"
NOT_READY = "Model is not ready to receive predictions."
READY = "Model ready to receive prediction requests."


class UploadTooLarge(Exception):
    """Request body over ``MAX_UPLOAD_BYTES``: 413 (same body as the native front end)."""


async def read_body(request: Request, limit: int) -> bytes:
    """The request body, refusing (``UploadTooLarge``) anything over ``limit`` bytes: by the
    declared Content-Length before reading, and by the streamed length while reading (chunked
    bodies carry no length), so an oversized body is never buffered whole."""
    declared = request.headers.get("content-length")
    if declared is not None:
        try:
            if int(declared) > limit:
                raise UploadTooLarge()
        except ValueError:
            pass
    chunks, n = [], 0
    async for chunk in request.stream():
        n += len(chunk)
        if n > limit:
            raise UploadTooLarge()
        chunks.append(chunk)
    return b"".join(chunks)


async def read_json(request: Request, limit: int):
    """``read_body`` + JSON decode; ``None`` for an empty or invalid body."""
    body = await read_body(request, limit)
    try:
        return json.loads(body) if body else None
    except ValueError:
        return None


class ServingRuntime:
    """Owns the plugin, its replica batchers and the service state for one app."""

    def __init__(self, settings: Settings, plugin: ModelPlugin, state: ServiceState, metrics: Metrics,
                 ctx: Optional[PluginContext] = None):
        self.settings = settings
        self.plugin = plugin
        self.state = state
        self.metrics = metrics
        self.ctx = ctx or PluginContext(settings=settings, devices=default_devices(settings))
        self.router: Optional[ReplicaRouter] = None
        self.watchdog: Optional[ReplicaWatchdog] = None
        self.loop: Optional[asyncio.AbstractEventLoop] = None
        self.reloader = None  # parallel.reload.ReloadCoordinator, after init

    # ---------------------------------------------------------------- lifecycle
    def init_model(self) -> None:
        """Runs on the background pool (reference ``init_model_helper``, main.py:77-82)."""
        logger.debug("Beginning Model Initialization Process.")
        self.state.mark_init_started()
        try:
            if not self.ctx.extra.get("preinitialized"):  # a respawned replica ran init before listening
                self.plugin.init(self.ctx)
            if self.plugin.batched:
                fut = asyncio.run_coroutine_threadsafe(self._start_batchers(), self.loop)
                fut.result(timeout=60)
            if self.ctx.world_size > 1:
                from ..parallel import dist as mdist

                if not mdist.all_reduce_health(True):
                    raise RuntimeError("another rank failed to initialise")
            if self.plugin.reload_spec() is not None:
                from ..parallel.reload import ReloadCoordinator

                self.reloader = ReloadCoordinator(self.plugin, self.ctx, self.settings)
        except BaseException as e:  # report, do not swallow (reference C6 defect)
            logger.exception("model init failed")
            self.state.mark_failed(e)
            self.metrics.ready.set(0)
            return
        # the model, engines and graphs are long-lived: move them out of the cyclic GC's young
        # generations so a collection never walks them on the request path
        import gc

        gc.collect()
        gc.freeze()
        self.state.mark_ready()
        self.metrics.ready.set(1)
        from ..parallel.launch import mark_replica_ready

        mark_replica_ready(self.ctx.rank)
        logger.debug("Finishing Model Initialization Process.")
        if self.ctx.rank == 0:
            discovery.start_heartbeat(self.state, self.settings)

    async def _start_batchers(self) -> None:
        s = self.settings
        batchers = []
        for i, run_batch in enumerate(self.plugin.replicas()):
            b = DynamicBatcher(run_batch, max_batch=int(s.MAX_BATCH), max_wait_us=int(s.MAX_WAIT_US),
                               max_queue=int(s.MAX_QUEUE), inflight=int(s.INFLIGHT), name=f"replica{i}",
                               on_batch=self.metrics.on_batch(str(i)))
            batchers.append(b)
        self.router = ReplicaRouter(batchers)
        await self.router.start()
        if float(s.WATCHDOG_INTERVAL_S) > 0:
            self.watchdog = ReplicaWatchdog(
                self.router, stall_s=float(s.WATCHDOG_STALL_S), max_failures=int(s.WATCHDOG_MAX_FAILURES),
                interval_s=float(s.WATCHDOG_INTERVAL_S), cooldown_s=float(s.WATCHDOG_COOLDOWN_S),
                probes=self.plugin.replica_probes(),
                on_change=lambda i, ok, why: (None if ok else self.metrics.replica_drains.labels(str(i)).inc()))
            self.watchdog.start()

        def collect_queues():
            for i, b in enumerate(self.router.batchers):
                self.metrics.queue_depth.labels(str(i)).set(b.queue_depth)
                self.metrics.replica_healthy.labels(str(i)).set(1 if b.healthy else 0)

        self.metrics.add_collector(collect_queues)

    async def shutdown(self) -> None:
        self.state.ready_to_predict = False
        self.metrics.ready.set(0)
        if self.watchdog is not None:
            await self.watchdog.stop()
        if self.router is not None:
            await self.router.stop()
        self.state.shutdown.set()
        await run_in_threadpool(self.state.pool.shutdown, True)
        if self.reloader is not None:
            self.reloader.close()
        self.plugin.close()

    # ---------------------------------------------------------------- requests
    async def predict(self, part: Part) -> dict:
        if self.plugin.batched:
            if self.router is None:
                raise PredictionException()
            sample = await run_in_threadpool(self.plugin.preprocess, part)
            try:
                out = await self.router.submit(sample, timeout=float(self.settings.REQUEST_TIMEOUT_S))
            except QueueFull as e:
                raise OverloadedException(str(e)) from e
            except BatcherClosed as e:
                raise PredictionException() from e
            return self.plugin.postprocess(out)
        return await run_in_threadpool(self.plugin.predict, part.to_upload_file())

    async def generate(self, req: dict) -> dict:
        plugin = self.plugin
        if hasattr(plugin, "submit_generate") and getattr(plugin, "engine", None) is not None:
            # continuous batching: the plugin's scheduler owns admission and batching
            from ..models.llama_serving import EngineFull

            sample = await run_in_threadpool(plugin.prepare_generate, req)
            try:
                fut = plugin.submit_generate(sample)
            except EngineFull as e:
                raise OverloadedException(str(e)) from e
            out = await asyncio.wait_for(asyncio.wrap_future(fut), float(self.settings.REQUEST_TIMEOUT_S))
            return plugin.finish_generate(out)
        if plugin.batched and hasattr(plugin, "prepare_generate"):
            if self.router is None:
                raise PredictionException()
            sample = await run_in_threadpool(plugin.prepare_generate, req)
            try:
                out = await self.router.submit(sample, timeout=float(self.settings.REQUEST_TIMEOUT_S))
            except QueueFull as e:
                raise OverloadedException(str(e)) from e
            return plugin.finish_generate(out)
        return await run_in_threadpool(plugin.generate, req)


def _validation_missing(field: str) -> RequestValidationError:
    return RequestValidationError([{"type": "missing", "loc": ("body", field), "msg": "Field required",
                                    "input": None}])


def create_app(settings: Optional[Settings] = None, plugin: Optional[ModelPlugin] = None,
               ctx: Optional[PluginContext] = None, auto_init: bool = True) -> FastAPI:
    if settings is None:
        load_dotenv()  # reference main.py:72
        settings = Settings.load()
    if plugin is None:
        plugin = load_plugin(settings.MODEL)
    state = ServiceState(pool_workers=int(settings.POOL_WORKERS))
    metrics = Metrics()
    gm = gpu_memory_collector(metrics)
    if gm is not None:
        metrics.add_collector(gm)
    runtime = ServingRuntime(settings, plugin, state, metrics, ctx)

    @contextlib.asynccontextmanager
    async def lifespan(app: FastAPI):
        runtime.loop = asyncio.get_running_loop()
        if auto_init:
            # init off the event loop; readiness flips asynchronously (reference main.py:61-85)
            state.pool.submit(runtime.init_model)
        yield
        await runtime.shutdown()

    app = FastAPI(title="mlmicroservicetemplate_amd", lifespan=lifespan)
    app.state.runtime = runtime
    app.state.settings = settings
    app.state.service = state
    app.state.metrics = metrics

    app.add_middleware(
        CORSMiddleware,
        allow_origins=list(settings.CORS_ORIGINS),
        allow_credentials=True,
        allow_methods=["*"],
        allow_headers=["*"],
    )

    @app.exception_handler(PredictionException)
    async def prediction_exception_handler(request: Request, exc: PredictionException):
        return JSONResponse(status_code=status.HTTP_503_SERVICE_UNAVAILABLE,
                            content={"status": "failure", "detail": NOT_READY})

    @app.exception_handler(OverloadedException)
    async def overloaded_handler(request: Request, exc: OverloadedException):
        return JSONResponse(status_code=status.HTTP_503_SERVICE_UNAVAILABLE,
                            content={"status": "failure", "detail": "Server overloaded; retry later."},
                            headers={"Retry-After": "1"})

    @app.exception_handler(asyncio.TimeoutError)
    async def timeout_handler(request: Request, exc: asyncio.TimeoutError):
        # REQUEST_TIMEOUT_S elapsed while the request waited in (or ran through) its replica
        return JSONResponse(status_code=504, content={"status": "failure", "detail": "Prediction timed out."})

    @app.exception_handler(UploadTooLarge)
    async def too_large_handler(request: Request, exc: UploadTooLarge):
        return JSONResponse(status_code=413, content={"status": "failure", "detail": "Upload too large."})

    @app.exception_handler(MultipartError)
    async def multipart_handler(request: Request, exc: MultipartError):
        return JSONResponse(status_code=400, content={"status": "failure", "detail": f"Malformed upload: {exc}"})

    @app.middleware("http")
    async def count_requests(request: Request, call_next):
        t0 = time.perf_counter()
        code = 500
        try:
            response = await call_next(request)
            code = response.status_code
            return response
        finally:
            route = request.url.path if request.url.path in ("/", "/status", "/predict", "/generate", "/health") else "other"
            metrics.requests.labels(route, str(code)).inc()
            metrics.latency.labels(route).observe(time.perf_counter() - t0)

    @app.get("/")
    async def root():
        """Liveness message (reference main.py:52-58; its set literal serialises as a list)."""
        return [ROOT_MESSAGE]

    @app.get("/status")
    async def check_status():
        """503 until ``init()`` finished (reference main.py:101-116)."""
        if not state.ready_to_predict:
            if state.init_error:
                return JSONResponse(status_code=503, content={"status": "failure", "detail": NOT_READY,
                                                              "error": state.init_error})
            raise PredictionException()
        router = runtime.router
        if router is not None and router.healthy_count == 0:
            return JSONResponse(status_code=503, content={"status": "failure", "detail": NOT_READY,
                                                          "error": "no healthy replica"})
        return {"status": "success", "detail": READY}

    @app.get("/health")
    async def health():
        return {
            "status": "ok",
            "ready": state.ready_to_predict,
            "connected": state.connected,
            "init_error": state.init_error,
            "model": plugin.name,
            "replicas": runtime.router.stats() if runtime.router else [],
            "watchdog_events": runtime.watchdog.events[-20:] if runtime.watchdog else [],
            "pid": os.getpid(),
            "worker": int(os.environ.get("MLS_WORKER_INDEX", "0")),
            "devices": list(runtime.ctx.devices),
        }

    @app.get("/info")
    async def info():
        return {"settings": settings.to_dict(), "model": plugin.describe(), "rank": runtime.ctx.rank,
                "world_size": runtime.ctx.world_size}

    @app.get("/metrics")
    async def prometheus_metrics():
        metrics.connected.set(1 if state.connected else 0)
        return Response(metrics.render(), media_type=CONTENT_TYPE_LATEST)

    @app.post("/predict")
    async def create_prediction(request: Request):
        """Multipart ``image_file`` upload (reference main.py:119-140), or legacy
        ``?filename=`` under ``IMAGE_DIR`` (old-rev main.pyc@L119-152)."""
        ctype = request.headers.get("content-type", "")
        part: Optional[Part] = None
        filename = request.query_params.get("filename")
        limit = int(settings.MAX_UPLOAD_BYTES)
        if ctype.lower().startswith("multipart/form-data"):
            body = await read_body(request, limit)
            fields = parse_multipart(body, ctype)
            parts = fields.get(plugin.form_field) or []
            if parts:
                part = parts[0]
            elif "filename" in fields and filename is None:
                filename = fields["filename"][0].text()
        elif ctype.lower().startswith("application/json"):
            payload = await read_json(request, limit)
            if isinstance(payload, dict) and payload.get(plugin.form_field) is not None:
                val = payload[plugin.form_field]
                data = val.encode("utf-8") if isinstance(val, str) else str(val).encode("utf-8")
                part = Part(name=plugin.form_field, data=data, content_type="text/plain")
            elif isinstance(payload, dict) and filename is None:
                filename = payload.get("filename")
        elif ctype.lower().startswith("application/x-www-form-urlencoded"):
            form = await read_body(request, limit)
            from urllib.parse import parse_qs

            q = parse_qs(form.decode("utf-8", errors="replace"), keep_blank_values=True)
            if q.get(plugin.form_field):  # e.g. text=... for the text classifier
                part = Part(name=plugin.form_field, data=q[plugin.form_field][0].encode("utf-8"),
                            content_type="text/plain")
            elif filename is None:
                filename = (q.get("filename") or [None])[0]
        if part is None and filename is not None:
            # legacy shared-volume flow: validate readiness first, then the file
            if not state.ready_to_predict:
                raise PredictionException()
            base = os.path.realpath(settings.IMAGE_DIR)
            path = os.path.realpath(os.path.join(base, filename))
            if not path.startswith(base + os.sep) or not os.path.isfile(path):
                logger.debug("Unable to open file: %s", filename)
                return JSONResponse(status_code=400, content={
                    "status": "failure",
                    "detail": f"Invalid file name provided: [{filename}]. Unable to find image on server."})
            with open(path, "rb") as f:
                data = f.read()
            part = Part(name=plugin.form_field, data=data, filename=os.path.basename(path))
        if part is None:
            raise _validation_missing(plugin.form_field)
        if not state.ready_to_predict:
            raise PredictionException()
        result = await runtime.predict(part)
        return {"status": "success", "result": result}

    @app.post("/admin/reload")
    async def reload_weights(request: Request):
        """Hot weight reload, in place under the captured hipGraphs; every DP rank over RCCL
        (parallel/reload.py).  JSON ``{"weights": <safetensors path>}`` or ``{"seed": n}``."""
        from ..parallel.reload import handle_reload_request

        payload = await read_json(request, int(settings.MAX_UPLOAD_BYTES))
        if not state.ready_to_predict:
            raise PredictionException()
        code, body = await run_in_threadpool(handle_reload_request, runtime.reloader, settings,
                                             dict(request.headers), payload)
        return JSONResponse(status_code=code, content=body)

    @app.post("/generate")
    async def generate(request: Request):
        req = await read_json(request, int(settings.MAX_UPLOAD_BYTES))
        if req is None:
            raise RequestValidationError([{"type": "json_invalid", "loc": ("body",), "msg": "JSON body required",
                                           "input": None}])
        if not isinstance(req, dict) or ("prompt" not in req and "input_ids" not in req):
            raise _validation_missing("prompt")
        if not state.ready_to_predict:
            raise PredictionException()
        if getattr(plugin, "task", "") != "generate":
            return JSONResponse(status_code=400, content={"status": "failure",
                                                          "detail": f"model {plugin.name!r} does not generate"})
        try:
            out = await runtime.generate(req)
        except ValueError as e:
            return JSONResponse(status_code=400, content={"status": "failure", "detail": str(e)})
        metrics.tokens.inc(int(out.get("num_tokens", 0)))
        return {"status": "success", "result": out}

    return app


def app_from_env() -> FastAPI:
    """uvicorn factory: ``uvicorn --factory mlmicroservicetemplate_amd.api.app:app_from_env``."""
    return create_app()
