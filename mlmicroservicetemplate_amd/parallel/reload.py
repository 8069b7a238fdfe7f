"""Hot weight reload (``POST /admin/reload``): X1 of SURVEY.md §2.E.2 "once at startup, and on hot
weight reload".

Single process: load (``WEIGHTS``-style safetensors path, or a ``seed`` for random weights), then
``plugin.apply_params`` -- which quiesces each engine (in-flight batches drain, new ones wait) and
copies the new parameters INTO the existing device tensors, so the captured hipGraphs keep
pointing at valid weights and are replayed unchanged (no re-capture, no allocation).

Data-parallel service (one process per GPU, any rank may receive the HTTP request): the receiving
rank writes the request to a small control directory shared by the service's ranks
(``/dev/shm/mls-reload-<PORT>-<MASTER_PORT>-<MLS_LAUNCH_ID>``: the launcher draws a random id per
launch, so a crashed earlier run's state is never picked up and the path cannot be guessed in
advance; the directory is created 0700 and refused if it is a symlink, owned by another user or
group/world accessible); every rank's watcher thread picks it up, rank 0
loads the checkpoint, broadcasts an ok flag and then the parameters as one flattened buffer per
dtype over RCCL/xGMI (``dist.broadcast_state``), every rank applies them and acknowledges; the
HTTP request returns once all ranks acknowledged.  The process group is otherwise idle in DP
serving, so the reload collectives never interleave with other collectives.

Ordering: a new generation is only written (under an ``fcntl`` lock on the control directory)
once every rank has acknowledged the previous one -- a second request meanwhile gets 409 -- so
every watcher applies every generation, in order, and all ranks issue the same collectives.  Rank
0 also broadcasts the generation it applies; a rank that read another one acknowledges with an
error instead of applying.  A watcher never dies on a failed generation (it writes an error ack),
and a generation older than the request timeout that some rank never acknowledged may be replaced,
so a lost rank cannot lock the endpoint into 409 for the life of the service.

Security: the endpoint is off unless ``API_KEY`` is set (403), the ``api_key`` header must match
it, and ``weights`` may only name a file under ``WEIGHTS_DIR`` (same 400 whether a path is outside
it or missing, so the endpoint does not reveal which paths exist).  Rank 0 re-validates the path
against ``WEIGHTS_DIR`` when it applies a generation, so a request that did not come through the
HTTP handler cannot load an arbitrary file either.
"""
from __future__ import annotations

import fcntl
import hmac
import json
import logging
import os
import shutil
import tempfile
import threading
import time
from typing import Any, Dict, Optional

logger = logging.getLogger("mlsamd.reload")


class ReloadError(ValueError):
    """Bad request (unknown file, shape mismatch, unsupported model): HTTP 400."""


class ReloadBusy(RuntimeError):
    """Another reload generation is still being applied by some rank: HTTP 409."""


class _DirLock:
    """Exclusive ``flock`` on ``<dir>/lock``: serialises reload requests across the ranks."""

    def __init__(self, directory: str):
        self.path = os.path.join(directory, "lock")
        self.fd = -1

    def __enter__(self):
        self.fd = os.open(self.path, os.O_CREAT | os.O_RDWR, 0o600)
        fcntl.flock(self.fd, fcntl.LOCK_EX)
        return self

    def __exit__(self, *exc):
        fcntl.flock(self.fd, fcntl.LOCK_UN)
        os.close(self.fd)
        self.fd = -1


def resolve_weights(settings, weights: Any) -> str:
    """``weights`` (relative to ``WEIGHTS_DIR``, or absolute inside it) -> a real file path under
    ``WEIGHTS_DIR``.  One error message for "outside" and "missing"."""
    base_setting = str(getattr(settings, "WEIGHTS_DIR", "") or "")
    if not base_setting:
        raise ReloadError("weights reload is disabled on this server (WEIGHTS_DIR is not set); use 'seed'")
    if not isinstance(weights, str) or not weights or "\x00" in weights:
        raise ReloadError("'weights' must be a file name under WEIGHTS_DIR")
    base = os.path.realpath(base_setting)
    path = os.path.realpath(os.path.join(base, weights))
    if not path.startswith(base + os.sep) or not os.path.isfile(path):
        raise ReloadError("'weights' must name an existing file under WEIGHTS_DIR")
    return path


def secure_control_dir(path: str) -> str:
    """Create ``path`` 0700 (if missing) and check it is a real directory owned by us and closed
    to group / world -- the ranks trust what they read there."""
    try:
        os.mkdir(path, 0o700)
    except FileExistsError:
        pass
    st = os.lstat(path)
    import stat as _stat

    if _stat.S_ISLNK(st.st_mode) or not _stat.S_ISDIR(st.st_mode):
        raise PermissionError(f"reload control path {path} is not a plain directory")
    if st.st_uid != os.getuid():
        raise PermissionError(f"reload control directory {path} is owned by uid {st.st_uid}, not {os.getuid()}")
    if st.st_mode & 0o077:
        raise PermissionError(f"reload control directory {path} is accessible to other users ({oct(st.st_mode & 0o777)})")
    return path


def _atomic_write(path: str, obj: dict) -> None:
    tmp = f"{path}.{os.getpid()}.tmp"
    with open(tmp, "w") as f:
        json.dump(obj, f)
    os.replace(tmp, path)


def _read(path: str) -> Optional[dict]:
    try:
        with open(path) as f:
            return json.load(f)
    except (OSError, ValueError):
        return None


class ReloadCoordinator:
    def __init__(self, plugin, ctx, settings, poll_s: float = 0.1):
        self.plugin = plugin
        self.ctx = ctx
        self.settings = settings
        self.poll_s = poll_s
        self.generation = 0
        self.last: Optional[dict] = None
        self._lock = threading.Lock()
        self._stop = threading.Event()
        self._thread: Optional[threading.Thread] = None
        self.ctl_dir: Optional[str] = None
        # set by serve.py's supervisor in a restarted DP replica's environment (serve._respawn_env)
        self.respawned = os.environ.get("MLS_RESPAWNED_REPLICA", "") == "1"
        if ctx.world_size > 1:
            base = os.environ.get("MLS_RELOAD_BASE") or ("/dev/shm" if os.path.isdir("/dev/shm")
                                                          else tempfile.gettempdir())
            launch = os.environ.get("MLS_LAUNCH_ID", "0")
            self.ctl_dir = secure_control_dir(os.path.join(
                base, f"mls-reload-{settings.PORT}-{os.environ.get('MASTER_PORT', '0')}-{launch}"))
            self._thread = threading.Thread(target=self._watch, name="mls-reload-watch", daemon=True)
            self._thread.start()

    @property
    def supported(self) -> bool:
        return self.plugin.reload_spec() is not None

    # ------------------------------------------------------------------ entry point (any rank)
    def request(self, weights: Optional[str] = None, seed: Optional[int] = None, timeout: float = 300.0) -> dict:
        if not self.supported:
            raise ReloadError(f"model {self.plugin.name!r} does not support weight reload")
        if weights is None and seed is None:
            raise ReloadError("give 'weights' (a safetensors path on the server) or 'seed'")
        t0 = time.perf_counter()
        if self.respawned:
            # a DP replica serve.py restarted runs outside the process group: a local reload here
            # would leave it serving other weights than the surviving replicas (which answer 409)
            raise ReloadBusy("this replica was restarted outside the process group; distributed reload is "
                             "unavailable until the service restarts")
        if self.ctl_dir is None:
            from ..utils import tracing

            with self._lock, tracing.range("reload.apply"):
                params = self.plugin.load_params(weights, seed)
                self.plugin.apply_params(params)
                self.generation += 1
                self.last = {"generation": self.generation, "weights": weights, "seed": seed}
            return {"generation": self.generation, "ranks": 1, "seconds": round(time.perf_counter() - t0, 3)}
        if os.path.exists(os.path.join(self.ctl_dir, "degraded")):
            raise ReloadBusy("a replica was restarted outside the process group; distributed reload is "
                             "unavailable until the service restarts")
        with self._lock, _DirLock(self.ctl_dir):
            cur = _read(os.path.join(self.ctl_dir, "request.json")) or {}
            prev = int(cur.get("generation", 0))
            stale = time.time() - float(cur.get("t", 0.0)) > float(cur.get("timeout", timeout))
            if prev and not stale and not all(os.path.exists(os.path.join(self.ctl_dir, f"ack-{prev}-{r}.json"))
                                              for r in range(self.ctx.world_size)):
                raise ReloadBusy(f"reload generation {prev} is still being applied; retry later")
            gen = prev + 1
            _atomic_write(os.path.join(self.ctl_dir, "request.json"),
                          {"generation": gen, "weights": weights, "seed": seed, "t": time.time(), "timeout": timeout})
        deadline = time.monotonic() + timeout
        while time.monotonic() < deadline:
            acks = [_read(os.path.join(self.ctl_dir, f"ack-{gen}-{r}.json")) for r in range(self.ctx.world_size)]
            if all(a is not None for a in acks):
                errs = [a["error"] for a in acks if a.get("error")]
                if errs:
                    raise ReloadError(errs[0])
                return {"generation": gen, "ranks": len(acks), "seconds": round(time.perf_counter() - t0, 3)}
            time.sleep(self.poll_s)
        raise TimeoutError(f"reload generation {gen}: not every rank acknowledged within {timeout} s")

    # ------------------------------------------------------------------ per-rank watcher
    def _watch(self) -> None:
        req_path = os.path.join(self.ctl_dir, "request.json")
        while not self._stop.is_set():
            req = _read(req_path)
            try:
                gen = int(req.get("generation", 0)) if req else 0
            except (TypeError, ValueError):
                gen = 0
            if gen > self.generation:
                try:
                    self._apply_distributed(req)
                except Exception as e:  # never let the watcher die silently: ack the failure
                    logger.exception("reload generation %d failed on rank %d", gen, self.ctx.rank)
                    self.generation = gen
                    _atomic_write(os.path.join(self.ctl_dir, f"ack-{gen}-{self.ctx.rank}.json"),
                                  {"rank": self.ctx.rank, "generation": gen, "error": f"{type(e).__name__}: {e}"})
            self._stop.wait(self.poll_s)

    def _apply_distributed(self, req: dict) -> None:
        import torch
        import torch.distributed as dist

        from . import dist as mdist

        gen = int(req["generation"])
        err = ""
        params = None
        if self.ctx.rank == 0:
            try:
                weights = req.get("weights")
                if weights is not None:  # re-check: the request file is not trusted to be from the handler
                    weights = resolve_weights(self.settings, weights)
                params = self.plugin.load_params(weights, req.get("seed"))
            except Exception as e:  # validated on rank 0 before any rank commits
                err = f"{type(e).__name__}: {e}"
        backend = dist.get_backend()
        dev = torch.device("cuda", torch.cuda.current_device()) if backend == "nccl" else torch.device("cpu")
        ok = torch.tensor([0 if err else 1, gen], dtype=torch.int64, device=dev)
        dist.broadcast(ok, src=0)
        flag, gen0 = (int(v) for v in ok.tolist())
        if gen0 != gen:  # cannot happen with the 409 gate; never apply out of step with rank 0
            err = f"rank {self.ctx.rank} read generation {gen}, rank 0 applies {gen0}"
            flag = 0
        if flag:
            try:
                from ..utils import tracing

                with tracing.range("reload.apply"):
                    params = mdist.broadcast_state(params, src=0, device=None, spec=self.plugin.reload_spec())
                    with self._lock:
                        self.plugin.apply_params(params)
                        self.last = {"generation": gen, "weights": req.get("weights"), "seed": req.get("seed")}
            except Exception as e:
                logger.exception("reload generation %d failed on rank %d", gen, self.ctx.rank)
                err = f"{type(e).__name__}: {e}"
        elif not err:
            err = "rank 0 could not load the weights"
        self.generation = gen
        _atomic_write(os.path.join(self.ctl_dir, f"ack-{gen}-{self.ctx.rank}.json"),
                      {"rank": self.ctx.rank, "generation": gen, "error": err})

    def close(self) -> None:
        self._stop.set()
        if self._thread is not None:
            self._thread.join(timeout=5)
        if self.ctl_dir and self.ctx.rank == 0:
            shutil.rmtree(self.ctl_dir, ignore_errors=True)


def handle_reload_request(coordinator: Optional[ReloadCoordinator], settings, headers: Dict[str, str],
                          payload: Any) -> tuple:
    """Shared by both front ends: ``(status, body_dict)``.  Auth: the ``api_key`` header must match
    ``API_KEY`` when one is configured (the key the service registers with, reference C10)."""
    key = str(getattr(settings, "API_KEY", "") or "")
    if not key:
        return 403, {"status": "failure", "detail": "admin endpoints are disabled (set API_KEY to enable)"}
    if not hmac.compare_digest(str(headers.get("api_key", "")).encode(), key.encode()):
        return 401, {"status": "failure", "detail": "invalid or missing api_key"}
    if coordinator is None:
        return 503, {"status": "failure", "detail": "Model is not ready to receive predictions."}
    if not isinstance(payload, dict):
        return 422, {"detail": [{"type": "dict_type", "loc": ["body"], "msg": "JSON object required", "input": None}]}
    seed = payload.get("seed")
    try:
        weights = payload.get("weights")
        if weights is not None:
            weights = resolve_weights(settings, weights)
        out = coordinator.request(weights=weights, seed=None if seed is None else int(seed))
    except ReloadBusy as e:
        return 409, {"status": "failure", "detail": str(e)}
    except (ReloadError, ValueError, KeyError) as e:
        return 400, {"status": "failure", "detail": str(e)}
    except TimeoutError as e:
        return 504, {"status": "failure", "detail": str(e)}
    return 200, {"status": "success", "result": out}
