"""Service launcher: ``python -m mlmicroservicetemplate_amd serve``.

Replaces the reference's ``uvicorn src.server.main:app --port ${PORT}`` compose command
(reference ``docker-compose.yml:6``) with an MI355X-first process layout:

* ``GPUS <= 1``: one uvicorn process, one engine (configs 1-3).
* ``GPUS = N > 1``, data-parallel models (resnet50, bert): N processes, one per GPU, all
  serving the SAME port through ``SO_REUSEPORT`` (the kernel spreads connections across
  them), joined in one RCCL process group: rank 0 builds the weights and broadcasts them over
  xGMI (X1), ``/status`` turns ready only after every rank reported healthy (X6), and only
  rank 0 runs the orchestrator heartbeat (one registered service).  (config 4)
* ``TP = N > 1`` (llama): N processes in one tensor-parallel group; rank 0 serves HTTP and
  broadcasts each request's tokens to the other ranks (X5), which run the TP forward in
  lockstep (config 5).

The parent only supervises and forwards SIGINT/SIGTERM.  Failure policy:

* start-up (before every rank reported ready) and TP groups: a dead rank stops the others -- it
  would hang the X1 / X6 / X2 collectives;
* DP replicas after start-up are independent (the process group is idle once the weights are
  broadcast): a dead replica is restarted as a FRESH standalone process (``WORLD_SIZE=1`` on the
  same GPU) that loads its own weights (``SEED`` / ``WEIGHTS``, or the last completed hot reload),
  runs its init BEFORE accepting connections (``MLS_DEFER_LISTEN``: no 503 window), and then
  shares the port again; the survivors keep serving throughout, so ``/status`` stays 200 while at
  least one replica is up.  At most ``MAX_RESTARTS`` restarts per replica in ``RESTART_WINDOW_S``;
  distributed hot reload is refused (409) once a replica has left the group.  Reference analogue:
  independent replica containers (reference ``README.md:36-40``).
"""
from __future__ import annotations

import argparse
import json
import logging
import os
import shutil
import signal
import socket
import subprocess
import sys
import tempfile
import time
from typing import Dict, List, Optional

from .config import Settings, load_dotenv

logger = logging.getLogger("mlsamd.serve")

DP_MODELS = {"resnet50", "bert", "identity", "stub", "toy_classifier"}


def secrets_token() -> str:
    import secrets  # stdlib (this package never shadows it: SURVEY.md §7.4)

    return secrets.token_hex(8)


def free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def reuseport_socket(host: str, port: int) -> socket.socket:
    sock = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
    sock.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
    if hasattr(socket, "SO_REUSEPORT"):
        sock.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEPORT, 1)
    sock.bind((host, port))
    sock.listen(2048)
    sock.set_inheritable(True)
    return sock


def _overrides_from_args(args) -> Dict[str, object]:
    o = {}
    for k in ("MODEL", "PORT", "GPUS", "TP", "MAX_BATCH", "MAX_WAIT_US", "BACKEND", "NAME", "SERVER_PORT",
              "WORKERS_PER_GPU", "FRONTEND", "IO_THREADS"):
        v = getattr(args, k.lower(), None)
        if v is not None:
            o[k] = v
    if getattr(args, "no_register", False):
        o["REGISTER"] = False
    return o


def run_rank(args) -> int:
    """Body of one rank (also the single-process path)."""
    import uvicorn

    from .api.app import create_app
    from .parallel import dist as mdist
    from .plugins.base import default_devices, PluginContext, load_plugin

    load_dotenv(args.env_file)
    settings = Settings.load(env_file=args.env_file, overrides=_overrides_from_args(args))
    logging.basicConfig(level=getattr(logging, settings.LOG_LEVEL.upper(), logging.INFO),
                        format="%(asctime)s %(levelname)s %(name)s: %(message)s")
    info = mdist.env_info()
    devices = default_devices(settings, info.world_size, info.local_rank)
    ngpu = len(devices)
    if ngpu == 1:
        from .parallel.affinity import bind_to_gpu

        bind_to_gpu(int(devices[0].split(":")[1]), max(info.world_size, int(settings.GPUS)))
    if info.world_size > 1:
        mdist.init_distributed(device_id=info.local_rank if ngpu else None)
    ctx = PluginContext(settings=settings, rank=info.rank, world_size=info.world_size, local_rank=info.local_rank,
                        devices=devices)
    plugin = load_plugin(settings.MODEL)
    if os.environ.get("MLS_DEFER_LISTEN") == "1":
        # a respawned DP replica: initialise before the shared socket is served, so clients never
        # see this process's not-ready 503 while the surviving replicas are answering 200
        if hasattr(plugin, "configure"):
            plugin.configure(settings)
        plugin.init(ctx)
        ctx.extra["preinitialized"] = True
    if info.world_size > 1 and settings.TP > 1 and info.rank != 0:
        # tensor-parallel follower: no HTTP, run the lockstep worker loop
        plugin.init(ctx)
        mdist.all_reduce_health(True)  # matches rank 0's readiness all-reduce (X6)
        return plugin.follower_loop() if hasattr(plugin, "follower_loop") else 0
    fd = os.environ.get("MLS_LISTEN_FD")
    if settings.FRONTEND == "native":
        from .frontend.native import NativeService, supports_native

        if supports_native(plugin, settings):
            svc = NativeService(settings, plugin, ctx, host=args.host,
                                listen_fd=int(fd) if fd is not None else None)
            return svc.serve_forever()
        logger.warning("model %s has no native front-end path; serving it with FRONTEND=python", plugin.name)
    app = create_app(settings, plugin, ctx)
    config = uvicorn.Config(app, host=args.host, port=settings.PORT, log_level=settings.LOG_LEVEL.lower(),
                            lifespan="on", timeout_graceful_shutdown=10)
    server = uvicorn.Server(config)
    if fd is not None:
        sock = socket.socket(fileno=int(fd))
        server.run(sockets=[sock])
    else:
        server.run()
    return 0


def launch(args) -> int:
    load_dotenv(args.env_file)
    settings = Settings.load(env_file=args.env_file, overrides=_overrides_from_args(args))
    world = max(settings.GPUS, settings.TP) if (settings.GPUS > 1 or settings.TP > 1) else 1
    wpg = max(1, int(settings.WORKERS_PER_GPU)) if settings.TP <= 1 else 1
    if wpg > 1:
        return launch_workers(args, settings, max(1, settings.GPUS), wpg)
    if world <= 1:
        return run_rank(args)
    master_port = free_port()
    sock = None
    if settings.TP <= 1:
        sock = reuseport_socket(args.host, settings.PORT)
    procs: List[subprocess.Popen] = []
    base_env = dict(os.environ)
    base_env.update({"WORLD_SIZE": str(world), "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(master_port),
                     "MLS_LAUNCH_ID": base_env.get("MLS_LAUNCH_ID") or secrets_token(),
                     "HSA_ENABLE_IPC_MODE_LEGACY": base_env.get("HSA_ENABLE_IPC_MODE_LEGACY", "0")})
    cmd = [sys.executable, "-m", "mlmicroservicetemplate_amd", "rank", *args.passthrough]
    sup_dir = tempfile.mkdtemp(prefix="mls-sup-")  # 0700: ready markers of the replicas
    base_env["MLS_SUPERVISOR_DIR"] = sup_dir
    for r in range(world):
        env = dict(base_env, RANK=str(r), LOCAL_RANK=str(r))
        pass_fds = ()
        if sock is not None:
            env["MLS_LISTEN_FD"] = str(sock.fileno())
            pass_fds = (sock.fileno(),)
        procs.append(subprocess.Popen(cmd, env=env, pass_fds=pass_fds))
    try:
        if settings.TP <= 1:
            return _supervise_dp(procs, cmd, base_env, sock, settings, sup_dir)
        return _supervise(procs)
    finally:
        shutil.rmtree(sup_dir, ignore_errors=True)


MAX_RESTARTS = 3
RESTART_WINDOW_S = 300.0


def _respawn_env(base_env: Dict[str, str], r: int, sock, settings) -> Dict[str, str]:
    """Environment of a restarted DP replica: a standalone process on GPU ``r`` (no process
    group), weights from the last completed hot reload if there was one."""
    env = dict(base_env, RANK="0", WORLD_SIZE="1", LOCAL_RANK="0", MLS_DEVICE=str(r), MLS_REPLICA_ID=str(r),
               MLS_DEFER_LISTEN="1", MLS_RESPAWNED_REPLICA="1")
    env.pop("MASTER_PORT", None)
    if sock is not None:
        env["MLS_LISTEN_FD"] = str(sock.fileno())
    if r != 0:
        env["REGISTER"] = "0"  # one registration heartbeat per service (rank 0's)
    last = _last_reload(base_env, settings)
    if last:
        if last.get("weights"):
            env["WEIGHTS"] = str(last["weights"])
        elif last.get("seed") is not None:
            env["SEED"] = str(int(last["seed"]))
            env["WEIGHTS"] = ""
    return env


def _ctl_dir(base_env: Dict[str, str], settings) -> str:
    base = base_env.get("MLS_RELOAD_BASE") or ("/dev/shm" if os.path.isdir("/dev/shm") else tempfile.gettempdir())
    return os.path.join(base, f"mls-reload-{settings.PORT}-{base_env.get('MASTER_PORT', '0')}-"
                              f"{base_env.get('MLS_LAUNCH_ID', '0')}")


def _last_reload(base_env: Dict[str, str], settings) -> Optional[dict]:
    """The newest reload generation every original rank acknowledged without error."""
    d = _ctl_dir(base_env, settings)
    try:
        with open(os.path.join(d, "request.json")) as f:
            req = json.load(f)
        gen = int(req["generation"])
        world = int(base_env["WORLD_SIZE"])
        for r in range(world):
            with open(os.path.join(d, f"ack-{gen}-{r}.json")) as f:
                if json.load(f).get("error"):
                    return None
        return req
    except (OSError, ValueError, KeyError, TypeError):
        return None


def _mark_degraded(base_env: Dict[str, str], settings, why: str) -> None:
    d = _ctl_dir(base_env, settings)
    if os.path.isdir(d) and not os.path.islink(d):
        try:
            with open(os.path.join(d, "degraded"), "w") as f:
                f.write(why)
        except OSError:
            pass


def _supervise_dp(procs: List[subprocess.Popen], cmd, base_env: Dict[str, str], sock, settings,
                  sup_dir: str) -> int:
    world = len(procs)
    stopping = {"flag": False}
    restarts: Dict[int, List[float]] = {r: [] for r in range(world)}
    gave_up = set()

    def forward(sig, _frame):
        stopping["flag"] = True
        for p in procs:
            if p is not None and p.poll() is None:
                p.send_signal(sig)

    signal.signal(signal.SIGINT, forward)
    signal.signal(signal.SIGTERM, forward)

    def all_ready() -> bool:
        return all(os.path.exists(os.path.join(sup_dir, f"ready-{r}")) for r in range(world))

    started = False
    rc = 0
    try:
        while True:
            started = started or all_ready()
            codes = [p.poll() for p in procs]
            if all(c is not None for c in codes):
                if not stopping["flag"]:
                    rc = next((c for c in codes if c), 0) or (1 if gave_up else 0)
                break
            for r, c in enumerate(codes):
                if c is None or c == 0 or stopping["flag"] or r in gave_up:
                    continue
                if not started:  # start-up: the others are (or will be) blocked in X1 / X6
                    logger.error("rank %d exited with %s during start-up; stopping the others", r, c)
                    forward(signal.SIGTERM, None)
                    rc = c if c > 0 else 1
                    break
                now = time.monotonic()
                recent = [t for t in restarts[r] if now - t < RESTART_WINDOW_S]
                if len(recent) >= MAX_RESTARTS:
                    logger.error("replica %d exited with %s; %d restarts in %.0f s -- leaving it down", r, c,
                                 len(recent), RESTART_WINDOW_S)
                    gave_up.add(r)
                    continue
                restarts[r] = recent + [now]
                logger.error("replica %d exited with %s; restarting it (the other replicas keep serving)", r, c)
                _mark_degraded(base_env, settings, f"replica {r} exited with {c}")
                try:
                    os.unlink(os.path.join(sup_dir, f"ready-{r}"))
                except OSError:
                    pass
                pass_fds = (sock.fileno(),) if sock is not None else ()
                procs[r] = subprocess.Popen(cmd, env=_respawn_env(base_env, r, sock, settings), pass_fds=pass_fds)
            if len(gave_up) == world:
                rc = 1
                break
            time.sleep(0.2)
    finally:
        deadline = time.time() + 20
        for p in procs:
            if p.poll() is None and not stopping["flag"] and rc:
                p.send_signal(signal.SIGTERM)
        for p in procs:
            try:
                p.wait(max(0.1, deadline - time.time()))
            except subprocess.TimeoutExpired:
                p.kill()
    return rc


def _supervise(procs: List[subprocess.Popen]) -> int:
    stopping = {"flag": False}

    def forward(sig, _frame):
        stopping["flag"] = True
        for p in procs:
            if p.poll() is None:
                p.send_signal(sig)

    signal.signal(signal.SIGINT, forward)
    signal.signal(signal.SIGTERM, forward)
    rc = 0
    try:
        while True:
            codes = [p.poll() for p in procs]
            if all(c is not None for c in codes):
                rc = next((c for c in codes if c), 0)
                break
            if any(c not in (None, 0) for c in codes) and not stopping["flag"]:
                logger.error("a worker exited with %s; stopping the others", codes)
                forward(signal.SIGTERM, None)
                stopping["flag"] = True
            time.sleep(0.2)
    finally:
        deadline = time.time() + 20
        for p in procs:
            try:
                p.wait(max(0.1, deadline - time.time()))
            except subprocess.TimeoutExpired:
                p.kill()
    return rc


def launch_workers(args, settings: Settings, gpus: int, wpg: int) -> int:
    """``WORKERS_PER_GPU = W > 1``: ``gpus * W`` independent serving processes sharing the port
    (SO_REUSEPORT); worker i drives GPU ``i // W``.  The HTTP front end (parsing, decode, JSON) is
    CPU-bound in Python, so one process per GPU caps a 37k img/s engine at ~1k HTTP req/s; W
    processes multiply that, each with its own engine and model copy (the GPU runs their kernels
    concurrently, HBM holds the copies easily).  Workers are standalone (no process group): each
    builds the same deterministic weights, or loads ``WEIGHTS``."""
    sock = reuseport_socket(args.host, settings.PORT)
    procs: List[subprocess.Popen] = []
    cmd = [sys.executable, "-m", "mlmicroservicetemplate_amd", "rank", *args.passthrough]
    for i in range(gpus * wpg):
        env = dict(os.environ, RANK="0", WORLD_SIZE="1", LOCAL_RANK="0", MLS_DEVICE=str(i // wpg),
                   MLS_WORKER_INDEX=str(i), MLS_LISTEN_FD=str(sock.fileno()),
                   HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"))
        if i > 0:
            env["REGISTER"] = "0"  # one registration heartbeat per service
        procs.append(subprocess.Popen(cmd, env=env, pass_fds=(sock.fileno(),)))
    return _supervise(procs)


def build_parser() -> argparse.ArgumentParser:
    ap = argparse.ArgumentParser(prog="mlmicroservicetemplate_amd")
    sub = ap.add_subparsers(dest="cmd")
    for name in ("serve", "rank"):
        p = sub.add_parser(name)
        p.add_argument("--env-file", default=".env")
        p.add_argument("--host", default="0.0.0.0")
        p.add_argument("--port", type=int)
        p.add_argument("--model")
        p.add_argument("--gpus", type=int)
        p.add_argument("--workers-per-gpu", type=int)
        p.add_argument("--tp", type=int)
        p.add_argument("--max-batch", type=int)
        p.add_argument("--max-wait-us", type=int)
        p.add_argument("--backend")
        p.add_argument("--frontend", choices=["python", "native"])
        p.add_argument("--io-threads", type=int)
        p.add_argument("--name")
        p.add_argument("--server-port", type=int)
        p.add_argument("--no-register", action="store_true")
    b = sub.add_parser("build", help="compile the HIP kernels for gfx950")
    b.add_argument("--force", action="store_true")
    sub.add_parser("plugins", help="list registered model plugins")
    e = sub.add_parser("export-weights", help="write a model's random-init weights as .safetensors")
    e.add_argument("--model", required=True, choices=["resnet50", "bert", "llama-tiny", "llama-8b"])
    e.add_argument("--out", required=True)
    e.add_argument("--seed", type=int, default=0)
    return ap


def export_weights(model: str, out: str, seed: int = 0) -> str:
    """The exact weights a ``SEED=seed`` server would random-initialise, under canonical names --
    a ``WEIGHTS=out`` server then loads them through the validated checkpoint path."""
    from .utils.checkpoint import save_state

    if model == "resnet50":
        from .models import resnet

        state = resnet.init_resnet50(seed)
    elif model == "bert":
        from .models import bert

        state = bert.init_bert(bert.BERT_BASE, seed)
    else:
        from .models import llama

        cfg = llama.LLAMA3_8B if model == "llama-8b" else llama.tiny_config()
        state = llama.full_llama_state(cfg, seed)
    save_state(out, state, metadata={"model": model, "seed": str(seed)})
    return out


def main(argv: Optional[List[str]] = None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    ap = build_parser()
    args = ap.parse_args(argv)
    if args.cmd == "build":
        from .frontend import build as fbuild
        from .ops import build

        print(build.build(force=args.force, verbose=True))
        print(*fbuild.build(force=args.force, verbose=True))
        return 0
    if args.cmd == "plugins":
        from .plugins.base import available_plugins

        print("\n".join(available_plugins()))
        return 0
    if args.cmd == "export-weights":
        print(export_weights(args.model, args.out, args.seed))
        return 0
    if args.cmd in ("serve", None):
        if args.cmd is None:
            args = ap.parse_args(["serve"])
        args.passthrough = argv[1:] if argv and argv[0] == "serve" else []
        return launch(args)
    if args.cmd == "rank":
        return run_rank(args)
    ap.print_help()
    return 2
