"""Single-node rank launcher: one child process per GPU, no torchrun needed.

``bench.py --gpus N`` (and anything else that wants N ranks) calls :func:`spawn_ranks` from a
parent that has touched neither the GPU nor ``torch.cuda``: the parent only picks a free
rendezvous port, starts N children of the SAME command with ``RANK`` / ``LOCAL_RANK`` /
``WORLD_SIZE`` / ``LOCAL_WORLD_SIZE`` / ``MASTER_ADDR=127.0.0.1`` / ``MASTER_PORT`` set (plus
``HSA_ENABLE_IPC_MODE_LEGACY=0``: this pool's driver only supports dmabuf IPC), relays rank 0's
stdout line by line, and returns non-zero if any rank fails.  Children are started with
``subprocess`` (never ``exec``) so the launcher stays a plain supervisor.

Fail-fast is the right policy for a *collective* job (a DP bench, a TP group): a dead rank
leaves the others blocked in their next collective, so the survivors are terminated.  The
serving supervisor for independent DP replicas (``serve.py``) uses per-replica restart instead.

Reference analogue: horizontal scale by starting more replicas with distinct PORTs
(reference ``README.md:36-40``, ``docker-compose.yml:5-6,14-15``).
"""
from __future__ import annotations

import os
import signal
import socket
import subprocess
import sys
import threading
import time
from typing import Dict, List, Optional, Sequence


def free_port(host: str = "127.0.0.1") -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind((host, 0))
        return s.getsockname()[1]


def rank_env(rank: int, world: int, master_port: int, base: Optional[Dict[str, str]] = None,
             local_rank: Optional[int] = None) -> Dict[str, str]:
    env = dict(os.environ if base is None else base)
    env.update({
        "RANK": str(rank),
        "LOCAL_RANK": str(rank if local_rank is None else local_rank),
        "WORLD_SIZE": str(world),
        "LOCAL_WORLD_SIZE": str(world),
        "MASTER_ADDR": "127.0.0.1",
        "MASTER_PORT": str(master_port),
        "HSA_ENABLE_IPC_MODE_LEGACY": env.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"),
        "PYTHONUNBUFFERED": "1",
    })
    return env


def _relay(stream, sink, tag: Optional[str] = None) -> None:
    for line in iter(stream.readline, b""):
        text = line.decode(errors="replace")
        sink.write(text if tag is None else f"[{tag}] {text}")
        sink.flush()
    stream.close()


def spawn_ranks(cmd: Sequence[str], world: int, timeout_s: Optional[float] = None,
                env: Optional[Dict[str, str]] = None, stdout=None, poll_s: float = 0.1) -> int:
    """Run ``cmd`` as ``world`` ranks; rank 0's stdout goes to ``stdout`` (default: ours), every
    rank's stderr is inherited.  Returns 0 iff every rank exited 0; the first failure terminates
    the rest (SIGTERM, then SIGKILL after 15 s).  ``timeout_s`` bounds the whole job."""
    if world < 1:
        raise ValueError("world must be >= 1")
    sink = stdout if stdout is not None else sys.stdout
    port = free_port()
    procs: List[subprocess.Popen] = []
    relays: List[threading.Thread] = []
    for r in range(world):
        p = subprocess.Popen(list(cmd), env=rank_env(r, world, port, env),
                             stdout=subprocess.PIPE if r == 0 else None, start_new_session=False)
        procs.append(p)
        if r == 0:
            t = threading.Thread(target=_relay, args=(p.stdout, sink), daemon=True)
            t.start()
            relays.append(t)

    def stop_all(sig=signal.SIGTERM):
        for p in procs:
            if p.poll() is None:
                try:
                    p.send_signal(sig)
                except ProcessLookupError:
                    pass

    old = {}
    if threading.current_thread() is threading.main_thread():
        for s in (signal.SIGINT, signal.SIGTERM):
            old[s] = signal.signal(s, lambda sig, _f: stop_all(sig))
    deadline = None if timeout_s is None else time.monotonic() + timeout_s
    rc = 0
    try:
        while True:
            codes = [p.poll() for p in procs]
            bad = [(r, c) for r, c in enumerate(codes) if c not in (None, 0)]
            if bad and rc == 0:
                rc = bad[0][1] if bad[0][1] > 0 else 128 - bad[0][1]
                sys.stderr.write(f"launch: rank {bad[0][0]} exited with {bad[0][1]}; stopping the others\n")
                stop_all()
            if all(c is not None for c in codes):
                break
            if deadline is not None and time.monotonic() > deadline:
                sys.stderr.write(f"launch: job exceeded {timeout_s:.0f} s; stopping all ranks\n")
                rc = rc or 124
                stop_all()
                deadline = None
            time.sleep(poll_s)
    finally:
        end = time.monotonic() + 15
        for p in procs:
            try:
                p.wait(max(0.1, end - time.monotonic()))
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()
        for t in relays:
            t.join(5)
        for s, h in old.items():
            signal.signal(s, h)
    return rc


# ----------------------------------------------------------------------------- replica readiness
def mark_replica_ready(rank: int) -> None:
    """A serving rank reports "initialised and serving" to its supervisor (``serve.py``) by
    creating ``<MLS_SUPERVISOR_DIR>/ready-<replica>``; the supervisor switches from fail-fast
    (start-up, where a dead rank would hang the X1 / X6 collectives) to per-replica restart."""
    d = os.environ.get("MLS_SUPERVISOR_DIR")
    if not d:
        return
    replica = os.environ.get("MLS_REPLICA_ID", str(rank))
    try:
        with open(os.path.join(d, f"ready-{replica}"), "w") as f:
            f.write(str(os.getpid()))
    except OSError:
        pass
