"""GPU-worker liveness watchdog: the reference has no failure detection beyond
its registration heartbeat (reference ``src/server/server_connection.py:15-32``) and swallows
init errors; here a dead or hung replica is detected and drained so the router stops sending
it traffic, and ``/status`` / ``/health`` report it.

A replica (one :class:`DynamicBatcher` + its GPU worker) is marked unhealthy when
  * a dispatched batch has been running longer than ``stall_s`` (hung kernel / wedged GPU), or
  * ``max_failures`` batches in a row raised (dead worker, device fault), or
  * the plugin's own probe for that replica returns False (e.g. ``GpuEngine.healthy``).
A replica drained for failures is re-admitted on probation after ``cooldown_s`` (one more
failure drains it again); a stalled one comes back only once its stuck batch finishes.
Fault injection for tests: :class:`FaultInjector` wraps a ``run_batch`` with scripted
failures / hangs.
"""
from __future__ import annotations

import asyncio
import logging
import threading
import time
from typing import Callable, List, Optional, Sequence

from .batcher import ReplicaRouter

logger = logging.getLogger("mlsamd.watchdog")


class ReplicaWatchdog:
    def __init__(self, router: ReplicaRouter, stall_s: float = 30.0, max_failures: int = 3,
                 interval_s: float = 1.0, cooldown_s: float = 30.0,
                 probes: Optional[Sequence[Optional[Callable[[], bool]]]] = None,
                 on_change: Optional[Callable[[int, bool, str], None]] = None):
        self.router = router
        self.stall_s = float(stall_s)
        self.max_failures = int(max_failures)
        self.interval_s = float(interval_s)
        self.cooldown_s = float(cooldown_s)
        self.probes = list(probes or [])
        self.on_change = on_change
        self._drained_at: dict = {}
        self._task: Optional[asyncio.Task] = None
        self.events: List[dict] = []

    def check_once(self) -> None:
        now = time.perf_counter()
        for i, b in enumerate(self.router.batchers):
            reason = None
            if b.oldest_running_s > self.stall_s:
                reason = f"batch running {b.oldest_running_s:.1f}s > stall limit {self.stall_s:.1f}s"
            elif b.healthy and b.consecutive_failures >= self.max_failures:
                # (a replica already drained for failures keeps its stale count until probation)
                reason = f"{b.consecutive_failures} consecutive failed batches"
            elif i < len(self.probes) and self.probes[i] is not None:
                try:
                    ok = bool(self.probes[i]())
                except Exception as e:  # a probe that throws is a failed probe
                    ok = False
                    reason = f"health probe raised {type(e).__name__}: {e}"
                if not ok and reason is None:
                    reason = "health probe failed"
            if reason is not None:
                if b.healthy:
                    self._set(i, False, reason)
                    self._drained_at[i] = now
                continue
            if not b.healthy and b.unhealthy_reason is not None and "consecutive failed" in b.unhealthy_reason:
                if now - self._drained_at.get(i, now) >= self.cooldown_s:
                    b.consecutive_failures = self.max_failures - 1  # probation: one failure re-drains
                    self._set(i, True, "re-admitted on probation after cooldown")
            elif not b.healthy and b.unhealthy_reason is not None and "stall" in b.unhealthy_reason:
                self._set(i, True, "stuck batch finished")

    def _set(self, i: int, healthy: bool, reason: str) -> None:
        if healthy:
            self.router.mark_healthy(i)
            logger.warning("replica %d healthy again: %s", i, reason)
        else:
            self.router.mark_unhealthy(i, reason)
            logger.error("replica %d drained: %s", i, reason)
        self.events.append({"replica": i, "healthy": healthy, "reason": reason, "t": time.time()})
        if self.on_change is not None:
            try:
                self.on_change(i, healthy, reason)
            except Exception:
                pass

    async def _run(self) -> None:
        while True:
            try:
                self.check_once()
            except Exception:  # the watchdog itself must never die
                logger.exception("watchdog check failed")
            await asyncio.sleep(self.interval_s)

    def start(self) -> None:
        if self._task is None:
            self._task = asyncio.get_running_loop().create_task(self._run(), name="replica-watchdog")

    async def stop(self) -> None:
        if self._task is not None:
            self._task.cancel()
            try:
                await self._task
            except (asyncio.CancelledError, Exception):
                pass
            self._task = None


class FaultInjector:
    """Wraps ``run_batch`` for fault-injection tests: ``fail_batches`` = set of batch indices that
    raise, ``fail_after`` = every batch from that index on raises, ``hang_batches`` = indices
    that block for ``hang_s`` (or until :meth:`release`)."""

    def __init__(self, run_batch, fail_batches=(), fail_after: Optional[int] = None, hang_batches=(),
                 hang_s: float = 5.0):
        self.run_batch = run_batch
        self.fail_batches = set(fail_batches)
        self.fail_after = fail_after
        self.hang_batches = set(hang_batches)
        self.hang_s = hang_s
        self.calls = 0
        self._release = threading.Event()
        self._lock = threading.Lock()

    def release(self) -> None:
        self._release.set()

    def __call__(self, samples):
        with self._lock:
            i = self.calls
            self.calls += 1
        if i in self.hang_batches:
            self._release.wait(self.hang_s)
        if i in self.fail_batches or (self.fail_after is not None and i >= self.fail_after):
            raise RuntimeError(f"injected fault in batch {i}")
        return self.run_batch(samples)
