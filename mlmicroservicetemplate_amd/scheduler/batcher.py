"""Async dynamic micro-batcher (T3 / P1 of SURVEY.md) and least-loaded replica router (P2).

The reference runs ``predict`` inline on the event loop, one request at a time
(reference ``src/server/main.py:135``) -- every concurrent request waits for the previous
one.  Here each request is ``await batcher.submit(sample)``: samples accumulate until
``max_batch`` are queued or the oldest has waited ``max_wait_us``, then the batch is handed
to ``run_batch`` on a worker thread (so the event loop never blocks) and every request's
future is resolved with its own row.

Design points:
  * one wake-up per batch, not per request: ``submit`` appends to a deque and only signals
    the collector when the deque becomes non-empty or reaches ``max_batch``;
  * ``inflight`` batches may execute concurrently per replica (the GPU engine pipelines
    H2D / graph replay / D2H across them);
  * per-request error isolation: ``run_batch`` may return an ``Exception`` instance in a
    row's slot to fail just that request; a raised exception fails the whole batch;
  * admission control: more than ``max_queue`` waiting requests -> :class:`QueueFull`
    (HTTP 503) instead of unbounded latency;
  * cancelled requests (client went away) stop counting at once: ``queue_depth``, ``load`` and
    ``max_queue`` admission count only live queued futures (a set maintained by a done-callback),
    and the cancelled entries are swept from the deque when the next batch is formed.
"""
from __future__ import annotations

import asyncio
import collections
import concurrent.futures as cf
import logging
import threading
import time
from typing import Any, Callable, Deque, List, Optional, Sequence, Tuple

from ..utils import tracing

logger = logging.getLogger("mlsamd.batcher")

RunBatch = Callable[[List[Any]], Sequence[Any]]


class QueueFull(Exception):
    """Admission control rejected the request."""


class BatcherClosed(Exception):
    pass


class DynamicBatcher:
    def __init__(
        self,
        run_batch: RunBatch,
        max_batch: int = 32,
        max_wait_us: int = 2000,
        max_queue: int = 4096,
        inflight: int = 2,
        name: str = "batcher",
        executor: Optional[cf.Executor] = None,
        on_batch: Optional[Callable[[int, float], None]] = None,
    ):
        if max_batch < 1:
            raise ValueError("max_batch must be >= 1")
        self.run_batch = run_batch
        self.max_batch = max_batch
        self.max_wait = max_wait_us / 1e6
        self.max_queue = max_queue
        self.inflight = max(1, inflight)
        self.name = name
        self._own_executor = executor is None
        self._executor = executor or cf.ThreadPoolExecutor(self.inflight, thread_name_prefix=f"{name}-exec")
        self._q: Deque[Tuple[Any, asyncio.Future, float]] = collections.deque()
        # futures queued and not cancelled: what queue_depth / load / admission count (the deque
        # may still hold cancelled entries until the collector sweeps them in _take)
        self._queued: set = set()
        self._wake: Optional[asyncio.Event] = None
        self._full: Optional[asyncio.Event] = None
        self._sem: Optional[asyncio.Semaphore] = None
        self._task: Optional[asyncio.Task] = None
        self._loop: Optional[asyncio.AbstractEventLoop] = None
        self._closed = False
        self._inflight_now = 0
        self.on_batch = on_batch
        self.healthy = True
        self.unhealthy_reason: Optional[str] = None
        # liveness signals read by the watchdog (scheduler.watchdog)
        self._running: dict = {}  # batch id -> dispatch time
        self._next_id = 0
        self.consecutive_failures = 0
        self.last_success = time.perf_counter()
        # stats
        self.batches = 0
        self.requests = 0
        self.failed = 0
        self.rejected = 0
        self.batch_sizes: collections.Counter = collections.Counter()

    # ----------------------------------------------------------------- lifecycle
    async def start(self) -> None:
        if self._task is not None:
            return
        self._loop = asyncio.get_running_loop()
        self._wake = asyncio.Event()
        self._full = asyncio.Event()
        self._sem = asyncio.Semaphore(self.inflight)
        self._task = asyncio.create_task(self._collector(), name=f"{self.name}-collector")

    async def stop(self, drain: bool = True) -> None:
        self._closed = True
        if self._task is not None:
            if drain:
                # let queued requests run
                while self._q or self._inflight_now:
                    if self._wake is not None:
                        self._wake.set()
                    await asyncio.sleep(0.001)
            self._task.cancel()
            try:
                await self._task
            except (asyncio.CancelledError, Exception):
                pass
            self._task = None
        while self._q:
            _s, fut, _t = self._q.popleft()
            self._queued.discard(fut)
            if not fut.done():
                fut.set_exception(BatcherClosed(f"{self.name} stopped"))
        if self._own_executor:
            self._executor.shutdown(wait=False)

    # ----------------------------------------------------------------- API
    @property
    def queue_depth(self) -> int:
        return len(self._queued)

    @property
    def load(self) -> int:
        """Outstanding requests (queued + executing) -- the router's least-loaded key."""
        return len(self._queued) + self._inflight_now * self.max_batch

    def _on_queued_done(self, fut: "asyncio.Future") -> None:
        # runs on the loop when a queued future completes; only a cancellation can complete it
        # while it is still queued (results are set after _take removed it from the set)
        if fut in self._queued:
            self._queued.discard(fut)
            if not self._queued:
                # nothing live is waiting: let the collector sweep the cancelled entries now
                if self._wake is not None:
                    self._wake.set()

    def _enqueue(self, item) -> None:
        self._q.append(item)
        fut = item[1]
        if fut not in self._queued and not fut.done():
            self._queued.add(fut)
            fut.add_done_callback(self._on_queued_done)

    def submit_nowait(self, sample: Any) -> "asyncio.Future":
        if self._closed:
            raise BatcherClosed(f"{self.name} is stopped")
        if self._task is None:
            raise RuntimeError("batcher not started")
        if len(self._queued) >= self.max_queue:
            self.rejected += 1
            raise QueueFull(f"{self.name}: {len(self._queued)} requests queued")
        fut = self._loop.create_future()
        self._enqueue((sample, fut, time.perf_counter()))
        n = len(self._queued)
        if n == 1:
            self._wake.set()
        if n >= self.max_batch:
            self._full.set()
        return fut

    async def submit(self, sample: Any, timeout: Optional[float] = None) -> Any:
        fut = self.submit_nowait(sample)
        if timeout is None:
            return await fut
        return await asyncio.wait_for(fut, timeout)

    def evict_queued(self) -> List[Tuple[Any, "asyncio.Future", float]]:
        """Remove and return every queued (not yet dispatched) request -- a drained replica's
        backlog, which the router hands to healthy replicas."""
        items = [it for it in self._q if not it[1].done()]
        self._q.clear()
        self._queued.clear()
        if self._full is not None:
            self._full.clear()
        return items

    def adopt(self, items) -> None:
        """Append requests evicted from another replica (their futures keep their waiters)."""
        for it in items:
            self._enqueue(it)
        if self._queued and self._wake is not None:
            self._wake.set()
            if len(self._queued) >= self.max_batch:
                self._full.set()

    # ----------------------------------------------------------------- internals
    def _take(self) -> List[Tuple[Any, asyncio.Future, float]]:
        batch = []
        while self._q and len(batch) < self.max_batch:
            item = self._q.popleft()
            self._queued.discard(item[1])
            if item[1].done():  # cancelled while queued
                continue
            batch.append(item)
        while self._q and self._q[0][1].done():  # sweep cancelled heads so the deadline is a live one
            self._queued.discard(self._q.popleft()[1])
        if len(self._queued) < self.max_batch:
            self._full.clear()
        if not self._q:
            self._wake.clear()
        return batch

    async def _collector(self) -> None:
        while True:
            await self._wake.wait()
            while self._q and self._q[0][1].done():  # cancelled while queued
                self._queued.discard(self._q.popleft()[1])
            if not self._q:
                self._wake.clear()
                continue
            # wait until full or until the oldest request's deadline
            oldest = self._q[0][2]
            remaining = oldest + self.max_wait - time.perf_counter()
            if len(self._queued) < self.max_batch and remaining > 0 and not self._closed:
                try:
                    await asyncio.wait_for(self._full.wait(), remaining)
                except asyncio.TimeoutError:
                    pass
            await self._sem.acquire()
            with tracing.range("batch.assemble"):
                batch = self._take()
            if not batch:
                self._sem.release()
                continue
            self._inflight_now += 1
            self._dispatch(batch)

    @property
    def oldest_running_s(self) -> float:
        """Age of the longest-running dispatched batch (0 if none) -- a hung GPU worker shows here."""
        if not self._running:
            return 0.0
        return time.perf_counter() - min(self._running.values())

    def _dispatch(self, batch) -> None:
        samples = [b[0] for b in batch]
        t0 = time.perf_counter()
        bid = self._next_id
        self._next_id += 1
        self._running[bid] = t0
        cfut = self._executor.submit(self._run_traced, samples)

        def done(f: cf.Future) -> None:
            try:
                self._loop.call_soon_threadsafe(self._resolve, batch, f, t0, bid)
            except RuntimeError:  # loop already closed (shutdown raced a running batch)
                pass

        cfut.add_done_callback(done)

    def _run_traced(self, samples):
        with tracing.range("batch.run"):
            return self.run_batch(samples)

    def _resolve(self, batch, f: cf.Future, t0: float, bid: int = -1) -> None:
        self._running.pop(bid, None)
        self._inflight_now -= 1
        self._sem.release()
        n = len(batch)
        self.batches += 1
        self.requests += n
        self.batch_sizes[n] += 1
        if self.on_batch is not None:
            try:
                self.on_batch(n, time.perf_counter() - t0)
            except Exception:  # metrics must never break serving
                pass
        exc = f.exception()
        if exc is None:
            self.consecutive_failures = 0
            self.last_success = time.perf_counter()
        else:
            self.consecutive_failures += 1
        if exc is not None:
            self.failed += n
            logger.warning("%s: batch of %d failed: %s", self.name, n, exc)
            for _s, fut, _t in batch:
                if not fut.done():
                    fut.set_exception(exc)
            return
        results = f.result()
        if len(results) != n:
            err = RuntimeError(f"run_batch returned {len(results)} results for {n} samples")
            for _s, fut, _t in batch:
                if not fut.done():
                    fut.set_exception(err)
            return
        for (_s, fut, _t), r in zip(batch, results):
            if fut.done():
                continue
            if isinstance(r, BaseException):
                self.failed += 1
                fut.set_exception(r)
            else:
                fut.set_result(r)

    def stats(self) -> dict:
        return {
            "name": self.name,
            "queue_depth": len(self._queued),
            "inflight": self._inflight_now,
            "batches": self.batches,
            "requests": self.requests,
            "failed": self.failed,
            "rejected": self.rejected,
            "mean_batch": (self.requests / self.batches) if self.batches else 0.0,
            "healthy": self.healthy,
            "unhealthy_reason": self.unhealthy_reason,
            "consecutive_failures": self.consecutive_failures,
            "oldest_running_s": round(self.oldest_running_s, 3),
        }


class ReplicaRouter:
    """Least-loaded dispatch over per-replica batchers (one per GPU).  A replica marked
    unhealthy (its worker died) is drained: no new requests are routed to it."""

    def __init__(self, batchers: Sequence[DynamicBatcher]):
        if not batchers:
            raise ValueError("need at least one replica")
        self.batchers = list(batchers)
        self._rr = 0
        self._lock = threading.Lock()

    async def start(self) -> None:
        for b in self.batchers:
            await b.start()

    async def stop(self) -> None:
        for b in self.batchers:
            await b.stop()

    def pick(self) -> DynamicBatcher:
        live = [b for b in self.batchers if b.healthy]
        if not live:
            raise QueueFull("no healthy replica")
        # least loaded; round-robin among ties so idle replicas share the work
        self._rr = (self._rr + 1) % len(live)
        rotated = live[self._rr:] + live[: self._rr]
        return min(rotated, key=lambda b: b.load)

    async def submit(self, sample: Any, timeout: Optional[float] = None) -> Any:
        return await self.pick().submit(sample, timeout)

    def mark_unhealthy(self, idx: int, reason: str = "marked unhealthy") -> None:
        """Drain replica ``idx``: no new requests, and its queued backlog moves to the healthy
        replicas (or fails with QueueFull when none is left)."""
        b = self.batchers[idx]
        b.healthy = False
        b.unhealthy_reason = reason
        backlog = b.evict_queued()
        live = [x for x in self.batchers if x.healthy]
        for j, item in enumerate(backlog):
            if live:
                live[j % len(live)].adopt([item])
            elif not item[1].done():
                item[1].set_exception(QueueFull(f"replica {idx} drained ({reason}); no healthy replica"))

    def mark_healthy(self, idx: int) -> None:
        self.batchers[idx].healthy = True
        self.batchers[idx].unhealthy_reason = None

    @property
    def healthy_count(self) -> int:
        return sum(1 for b in self.batchers if b.healthy)

    def stats(self) -> List[dict]:
        return [b.stats() for b in self.batchers]
