"""Race detection for the dynamic micro-batcher and replica router.

The reference shares its readiness flags across threads unprotected (`dependency.py:6-20`,
`main.py:80,90`); here the equivalent hand-off is batcher queue -> executor thread -> event loop,
so these tests hammer it with many producers, random cancellations, per-row errors and runner
threads that finish out of order, with the event loop in asyncio DEBUG mode: debug mode raises
on any non-thread-safe loop call made from a runner thread (a missed ``call_soon_threadsafe``)
and reports never-retrieved exceptions.  Invariants checked on every run:

* every surviving request gets exactly the result computed from its own input (no cross-wiring
  between futures and batch rows);
* no sample is executed twice, no batch exceeds ``max_batch``, at most ``inflight`` batches run;
* the counters in ``stats()`` add up to what the runner saw.
"""
import asyncio
import logging
import random
import threading
import time

import pytest

from mlmicroservicetemplate_amd.scheduler.batcher import DynamicBatcher, ReplicaRouter


class _Runner:
    """Thread-executed batch function that records what it saw."""

    def __init__(self, max_batch: int, seed: int):
        self.lock = threading.Lock()
        self.seen = []
        self.active = 0
        self.peak = 0
        self.max_batch = max_batch
        self.too_big = 0
        self.rng = random.Random(seed)

    def __call__(self, samples):
        with self.lock:
            self.active += 1
            self.peak = max(self.peak, self.active)
            self.seen.extend(samples)
            if len(samples) > self.max_batch:
                self.too_big += 1
            delay = self.rng.random() * 0.003
        time.sleep(delay)  # batches finish out of order
        with self.lock:
            self.active -= 1
        return [ValueError(f"bad {s}") if s % 97 == 13 else s * 3 + 1 for s in samples]


async def _producer(b, ids, rng, results, cancelled):
    for i in ids:
        fut = b.submit_nowait(i)
        if rng.random() < 0.1:
            fut.cancel()
            cancelled.add(i)
            continue
        results[i] = fut
        if rng.random() < 0.3:
            await asyncio.sleep(0)


def _check(results, cancelled, runner, n):
    for i, fut in results.items():
        if i % 97 == 13:
            assert isinstance(fut.exception(), ValueError) and str(fut.exception()) == f"bad {i}"
        else:
            assert fut.result() == i * 3 + 1, f"request {i} got {fut.result()}"
    assert len(runner.seen) == len(set(runner.seen)), "a sample was executed twice"
    assert set(results) <= set(runner.seen)
    assert set(results) | cancelled == set(range(n))
    assert runner.too_big == 0


@pytest.mark.parametrize("seed", [0, 1, 2])
@pytest.mark.parametrize("max_batch,inflight", [(1, 1), (7, 2), (32, 4)])
def test_batcher_stress_debug_loop(seed, max_batch, inflight, caplog):
    n = 1500
    runner = _Runner(max_batch, seed)

    async def main():
        loop = asyncio.get_running_loop()
        loop.slow_callback_duration = 1.0  # only report truly blocking callbacks
        b = DynamicBatcher(runner, max_batch=max_batch, max_wait_us=200, inflight=inflight, max_queue=n + 1)
        await b.start()
        rng = random.Random(seed)
        results, cancelled = {}, set()
        chunks = [list(range(k, n, 8)) for k in range(8)]
        await asyncio.gather(*[_producer(b, c, random.Random(rng.random()), results, cancelled) for c in chunks])
        await asyncio.gather(*results.values(), return_exceptions=True)
        st = b.stats()
        await b.stop()
        return results, cancelled, st

    with caplog.at_level(logging.ERROR, logger="asyncio"):
        results, cancelled, st = asyncio.run(main(), debug=True)
    _check(results, cancelled, runner, n)
    assert runner.peak <= inflight
    assert st["requests"] == len(runner.seen)
    assert st["queue_depth"] == 0 and st["inflight"] == 0
    # debug mode logs un-retrieved exceptions / thread-unsafe calls through the asyncio logger
    assert not [r for r in caplog.records if r.name == "asyncio"], [r.getMessage() for r in caplog.records]


def test_router_stress_debug_loop(caplog):
    n, reps = 1200, 3
    runners = [_Runner(8, 100 + r) for r in range(reps)]

    async def main():
        bs = [DynamicBatcher(runners[r], max_batch=8, max_wait_us=300, inflight=2, name=f"r{r}", max_queue=n + 1)
              for r in range(reps)]
        router = ReplicaRouter(bs)
        await router.start()
        rng = random.Random(7)

        async def one(i):
            if rng.random() < 0.05:
                await asyncio.sleep(0)
            return await router.submit(i)

        # drain replica 1 half-way through: nothing new may be routed to it afterwards
        first = [asyncio.ensure_future(one(i)) for i in range(n // 2)]
        await asyncio.sleep(0)
        router.mark_unhealthy(1, "test drain")
        seen_before = len(runners[1].seen)
        second = [asyncio.ensure_future(one(i)) for i in range(n // 2, n)]
        res = await asyncio.gather(*first, *second, return_exceptions=True)
        await router.stop()
        return res, seen_before

    with caplog.at_level(logging.ERROR, logger="asyncio"):
        res, seen_before = asyncio.run(main(), debug=True)
    for i, r in enumerate(res):
        if i % 97 == 13:
            assert isinstance(r, ValueError)
        else:
            assert r == i * 3 + 1
    everything = [s for rn in runners for s in rn.seen]
    assert sorted(everything) == list(range(n)), "lost or duplicated requests across replicas"
    assert all(s < n // 2 for s in runners[1].seen[seen_before:]), "drained replica received new work"
    assert not [r for r in caplog.records if r.name == "asyncio"]


def test_cancelled_requests_leave_the_accounting_at_once():
    """A cancelled queued request stops counting toward queue_depth / load / max_queue admission
    immediately (not only when the collector next forms a batch)."""
    from mlmicroservicetemplate_amd.scheduler.batcher import QueueFull

    gate = threading.Event()

    def run(samples):
        gate.wait(5)
        return samples

    async def main():
        b = DynamicBatcher(run, max_batch=3, max_wait_us=10_000_000, inflight=1, max_queue=3)
        await b.start()
        futs = [b.submit_nowait(i) for i in range(3)]
        assert b.queue_depth == 3
        with pytest.raises(QueueFull):
            b.submit_nowait(99)
        for f in futs:
            f.cancel()
        await asyncio.sleep(0)  # done-callbacks run on the next loop iteration
        assert b.queue_depth == 0 and b.load == 0 and b.stats()["queue_depth"] == 0
        live = [b.submit_nowait(10 + i) for i in range(3)]  # admission capacity is back
        assert b.queue_depth == 3  # and the 3 live requests fill one batch
        gate.set()
        res = await asyncio.gather(*live)
        assert res == [10, 11, 12]
        assert b.queue_depth == 0
        await b.stop()

    asyncio.run(main(), debug=True)
