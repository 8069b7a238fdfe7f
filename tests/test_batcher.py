"""Dynamic micro-batcher and replica router on a pure-asyncio fake executor (no GPU)."""
import asyncio
import threading
import time

import pytest

from mlmicroservicetemplate_amd.scheduler.batcher import DynamicBatcher, QueueFull, ReplicaRouter


def run(coro):
    return asyncio.run(coro)


def test_max_batch_flush_and_order():
    sizes = []

    def rb(samples):
        sizes.append(len(samples))
        return [s * 2 for s in samples]

    async def main():
        b = DynamicBatcher(rb, max_batch=4, max_wait_us=10_000_000, inflight=1)
        await b.start()
        res = await asyncio.gather(*[b.submit(i) for i in range(8)])
        await b.stop()
        return res

    assert run(main()) == [i * 2 for i in range(8)]
    assert sizes == [4, 4]  # flushed by size, never waited for the 10 s deadline


def test_deadline_flush():
    async def main():
        b = DynamicBatcher(lambda s: s, max_batch=64, max_wait_us=20_000)
        await b.start()
        t0 = time.perf_counter()
        r = await b.submit("x")
        dt = time.perf_counter() - t0
        await b.stop()
        return r, dt

    r, dt = run(main())
    assert r == "x" and 0.015 <= dt < 0.5


def test_error_isolation_and_batch_failure():
    def rb(samples):
        if "boom" in samples:
            raise RuntimeError("batch failed")
        return [ValueError("bad row") if s == "bad" else s for s in samples]

    async def main():
        b = DynamicBatcher(rb, max_batch=3, max_wait_us=5_000)
        await b.start()
        r = await asyncio.gather(b.submit("a"), b.submit("bad"), b.submit("c"), return_exceptions=True)
        r2 = await asyncio.gather(b.submit("boom"), return_exceptions=True)
        r3 = await b.submit("after")
        await b.stop()
        return r, r2, r3, b.stats()

    r, r2, r3, st = run(main())
    assert r[0] == "a" and isinstance(r[1], ValueError) and r[2] == "c"
    assert isinstance(r2[0], RuntimeError)
    assert r3 == "after"
    assert st["failed"] == 2


def test_backpressure():
    gate = threading.Event()

    def rb(samples):
        gate.wait(2)
        return samples

    async def main():
        b = DynamicBatcher(rb, max_batch=1, max_wait_us=0, max_queue=2, inflight=1)
        await b.start()
        futs = [b.submit_nowait(i) for i in range(2)]
        await asyncio.sleep(0.05)  # first one dispatched, queue has room again
        futs.append(b.submit_nowait(2))  # queue: [1, 2] -> full
        with pytest.raises(QueueFull):
            b.submit_nowait(3)
        gate.set()
        res = await asyncio.gather(*futs)
        await b.stop()
        return res, b.rejected

    res, rej = run(main())
    assert res == [0, 1, 2] and rej == 1


def test_inflight_concurrency():
    active = []
    peak = [0]
    lock = threading.Lock()

    def rb(samples):
        with lock:
            active.append(1)
            peak[0] = max(peak[0], len(active))
        time.sleep(0.05)
        with lock:
            active.pop()
        return samples

    async def main():
        b = DynamicBatcher(rb, max_batch=2, max_wait_us=1000, inflight=3)
        await b.start()
        await asyncio.gather(*[b.submit(i) for i in range(12)])
        await b.stop()

    run(main())
    assert peak[0] == 3


def test_cancelled_requests_are_dropped():
    seen = []

    def rb(samples):
        seen.extend(samples)
        return samples

    async def main():
        b = DynamicBatcher(rb, max_batch=8, max_wait_us=30_000)
        await b.start()
        f1 = b.submit_nowait("keep")
        f2 = b.submit_nowait("cancel")
        f2.cancel()
        await f1
        await b.stop()

    run(main())
    assert seen == ["keep"]


def test_router_least_loaded_and_unhealthy_drain():
    calls = {0: 0, 1: 0}

    def mk(i):
        def rb(samples):
            calls[i] += len(samples)
            time.sleep(0.01)
            return [i] * len(samples)

        return rb

    async def main():
        r = ReplicaRouter([DynamicBatcher(mk(0), 4, 1000), DynamicBatcher(mk(1), 4, 1000)])
        await r.start()
        out = await asyncio.gather(*[r.submit(k) for k in range(40)])
        r.mark_unhealthy(0)
        out2 = await asyncio.gather(*[r.submit(k) for k in range(8)])
        await r.stop()
        return out, out2

    out, out2 = run(main())
    assert set(out) == {0, 1} and calls[0] > 5 and calls[1] > 5
    assert set(out2) == {1}
