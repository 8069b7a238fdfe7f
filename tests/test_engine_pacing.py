"""Launch pacing of the GPU engine (engine/worker.py:_pace_launch / _note_done), host logic only:
no wait at light load, a Little's-law gap (latency EWMA / inflight) near saturation."""
import queue
import threading
import time

from mlmicroservicetemplate_amd.engine.worker import GpuEngine


class _T:
    def __init__(self, t_submit):
        self.t_submit = t_submit


def _engine(inflight=5, pace=1.0, busy=4):
    e = object.__new__(GpuEngine)  # no device: only the pacing state
    e.inflight = inflight
    e._pace, e._fixed_gap_s = pace, 0.0
    e._last_launch, e._lat_s, e._lat_n = 0.0, 0.0, 0
    e._pace_lock = threading.Lock()
    e._pace_min_busy = max(1, inflight - 2)
    e._free = queue.Queue()
    for _ in range(inflight - busy - 1):  # this launch's slot is already taken
        e._free.put(object())
    return e


def test_latency_ewma_sets_the_gap():
    e = _engine()
    for _ in range(e.inflight):  # the first pipeline turn is ignored (cold graphs)
        e._note_done(_T(time.perf_counter() - 0.5))
    assert e._lat_s == 0.0
    e._note_done(_T(time.perf_counter() - 0.010))
    assert abs(e._lat_s - 0.010) < 1e-3
    for _ in range(50):
        e._note_done(_T(time.perf_counter() - 0.005))
    assert 0.0045 < e._lat_s < 0.0060  # converges to the new latency
    e._note_done(_T(time.perf_counter() - 1.0))  # one stall moves it by at most 10 % of 2x
    assert e._lat_s < 0.0065


def test_waits_near_saturation():
    e = _engine(busy=4)
    e._lat_s = 0.010  # -> gap 2 ms at inflight 5
    e._last_launch = time.perf_counter()
    t0 = time.perf_counter()
    e._pace_launch()
    assert time.perf_counter() - t0 >= 0.0019


def test_no_wait_at_light_load_or_when_disabled():
    for e in (_engine(busy=1), _engine(busy=4, pace=0.0)):
        e._lat_s = 0.010
        e._last_launch = time.perf_counter()
        t0 = time.perf_counter()
        e._pace_launch()
        assert time.perf_counter() - t0 < 0.0015
