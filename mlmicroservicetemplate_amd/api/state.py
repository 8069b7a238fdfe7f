"""Process-wide service state (reference ``src/server/dependency.py``).

The reference keeps readiness in a pydantic-v1 ``BaseSettings`` singleton
(``dependency.py:6-10``), the discovery flags ``connected``/``shutdown`` as bare module
globals (``:17-18``) and a ``ThreadPoolExecutor(10)`` (``:19``).  Here the same state lives in
one object owned by the app, with an ``Event`` for shutdown (so sleeping threads wake
immediately instead of polling 1 s slices) and an explicit ``init_error`` so a failing
``init()`` is reported by ``/status`` instead of being swallowed in a Future (C6 defect).
"""
from __future__ import annotations

import threading
import time
from concurrent.futures import ThreadPoolExecutor
from dataclasses import dataclass, field
from typing import Optional


class PredictionException(Exception):
    """Raised when the model is not ready; mapped to HTTP 503 (reference ``main.py:41-49``)."""

    def __init__(self, detail: str = "Model is not ready to receive predictions.") -> None:
        super().__init__(detail)
        self.detail = detail


class OverloadedException(Exception):
    """Admission control rejected the request (queue full); mapped to HTTP 503 + Retry-After."""


@dataclass
class ServiceState:
    pool_workers: int = 10
    ready_to_predict: bool = False
    connected: bool = False
    init_error: Optional[str] = None
    init_started_at: Optional[float] = None
    init_finished_at: Optional[float] = None
    shutdown: threading.Event = field(default_factory=threading.Event)
    pool: ThreadPoolExecutor = None  # type: ignore[assignment]
    registrations: int = 0
    last_register_error: Optional[str] = None

    def __post_init__(self) -> None:
        if self.pool is None:
            self.pool = ThreadPoolExecutor(self.pool_workers, thread_name_prefix="mlsamd-bg")

    def mark_init_started(self) -> None:
        self.init_started_at = time.time()

    def mark_ready(self) -> None:
        self.init_finished_at = time.time()
        self.init_error = None
        self.ready_to_predict = True

    def mark_failed(self, err: BaseException) -> None:
        self.init_finished_at = time.time()
        self.init_error = f"{type(err).__name__}: {err}"
        self.ready_to_predict = False

    def begin_shutdown(self, wait: bool = True) -> None:
        self.ready_to_predict = False
        self.shutdown.set()
        self.pool.shutdown(wait=wait)
