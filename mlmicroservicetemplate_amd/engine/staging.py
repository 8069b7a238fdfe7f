"""Host staging copies for :class:`~.worker.GpuEngine` (request arrays -> one pinned slot).

Wraps the C++ pool in ``csrc/staging.cpp`` (built in-tree by ``frontend/build.py``): persistent
copy threads, GIL released, the calling thread copies too, 256 KiB chunks from an atomic cursor.
``MLS_STAGE_THREADS`` sets the number of pool threads (default 4, plus the caller; with several
ranks per node the budget ``parallel.affinity.bind_to_gpu`` derives from the rank's CPU share);
``MLS_NATIVE_STAGING=0`` selects the Python thread-pool path (kept for A/B and for hosts where
the module has not been built).  A serving process never compiles: a missing module, or one whose
build stamp does not match the current sources, falls back to the Python path with a warning
(build it with ``python -m mlmicroservicetemplate_amd build``).
"""
from __future__ import annotations

import importlib.util
import logging
import os
from concurrent.futures import ThreadPoolExecutor
from typing import Optional, Sequence

import numpy as np

logger = logging.getLogger("mlsamd.engine")

_mod = None
_mod_err: Optional[str] = None


def _load():
    global _mod, _mod_err
    if _mod is not None or _mod_err is not None:
        return _mod
    from ..frontend import build as fbuild

    path = fbuild.staging_path()
    try:
        if not os.path.exists(path):
            raise FileNotFoundError(f"{path} is not built")
        if not fbuild.staging_current():
            raise RuntimeError(f"{path} is stale (built from other staging sources); rebuild it")
        spec = importlib.util.spec_from_file_location("_staging", path)
        mod = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(mod)
        _mod = mod
    except Exception as e:  # noqa: BLE001 -- host-side fallback, logged
        _mod_err = f"{type(e).__name__}: {e}"
        logger.warning("native staging unavailable (%s); using the Python copy threads", _mod_err)
    return _mod


class HostStager:
    """Copies ``n`` per-request arrays of ``sample_bytes`` each into a pinned buffer."""

    def __init__(self, threads: Optional[int] = None, name: str = "engine", native: Optional[bool] = None):
        if threads is None:
            env = os.environ.get("MLS_STAGE_THREADS")
            if env is not None:
                threads = int(env)
            else:  # multi-rank: this rank's share of its NUMA node's CPUs (parallel/affinity.py)
                from ..parallel.affinity import STAGE_THREADS_CAP, stage_threads_hint

                threads = stage_threads_hint() or STAGE_THREADS_CAP
        if native is None:
            native = os.environ.get("MLS_NATIVE_STAGING", "1") != "0"
        self.threads = max(0, int(threads))
        self._native = None
        self._pool = None
        if native:
            mod = _load()
            if mod is not None:
                self._native = mod.Stager(self.threads)
        if self._native is None and self.threads > 1:
            self._pool = ThreadPoolExecutor(max_workers=self.threads, thread_name_prefix=f"{name}-stage")

    @property
    def native(self) -> bool:
        return self._native is not None

    def gather(self, dst: np.ndarray, samples: Sequence[np.ndarray]) -> None:
        """``dst[i] = samples[i]`` for every request (``dst`` a pinned ``[max_b, ...]`` view)."""
        n = len(samples)
        if n > dst.shape[0]:
            raise ValueError(f"{n} samples do not fit a staging buffer of {dst.shape[0]} rows")
        if not dst.flags.c_contiguous:
            raise ValueError("staging destination must be C-contiguous")
        if self._native is not None and n > 0:
            each = dst[0].nbytes
            srcs = [s if (isinstance(s, np.ndarray) and s.dtype == dst.dtype and s.flags.c_contiguous)
                    else np.ascontiguousarray(s, dtype=dst.dtype) for s in samples]
            for s in srcs:
                if s.nbytes != each:
                    raise ValueError(f"sample of shape {s.shape} does not fit the slot row {dst.shape[1:]}")
            self._native.gather(dst.ctypes.data, srcs, each)
            return
        if self._pool is not None and n >= 8:
            step = -(-n // self._pool._max_workers)

            def _copy(lo):
                for i in range(lo, min(n, lo + step)):
                    dst[i] = samples[i]

            for f in [self._pool.submit(_copy, lo) for lo in range(0, n, step)]:
                f.result()
            return
        for i, s in enumerate(samples):
            dst[i] = s
