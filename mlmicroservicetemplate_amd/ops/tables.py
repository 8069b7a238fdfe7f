"""Measured per-shape dispatch tables (ops/tuned/*.json) and their lookups -- a served shape that misses a table is logged once per process."""
from __future__ import annotations

import functools
import json
import os
from typing import Dict, List, Optional, Tuple

import torch



_TUNED_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "tuned")


def load_blas_tuning(path: Optional[str] = None) -> bool:
    """Make hipBLASLt use the solutions PyTorch TunableOp measured fastest on MI355X for the shapes
    in ``tuned/tunableop_gfx950.csv`` (BERT FFN-up + GELU: 26.4 vs 30.1 us at 4-way concurrency,
    ``profiles/r1_bert_gemm_probe.jsonl``).  Lookup only -- tuning stays off, so nothing is timed or
    written at run time, and untuned shapes keep the library default.  ``MLS_BLAS_TUNING=0``
    disables it; ``MLS_BLAS_TUNING_FILE`` reads another table (A/B).  Returns whether it loaded."""
    if os.environ.get("MLS_BLAS_TUNING", "1") == "0" or not torch.cuda.is_available():
        return False
    from torch.cuda import tunable

    tunable.enable(True)
    tunable.tuning_enable(False)
    path = path or os.environ.get("MLS_BLAS_TUNING_FILE") or os.path.join(_TUNED_DIR, "tunableop_gfx950.csv")
    ok = bool(tunable.read_file(path))
    if not ok:
        tunable.enable(False)
    return ok


@functools.lru_cache(maxsize=None)
def gemm_plan() -> Dict[Tuple[int, int, int], Tuple[int, int]]:
    """Measured per-shape choices for :func:`linear` (``tuned/gemm_plan_gfx950.json``): exact
    ``(M, N, K)`` -> ``(cfg, splitk)`` of the native kernel, cfg 0 = its own heuristic pick.  ``MLS_GEMM_PLAN=0``
    disables it."""
    if os.environ.get("MLS_GEMM_PLAN", "1") == "0":
        return {}
    with open(os.path.join(_TUNED_DIR, "gemm_plan_gfx950.json")) as f:
        doc = json.load(f)
    return {(e["M"], e["N"], e["K"]): (int(e["plan"][0]), int(e["plan"][1])) for e in doc["entries"]}


_TABLE_MISSES: set = set()


_ops_log = __import__("logging").getLogger("mlsamd.ops")


def _note_miss(table: str, M: int, N: int, K: int) -> None:
    """Log ONCE per process and projection (N, K) when a served GEMM shape is not in a tuning table
    (it then runs the kernel's heuristic tile, which can be far off the measured best)."""
    # one line per projection (N, K) and table: a prefill sees a new M for nearly every batch
    key = (table, N, K)
    if key in _TABLE_MISSES:
        return
    _TABLE_MISSES.add(key)
    _ops_log.warning("GEMM shape M=%d N=%d K=%d is not in %s: heuristic config (tune it with "
                     "tools/gemm_tile_probe.py / ops.autotune; further misses of this N x K not logged)",
                     M, N, K, table)


def tile_cfg_for(M: int, N: int, K: int) -> Tuple[int, int]:
    """gemm_tile (config, K splits) for a shape: measured choices first (``tuned/gemm_tile_gfx950.json``),
    else the kernel's own pick (largest tile that still fills the chip), no split -- logged once."""
    impl, cfg, sk = tile_route_for(M, N, K)
    return (cfg, sk) if impl == "tile" else (0, 1)


def tile_route_for(M: int, N: int, K: int) -> Tuple[str, int, int]:
    """``(impl, cfg, splitk)`` of a large-M projection: impl "tile" (gemm_tile) or "conv" (the conv_gemm
    kernel, for short-M shapes whose tiles cannot fill the chip) -- the table's per-shape winner; a
    miss runs the tile kernel's own pick (logged once).  The shipped table has no library route
    (tests/test_gemm_tables.py); :func:`ops.linear` runs any other kind on the tile kernel."""
    e = gemm_tile_plan().get((M, N, K))
    if e is not None:
        return e
    for lo, hi, route in gemm_tile_ranges().get((N, K), ()):
        if lo <= M <= hi:
            return route
    _note_miss("gemm_tile_gfx950.json", M, N, K)
    return ("tile", 0, 1)


def small_m_plan_for(M: int, N: int, K: int) -> Optional[Tuple[int, int]]:
    """The measured (cfg, splitk) of a small-M projection (``tuned/gemm_plan_gfx950.json``), or
    None (logged once: the conv_gemm heuristic runs it)."""
    plan = gemm_plan()
    e = plan.get((M, N, K))
    if e is None and plan:
        _note_miss("gemm_plan_gfx950.json", M, N, K)
    return e


@functools.lru_cache(maxsize=None)
def gemm_tile_plan() -> Dict[Tuple[int, int, int], Tuple[int, int]]:
    path = os.environ.get("MLS_GEMM_TILE_TABLE") or os.path.join(_TUNED_DIR, "gemm_tile_gfx950.json")
    if os.environ.get("MLS_GEMM_PLAN", "1") == "0" or not os.path.exists(path):
        return {}
    with open(path) as f:
        doc = json.load(f)
    return {(e["M"], e["N"], e["K"]): (e.get("impl", "tile"), int(e.get("cfg", 0)), int(e.get("splitk", 1)))
            for e in doc["entries"] if "M" in e}


@functools.lru_cache(maxsize=None)
def gemm_tile_ranges() -> Dict[Tuple[int, int], List[Tuple[int, int, Tuple[str, int, int]]]]:
    """Row-range entries of the tile table (``"M_min"`` / ``"M_max"`` instead of ``"M"``): a projection
    (N, K) whose winner does not change over a range of token counts -- a prefill sees a new M for
    nearly every batch.  Exact entries take precedence."""
    path = os.environ.get("MLS_GEMM_TILE_TABLE") or os.path.join(_TUNED_DIR, "gemm_tile_gfx950.json")
    if os.environ.get("MLS_GEMM_PLAN", "1") == "0" or not os.path.exists(path):
        return {}
    with open(path) as f:
        doc = json.load(f)
    out: Dict[Tuple[int, int], list] = {}
    for e in doc["entries"]:
        if "M_min" in e:
            out.setdefault((e["N"], e["K"]), []).append(
                (int(e["M_min"]), int(e.get("M_max", 1 << 30)),
                 (e.get("impl", "tile"), int(e.get("cfg", 0)), int(e.get("splitk", 1)))))
    return out
