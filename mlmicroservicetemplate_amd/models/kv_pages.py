"""Paged KV cache bookkeeping (SURVEY.md §2.E.1 K13 "paged write", §5.7 paged allocator).

The fused decode-attention kernel walks a sequence's keys in splits of ``page_rows`` (64) rows,
so one page is exactly one split: a block reads ONE page-table entry and then the same contiguous
rows it read from a per-sequence cache.  The caches become page pools ``[pages, page_rows, Hkv,
D]`` per layer, shared by every sequence, and a sequence holds only the pages its prompt +
generation budget needs instead of a ``max_seq`` slab -- on 288 GB of HBM the pool is sized by
the tokens actually in flight, not by ``max_batch x max_seq``.

Page 0 is a scratch page that every unassigned table entry points at: idle decode slots (the
fixed-shape decode graph runs all ``max_batch`` rows) write their dummy token there, never into
a live sequence's page.
"""
from __future__ import annotations

from typing import Dict, List, Optional

import torch


class OutOfPages(RuntimeError):
    pass


class PageTable:
    """Host page allocator + the ``[max_batch, pages_per_seq]`` int32 table the kernels read.

    ``assign(slot, rows)`` gives a slot pages for ``rows`` cache rows (growing its list),
    ``release(slot)`` returns them; ``device_table()`` copies the host table into a static device
    buffer (the captured decode graphs read that same buffer, so it is refreshed in place)."""

    def __init__(self, num_pages: int, page_rows: int, max_batch: int, pages_per_seq: int, device="cpu"):
        if num_pages < 2:
            raise ValueError("need at least one scratch page and one data page")
        self.num_pages, self.page_rows = int(num_pages), int(page_rows)
        self.max_batch, self.pages_per_seq = int(max_batch), int(pages_per_seq)
        self.device = torch.device(device)
        self._free: List[int] = list(range(self.num_pages - 1, 0, -1))  # page 0 = scratch
        self._owned: Dict[int, List[int]] = {}
        pin = self.device.type == "cuda"
        self.host = torch.zeros(self.max_batch, self.pages_per_seq, dtype=torch.int32, pin_memory=pin)
        self.dev = torch.zeros(self.max_batch, self.pages_per_seq, dtype=torch.int32, device=self.device)
        self._dirty = False

    # ------------------------------------------------------------------ accounting
    @property
    def free_pages(self) -> int:
        return len(self._free)

    def pages_for(self, rows: int) -> int:
        return -(-int(rows) // self.page_rows)

    def can_fit(self, rows: int, slot: Optional[int] = None) -> bool:
        have = len(self._owned.get(slot, ())) if slot is not None else 0
        return self.pages_for(rows) - have <= len(self._free)

    def pages_of(self, slot: int) -> List[int]:
        return list(self._owned.get(slot, ()))

    # ------------------------------------------------------------------ assignment
    def assign(self, slot: int, rows: int) -> None:
        """Make ``slot`` cover cache rows ``[0, rows)``; raises :class:`OutOfPages` (changing
        nothing) when the pool cannot."""
        if not 0 <= slot < self.max_batch:
            raise ValueError(f"slot {slot} outside [0, {self.max_batch})")
        need = self.pages_for(rows)
        if need > self.pages_per_seq:
            raise ValueError(f"{rows} rows exceed the {self.pages_per_seq * self.page_rows}-row sequence limit")
        owned = self._owned.setdefault(slot, [])
        extra = need - len(owned)
        if extra <= 0:
            return
        if extra > len(self._free):
            raise OutOfPages(f"slot {slot} needs {extra} more pages, {len(self._free)} free")
        for _ in range(extra):
            page = self._free.pop()
            self.host[slot, len(owned)] = page
            owned.append(page)
        self._dirty = True

    def release(self, slot: int) -> None:
        pages = self._owned.pop(slot, [])
        if pages:
            self._free.extend(reversed(pages))
            self.host[slot].zero_()
            self._dirty = True

    def reset(self) -> None:
        for slot in list(self._owned):
            self.release(slot)

    def device_table(self) -> torch.Tensor:
        if self._dirty:
            self.dev.copy_(self.host, non_blocking=self.device.type == "cuda")
            self._dirty = False
        return self.dev

    # ------------------------------------------------------------------ row addressing
    def rows(self, slots: torch.Tensor, positions: torch.Tensor) -> torch.Tensor:
        """Flat pool row of (slot, position) pairs (broadcasting) from the DEVICE table."""
        table = self.device_table()
        p = positions.long()
        page = table[slots.long(), torch.div(p, self.page_rows, rounding_mode="floor")]
        return page.long() * self.page_rows + p % self.page_rows
