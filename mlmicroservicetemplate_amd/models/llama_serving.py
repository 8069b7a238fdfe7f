"""Continuous (iteration-level) batching for ``/generate``.

A whole-request batch -- every sequence prefilled together, then decoded in lockstep until the
longest finishes -- makes a request that arrives one step late wait for the entire batch.  Here
one scheduler thread owns the model's ``max_batch`` KV-cache slots and runs iterations:

1. admit queued requests into free slots: one batched prefill writes their prompts into their
   own cache rows (``LlamaTP.step(..., slot_ids=...)``) and yields their first tokens;
2. one decode step over all ``max_batch`` slots (a fixed-shape hipGraph; idle slots decode a
   dummy token into their own, unused cache row), one token per active sequence;
3. retire sequences that hit ``max_new_tokens`` or an end-of-sequence id; their slots are free
   for the next iteration's admissions.

With a paged KV cache (``LlamaTP(kv_pages=...)``) a request is admitted only while the page pool
holds its prompt + ``max_new_tokens`` rows (FIFO: the head of the queue waits for pages rather
than being overtaken), and its pages return to the pool when it retires.

Each sequence samples with its own parameters and the same seeded rule as a batch-of-one
``LlamaTP.generate`` (``pick_token``), so results do not depend on what else is in flight.

Tensor parallelism: rank 0 runs the scheduler and broadcasts each iteration's admissions; every
rank then executes the identical iteration (same prefills, same decode steps, the same sampled
tokens from the all-gathered candidates), so followers need no other coordination.
"""
from __future__ import annotations

import collections
import concurrent.futures as cf
import logging
import threading
import time
from dataclasses import dataclass, field
from typing import Callable, Deque, List, Optional

import torch

from .llama import GenParams, LlamaTP

logger = logging.getLogger("mlsamd.llama_serving")


class EngineFull(Exception):
    pass


@dataclass
class _Seq:
    ids: List[int]
    gp: GenParams
    future: Optional[cf.Future]
    slot: int = -1
    out: List[int] = field(default_factory=list)
    cur: int = 0  # position of the next token to feed
    t_submit: float = field(default_factory=time.perf_counter)


class ContinuousLlama:
    def __init__(self, model: LlamaTP, max_queue: int = 4096,
                 broadcast: Optional[Callable[[Optional[List[_Seq]]], Optional[List[_Seq]]]] = None):
        self.m = model
        self.B = model.max_batch
        self.max_queue = max_queue
        self.broadcast = broadcast  # TP: rank 0 publishes each iteration's admissions
        self.slots: List[Optional[_Seq]] = [None] * self.B
        self._pending: Deque[_Seq] = collections.deque()
        self._lock = threading.Lock()
        self._wake = threading.Condition(self._lock)
        self._stop = False
        self._thread: Optional[threading.Thread] = None
        self.iterations = 0
        self.tokens = 0
        self.eos = set(model.cfg.eos_ids)

    # ---------------------------------------------------------------- client side
    def start(self) -> "ContinuousLlama":
        self._thread = threading.Thread(target=self._loop, name="llama-continuous", daemon=True)
        self._thread.start()
        return self

    def stop(self) -> None:
        with self._wake:
            self._stop = True
            self._wake.notify_all()
        if self._thread is not None:
            self._thread.join(30)

    def submit(self, ids: List[int], gp: GenParams) -> cf.Future:
        if not ids:
            raise ValueError("empty prompt")
        if len(ids) + gp.max_new_tokens > self.m.max_seq:
            raise ValueError(f"prompt + max_new_tokens exceeds the {self.m.max_seq}-token KV cache")
        pages = self.m.pages
        if pages is not None and pages.pages_for(len(ids) + gp.max_new_tokens) > pages.num_pages - 1:
            raise ValueError("prompt + max_new_tokens exceeds the whole KV page pool")
        fut: cf.Future = cf.Future()
        with self._wake:
            if self._stop:
                raise RuntimeError("engine stopped")
            if len(self._pending) >= self.max_queue:
                raise EngineFull(f"{len(self._pending)} generate requests queued")
            self._pending.append(_Seq(list(ids), gp, fut))
            self._wake.notify()
        return fut

    def stats(self) -> dict:
        d = {"active": sum(s is not None for s in self.slots), "queued": len(self._pending),
             "iterations": self.iterations, "tokens": self.tokens, "slots": self.B}
        if self.m.pages is not None:
            d["kv_pages_free"] = self.m.pages.free_pages
            d["kv_pages"] = self.m.pages.num_pages
        return d

    # ---------------------------------------------------------------- scheduler (rank 0)
    def _take_admissions(self) -> Optional[List[_Seq]]:
        with self._wake:
            while not self._stop and not self._pending and all(s is None for s in self.slots):
                self._wake.wait(0.05)
            if self._stop:
                return None
            free = [i for i, s in enumerate(self.slots) if s is None]
            admit = []
            pages = self.m.pages
            budget = pages.free_pages if pages is not None else 0
            while self._pending and free:
                seq = self._pending[0]
                if seq.future is not None and seq.future.cancelled():
                    self._pending.popleft()
                    continue
                if pages is not None:  # paged KV: admit while the pool holds prompt + budget (FIFO)
                    need = pages.pages_for(len(seq.ids) + seq.gp.max_new_tokens)
                    if need > budget:
                        break
                    budget -= need
                self._pending.popleft()
                seq.slot = free.pop(0)
                admit.append(seq)
            return admit

    def _loop(self) -> None:
        while True:
            admit = self._take_admissions()
            if self.broadcast is not None:
                self.broadcast(admit)  # None = stop, announced to the followers too
            if admit is None:
                break
            try:
                self.iteration(admit)
            except BaseException as e:  # fail everything in flight, keep serving
                logger.exception("generate iteration failed")
                for i, s in enumerate(self.slots):
                    if s is not None:
                        if s.future is not None and not s.future.done():
                            s.future.set_exception(e)
                        self.slots[i] = None
                        if self.m.pages is not None:
                            self.m.pages.release(i)

    # ---------------------------------------------------------------- one iteration (all ranks)
    @torch.no_grad()
    def iteration(self, admit: List[_Seq]) -> None:
        m = self.m
        if admit:
            for seq in admit:
                self.slots[seq.slot] = seq
                if m.pages is not None:  # every rank assigns the same pages (same calls, same order)
                    m.pages.assign(seq.slot, len(seq.ids) + seq.gp.max_new_tokens)
            S = max(len(s.ids) for s in admit)
            ids = torch.zeros(len(admit), S, dtype=torch.int32)
            for j, s in enumerate(admit):
                ids[j, : len(s.ids)] = torch.tensor(s.ids, dtype=torch.int32)
            lens = torch.tensor([len(s.ids) for s in admit], dtype=torch.int32, device=m.device)
            pos = torch.arange(S, dtype=torch.int32, device=m.device).unsqueeze(0).expand(len(admit), S).contiguous()
            k = max(1, min(max(s.gp.top_k for s in admit), m.top_k_max))
            slot_ids = torch.tensor([s.slot for s in admit], dtype=torch.int32, device=m.device)
            vals, idx = m.step(ids.to(m.device), pos, lens, decode=False, k=k, slot_ids=slot_ids)
            cv, ci = m.gather_candidates(vals, idx)
            for s, t in zip(admit, self._pick_rows(cv, ci, [(j, s.gp, 0) for j, s in enumerate(admit)])):
                s.out.append(t)
                s.cur = len(s.ids)
            self.tokens += len(admit)
            self._retire()
        active = [s for s in self.slots if s is not None]
        if active:
            # host lists -> one tensor each (per-element tensor writes cost ~us apiece at 128 slots)
            tok_l, cur_l = [0] * self.B, [0] * self.B
            for s in active:
                tok_l[s.slot] = s.out[-1]
                cur_l[s.slot] = s.cur
            tok = torch.tensor(tok_l, dtype=torch.int32)
            cur = torch.tensor(cur_l, dtype=torch.int32)
            k = max(1, min(max(s.gp.top_k for s in active), m.top_k_max))
            max_ctx = max(s.cur for s in active) + 1
            vals, idx = m.decode_step(tok.to(m.device), cur.to(m.device), k, max_ctx=max_ctx)
            cv, ci = m.gather_candidates(vals, idx)
            picks = self._pick_rows(cv, ci, [(s.slot, s.gp, len(s.out)) for s in active])
            for s, t in zip(active, picks):
                s.out.append(t)
                s.cur += 1
            self.tokens += len(active)
            self._retire()
        self.iterations += 1

    def _pick_rows(self, cv: torch.Tensor, ci: torch.Tensor, rows) -> List[int]:
        """Next token of each ``(row, gen params, step)``: the greedy rows in one vectorised
        argmax / gather (first maximum, as ``pick_token``), sampled rows one by one."""
        out: List[Optional[int]] = [None] * len(rows)
        greedy = [j for j, (_r, gp, _t) in enumerate(rows) if gp.top_k <= 1]
        if greedy:
            r = torch.tensor([rows[j][0] for j in greedy], dtype=torch.long)
            best = ci[r].gather(1, cv[r].argmax(1, keepdim=True)).squeeze(1).tolist()
            for j, t in zip(greedy, best):
                out[j] = int(t)
        for j, (r, gp, step) in enumerate(rows):
            if out[j] is None:
                out[j] = self.m.pick_token(cv[r], ci[r], gp, step)
        return out  # type: ignore[return-value]

    def _retire(self) -> None:
        for i, s in enumerate(self.slots):
            if s is None:
                continue
            if len(s.out) >= s.gp.max_new_tokens or (s.out and s.out[-1] in self.eos):
                self.slots[i] = None
                if self.m.pages is not None:
                    self.m.pages.release(i)
                if s.future is not None and not s.future.done():
                    s.future.set_result(list(s.out))
