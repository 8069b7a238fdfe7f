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

Tensor parallelism: rank 0 runs the scheduler and publishes each iteration's admissions; every
rank then executes the identical iteration (same prefills, same decode steps, the same sampled
tokens from the all-gathered candidates), so followers need no other coordination.  What a
follower must learn per iteration is rank 0's header (stop? how many admissions, longest prompt).
With the device-resident iterations at TP > 1 that header rides the decode step's X4 gather: before
replaying iteration i's decode graph rank 0 already takes iteration i+1's admissions (from the slots
free at that point -- a slot freed by iteration i is refilled one iteration later) and writes the
header into its control row (``LlamaTP.serve_state`` ``ctl_in``); every rank reads it back with the
iteration's one ``E`` copy.  A follower then issues a collective only when there is something to
receive: the admissions' metadata / prompt ids, or an explicit header when no decode step ran (the
engine was idle).  ``MLS_TP_CARRY_HEADER=0`` restores one header broadcast per iteration.

Device-resident iterations (default whenever ``LlamaTP._device_loop_ok`` holds -- the fused
backend on a GPU with graph-capturable collectives; ``MLS_SERVE_DEVICE_PICK=0`` forces the host
path): every slot's next-token state (token, position, length, step, sampling parameters, an
active mask) lives on the device (``LlamaTP.serve_state``).  The prefill of new sequences ends
with the X4 merge + pick writing straight into their slots (``ops.decode_pick(rows=...)``), the
decode step is ONE captured graph (forward + on-device all-gather + pick of the active slots,
``LlamaTP.serve_graph``), and the host reads back one ``[2, B]`` int32 tensor per iteration for
end-of-sequence / retirement -- no uncaptured collectives, no host token picking.

Failure detection: every ``MLS_TP_HEALTH_EVERY`` iterations all ranks poll the one-shot
all-reduce's error word (``LlamaTP.check_comm_health``, a collective); a peer that missed a
collective fails every in-flight request (rank 0's futures get ``TPCommError``), the IPC path is
dropped and serving continues on RCCL.  Followers run the same :meth:`ContinuousLlama.run_iteration`
(same checks, same slot resets), so the ranks stay in step.
"""
from __future__ import annotations

import collections
import concurrent.futures as cf
import logging
import os
import threading
import time
from dataclasses import dataclass, field
from typing import Callable, Deque, List, Optional

import torch

from .llama import CTL_WORDS, GenParams, LlamaTP, TPCommError

logger = logging.getLogger("mlsamd.llama_serving")

OP_STOP, OP_GENERATE, OP_ITER = 0, 1, 2  # TP control header ops (plugins/llm.py)


class EngineFull(Exception):
    pass


class HeaderLost(RuntimeError):
    """A follower read a carried header that fails its check: the decode step's exchange with
    rank 0 is broken, so this rank cannot know what rank 0 does next -- it stops following (the
    process exits non-zero) rather than guess."""


def ctl_check(iteration: int, op: int, n: int, S: int) -> int:
    """Check word of a carried header: ties it to the iteration all ranks are in (a stale or torn
    control row from a timed-out exchange fails it)."""
    h = (iteration * 2654435761 + op * 40503 + n * 9973 + S * 131 + 0x4D4C5331) & 0x7FFFFFFF
    return int(h)


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
                 broadcast: Optional[Callable[[Optional[List[_Seq]]], Optional[List[_Seq]]]] = None,
                 channel=None):
        self.m = model
        self.B = model.max_batch
        self.max_queue = max_queue
        self.broadcast = broadcast  # TP (legacy hook): rank 0 publishes each iteration's admissions
        # TP: the control channel (plugins/llm.py LlamaPlugin: send_header / send_admissions on rank
        # 0, recv_header / recv_admissions on the followers); headers ride the decode gather when
        # they can (module docstring)
        self.channel = channel
        self.leader = int(getattr(model, "rank", 0)) == 0
        self._carry = (channel is not None and model.tp > 1
                       and os.environ.get("MLS_TP_CARRY_HEADER", "1") != "0")
        self._next_hdr = None  # (op, n, S) of the next iteration, read back from this one's decode step
        self._planned: Optional[List[_Seq]] = None  # rank 0: the admissions that header announced
        self._ctl_host = None  # rank 0: pinned int32 [CTL_WORDS] staging of the header
        self._carry_check = False  # this iteration's carried header needs the health all-reduce
        self._ctl_bad = None  # the control row read back failed its check (its words)
        # how iteration headers reached the followers (diagnostics; tests/llama_tp_worker.py)
        self.proto = {"explicit_headers": 0, "carried_headers": 0, "admission_broadcasts": 0,
                      "iters_no_admit_bcast": 0}
        self.slots: List[Optional[_Seq]] = [None] * self.B
        self._pending: Deque[_Seq] = collections.deque()
        self._lock = threading.Lock()
        self._wake = threading.Condition(self._lock)
        self._stop = False
        self._thread: Optional[threading.Thread] = None
        self.iterations = 0
        self.tokens = 0
        self.eos = set(model.cfg.eos_ids)
        self.health_every = max(0, int(getattr(model, "health_every", 32)))
        self.failures = 0
        # device-resident iterations (module docstring); re-decided only while no sequence is in flight
        self._want_dev = os.environ.get("MLS_SERVE_DEVICE_PICK", "1") != "0"
        self.dev_mode = False
        self.host_reads = 0  # device -> host copies made by the iterations (diagnostics / tests)

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
        # the temperature every rank samples with: the followers receive it in 1/1000 units
        # (plugins/llm.py _broadcast_iter), so rank 0 uses the same quantised value
        gp = GenParams(gp.max_new_tokens, gp.top_k, round(float(gp.temperature) * 1000) / 1000.0, gp.seed)
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
    def _take_admissions(self, block: bool = True) -> Optional[List[_Seq]]:
        """Queued requests for the free slots (None = stop).  ``block``: wait while there is
        nothing to do at all."""
        with self._wake:
            while block and not self._stop and not self._pending and all(s is None for s in self.slots):
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
            admit = self._leader_admissions()
            if admit is None:
                break
            self.run_iteration(admit)

    def _leader_admissions(self) -> Optional[List[_Seq]]:
        """Rank 0: this iteration's admissions (None = stop), announced to the followers -- by
        nothing more when the last decode step already carried the header, else explicitly."""
        hdr, self._next_hdr = self._next_hdr, None
        if hdr is not None:
            admit, self._planned = self._planned, None
            self.proto["carried_headers"] += 1
            if hdr[0] == OP_STOP:
                return None
            if admit:
                self.channel.send_admissions(admit)
                self.proto["admission_broadcasts"] += 1
            return admit or []
        admit = self._take_admissions()
        if self.channel is not None:
            self.channel.send_header(admit)  # None = stop; admissions follow the header when any
            self.proto["explicit_headers"] += 1
            if admit:
                self.proto["admission_broadcasts"] += 1
        elif self.broadcast is not None:
            self.broadcast(admit)  # None = stop, announced to the followers too
        return admit

    def follow(self) -> int:
        """Ranks > 0 (TP): replay rank 0's iterations until it stops.  Each header comes from the
        previous decode step's read-back when it carried one, else from the channel; admissions
        are received only when the header announces some."""
        # hdr_s: time spent learning each iteration's header (+ receiving its admissions); first_hdr_s:
        # the first of them, which also waits out rank 0's start-up (weights, graph capture)
        st = self.follower_stats = {"iters": 0, "hdr_s": 0.0, "hdr_max_s": 0.0, "iter_s": 0.0, "first_hdr_s": None,
                                    "explicit_s": 0.0, "carried_s": 0.0}
        while True:
            t0 = time.perf_counter()
            hdr, self._next_hdr = self._next_hdr, None
            bcast = hdr is None
            if hdr is None:
                hdr = self.channel.recv_header()
                self.proto["explicit_headers"] += 1
            else:
                self.proto["carried_headers"] += 1
            op, n, S = hdr
            if op == OP_STOP:
                logger.info("follower: stop")
                return 0
            admit: List[_Seq] = []
            if n:
                admit = self.channel.recv_admissions(n, S)
                self.proto["admission_broadcasts"] += 1
                bcast = True
            elif bcast:
                self.proto["iters_no_admit_bcast"] += 1
            dt = time.perf_counter() - t0
            if st["first_hdr_s"] is None:
                st["first_hdr_s"] = dt
            else:
                st["hdr_s"] += dt
                st["hdr_max_s"] = max(st["hdr_max_s"], dt)
                st["explicit_s" if bcast else "carried_s"] += dt
            t1 = time.perf_counter()
            try:
                self.run_iteration(admit)  # same failure handling / health checks as rank 0
            except HeaderLost:
                logger.error("follower: carried header lost; leaving the TP group")
                return 3
            st["iter_s"] += time.perf_counter() - t1
            st["iters"] += 1

    def _plan_next(self, st) -> None:
        """Rank 0, before the decode replay: take the next iteration's admissions now and write
        their header into the control row the decode step's gather carries to every rank."""
        planned = self._take_admissions(block=False)
        self._planned = planned
        if planned is None:
            hdr = (OP_STOP, 0, 0)
        else:
            hdr = (OP_ITER, len(planned), max((len(q.ids) for q in planned), default=0))
        if self._ctl_host is None:
            self._ctl_host = torch.zeros(CTL_WORDS, dtype=torch.int32, pin_memory=torch.cuda.is_available())
        self._ctl_host.numpy()[:] = [*hdr, ctl_check(self.iterations, *hdr)]
        st["ctl_in"].copy_(self._ctl_host, non_blocking=True)

    def _sync_iterations(self) -> None:
        """Collective (after a TPCommError, which every rank raises from the same all-reduce):
        every rank continues from the largest iteration count."""
        import torch.distributed as dist

        group = getattr(self.m.comm, "group", None)
        dev = self.m.device if dist.get_backend(group) == "nccl" else torch.device("cpu")
        t = torch.tensor([self.iterations], dtype=torch.int64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
        self.iterations = int(t.item())

    def _unplan(self) -> None:
        """Rank 0 after a failed iteration: the planned admissions go back to the queue head."""
        planned, self._planned = self._planned, None
        self._next_hdr = None
        if planned:
            with self._wake:
                for q in reversed(planned):
                    q.slot = -1
                    self._pending.appendleft(q)

    def run_iteration(self, admit: List[_Seq]) -> None:
        """One iteration + the periodic comm-health check; on any failure every in-flight request
        fails and the slots are freed (rank 0 and the followers alike, so the ranks stay in step)."""
        finished: List[_Seq] = []
        try:
            finished = self.iteration(admit)
            # a result leaves only after a health check that covers the steps which produced it (a
            # peer that missed a one-shot all-reduce leaves partial sums behind): every iteration
            # that retires a sequence, and every health_every-th one (all ranks: same decisions);
            # also every iteration whose carried header is in doubt or announces admissions
            doubt, self._carry_check = self._carry_check, False
            if self.m.tp > 1 and (doubt or finished or (self.health_every and self.iterations % self.health_every == 0)):
                self.m.check_comm_health()
            bad, self._ctl_bad = self._ctl_bad, None
            if bad is not None:  # torn control row, yet no rank saw a timeout: cannot resynchronise
                raise HeaderLost(f"iteration {self.iterations - 1}: control row {bad} fails its check")
            for q in finished:
                if q.future is not None and not q.future.done():
                    q.future.set_result(list(q.out))
        except HeaderLost:
            raise
        except BaseException as e:  # fail everything in flight, keep serving
            self._unplan()  # the next header goes out explicitly (every rank resets alike)
            self._carry_check, self._ctl_bad = False, None
            if isinstance(e, TPCommError) and self._carry:
                # raised on every rank by the same all-reduce; with carried headers a rank in doubt
                # may have reached it one iteration before its peers: agree on the count again
                self._sync_iterations()
            logger.exception("generate iteration failed")
            self.failures += 1
            for q in finished:
                if q.future is not None and not q.future.done():
                    q.future.set_exception(e)
            for i, s in enumerate(self.slots):
                if s is not None:
                    if s.future is not None and not s.future.done():
                        s.future.set_exception(e)
                    self.slots[i] = None
                    if self.m.pages is not None:
                        self.m.pages.release(i)
            if self.dev_mode:
                st = self.m.serve_state(self.B)
                st["active"].zero_()
                st["pos"].zero_()
                st["lens"].fill_(1)

    # ---------------------------------------------------------------- one iteration (all ranks)
    def _dev_ok(self) -> bool:
        if not self._want_dev:
            return False
        if any(s is not None for s in self.slots):  # sequences in flight keep their mode
            return self.dev_mode
        return self.m._device_loop_ok(self.B, self.m.top_k_max)

    @torch.no_grad()
    def iteration(self, admit: List[_Seq]) -> List[_Seq]:
        """Admit, decode one step, retire.  Returns the retired sequences (slots already freed);
        :meth:`run_iteration` resolves their futures once the comm-health check has passed."""
        self.dev_mode = self._dev_ok()
        if self.dev_mode:
            return self._iteration_dev(admit)
        return self._iteration_host(admit)

    @torch.no_grad()
    def _iteration_dev(self, admit: List[_Seq]) -> List[_Seq]:
        m = self.m
        dev = m.device
        st = m.serve_state(self.B)
        ops = m.ops
        if admit:
            for seq in admit:
                self.slots[seq.slot] = seq
                if m.pages is not None:
                    m.pages.assign(seq.slot, len(seq.ids) + seq.gp.max_new_tokens)
            S = max(len(s.ids) for s in admit)
            ids = torch.zeros(len(admit), S, dtype=torch.int32)
            for j, s in enumerate(admit):
                ids[j, : len(s.ids)] = torch.tensor(s.ids, dtype=torch.int32)
            # one H2D of the new slots' state: slot, pos (the pick advances it to the prompt length),
            # lens, top_k, seed; temperatures separately (fp32)
            meta = torch.tensor([[s.slot, len(s.ids) - 1, len(s.ids), s.gp.top_k, s.gp.seed] for s in admit],
                                dtype=torch.int64).to(dev, non_blocking=True)
            temps = torch.tensor([s.gp.temperature for s in admit], dtype=torch.float32).to(dev, non_blocking=True)
            slot_ids = meta[:, 0].to(torch.int32)
            lens = meta[:, 2].to(torch.int32)
            pos = torch.arange(S, dtype=torch.int32, device=dev).unsqueeze(0).expand(len(admit), S).contiguous()
            k = max(1, min(max(s.gp.top_k for s in admit), m.top_k_max))
            vals, idx = m.step(ids.to(dev), pos, lens, decode=False, k=k, slot_ids=slot_ids)
            cv, ci = m._gather_dev(vals, idx)
            sl = meta[:, 0]
            st["pos"][sl] = meta[:, 1].to(torch.int32)
            st["lens"][sl] = lens
            st["step"][sl] = 0
            st["topk"][sl] = meta[:, 3].to(torch.int32)
            st["seed"][sl] = meta[:, 4]
            st["temp"][sl] = temps
            st["active"][sl] = 1
            ops.decode_pick(cv, ci, st["tok"], st["pos"], st["lens"], st["step"], topk=st["topk"], temp=st["temp"],
                            seed=st["seed"], rows=slot_ids, emit=st["E"][0])
            for s in admit:
                s.cur = len(s.ids)
        active = [s for s in self.slots if s is not None]
        carry = self._carry and m.tp > 1
        if active:
            k = max(1, min(max(s.gp.top_k for s in active), m.top_k_max))
            max_ctx = max(s.cur for s in active) + 1
            g = m.serve_graph(self.B, k, m.ctx_bucket(max_ctx))
            if m.pages is not None:
                m.pages.device_table()  # the graph reads the table buffer in place
            if carry and self.leader:
                self._plan_next(st)  # the next iteration's header rides this step's gather
            g.replay()
        if admit or active:
            E_all = st["E_all"].cpu()  # the iteration's one device -> host copy
            self.host_reads += 1
            E = E_all[: 2 * self.B].view(2, self.B)
            e0, e1 = E[0].tolist(), E[1].tolist()
            if active and carry:
                c = E_all[2 * self.B:].tolist()
                ok = c[3] == ctl_check(self.iterations, c[0], c[1], c[2]) and c[0] in (OP_STOP, OP_ITER)
                # a carried header is trusted only with no peer timeout on this rank; any doubt, and
                # any header that announces admissions (the process group is about to be used), goes
                # through the comm-health all-reduce first -- a rank in doubt stops taking part in
                # the one-shot collectives, so its peers time out too and join that all-reduce
                self._carry_check = (not ok) or c[4] != 0 or c[1] > 0
                self._ctl_bad = None if ok else c[:4]
                self._next_hdr = (c[0], c[1], c[2]) if ok else None
            new = {id(s) for s in admit}
            for s in admit:
                s.out.append(int(e0[s.slot]))
                self.tokens += 1
            for s in active:
                if id(s) in new and (len(s.out) >= s.gp.max_new_tokens or s.out[-1] in self.eos):
                    continue  # finished on its prefill token: the decode pick is discarded
                s.out.append(int(e1[s.slot]))
                s.cur += 1
                self.tokens += 1
            done = self._retire()
            if done:
                idx_t = torch.tensor([q.slot for q in done], dtype=torch.int64).to(dev, non_blocking=True)
                st["active"][idx_t] = 0
                st["pos"][idx_t] = 0
                st["lens"][idx_t] = 1
        else:
            done = []
        self.iterations += 1
        return done

    @torch.no_grad()
    def _iteration_host(self, admit: List[_Seq]) -> List[_Seq]:
        m = self.m
        done: List[_Seq] = []
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
            done += self._retire()
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
            done += self._retire()
        self.iterations += 1
        return done

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

    def _retire(self) -> List[_Seq]:
        """Free the slots of finished sequences (their futures are resolved by run_iteration)."""
        done = []
        for i, s in enumerate(self.slots):
            if s is None:
                continue
            if len(s.out) >= s.gp.max_new_tokens or (s.out and s.out[-1] in self.eos):
                self.slots[i] = None
                done.append(s)
                if self.m.pages is not None:
                    self.m.pages.release(i)
        return done
