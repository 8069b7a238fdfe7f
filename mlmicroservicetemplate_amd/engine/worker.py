"""Per-GPU execution engine (T4 / P4 / P5 of SURVEY.md §1.2, §2.E.3).

One :class:`GpuEngine` owns one model replica on one device and runs fixed-shape batches:

    host request arrays --memcpy--> pinned slot --H2D stream--> device slot
        --compute stream: hipGraph replay (bucket b)--> device outputs --D2H stream--> pinned out

* **Buckets**: a batch of ``n`` requests is padded to the smallest graph bucket ``>= n``
  (1, 2, 4, ... MAX_BATCH); each (slot, bucket) has its own captured hipGraph, replayed with
  static input/output buffers, so the steady-state step is one graph launch.
* **Slots**: ``inflight`` independent staging slots (pinned host in/out + device input) so
  batch i+1's host copy and H2D overlap batch i's graph, and batch i's D2H overlaps batch
  i+1's compute -- event-ordered across three HIP streams, no device-wide syncs.
* The host thread only blocks on a *blocking-sync* event of its own slot, so concurrent
  callers (the batcher's executor threads) keep the GPU fed.
* **Concurrent slots** (``concurrent=True``): each slot replays its graphs on its own compute
  stream from its own graph memory pool, so two batches' kernels co-run -- the small
  latency-bound layers of one batch fill the CUs the other leaves idle.  The model must then
  keep per-stream scratch (``ResNet50Fused`` keys its split-K workspace by stream).

The engine is model-agnostic: a model adapter provides ``sample_shape``/``sample_dtype`` of
one request and ``forward(device_batch) -> tuple[Tensor, ...]`` (fixed-shape outputs whose
first dim is the batch).
"""
from __future__ import annotations

import contextlib
import logging
import os
import queue
import threading
import time
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from ..utils import tracing
from .staging import HostStager

logger = logging.getLogger("mlsamd.engine")

_NP_DTYPES = {torch.uint8: np.uint8, torch.int32: np.int32, torch.int64: np.int64, torch.float32: np.float32,
              torch.bfloat16: None, torch.float16: np.float16}


def pick_bucket(n: int, buckets: Sequence[int]) -> int:
    for b in buckets:
        if b >= n:
            return b
    raise ValueError(f"batch of {n} exceeds the largest bucket {buckets[-1]}")


@dataclass
class _Slot:
    idx: int
    host_in: torch.Tensor  # pinned [max_b, *sample_shape]
    dev_in: torch.Tensor  # device [max_b, *sample_shape]
    # pinned int64 cell holding the address the graph's input pull reads from (ops.h2d_pull_cell):
    # host_in's by default, a pre-staged batch's own pinned buffer for launch_prepared()
    src_cell: Optional[torch.Tensor] = None
    cell_np: Optional[np.ndarray] = None  # numpy view of src_cell (cheap host writes)
    outs: Dict[int, Tuple[torch.Tensor, ...]] = field(default_factory=dict)  # bucket -> device outputs
    host_out: Dict[int, Tuple[torch.Tensor, ...]] = field(default_factory=dict)  # bucket -> pinned outputs
    graphs: Dict[int, torch.cuda.CUDAGraph] = field(default_factory=dict)
    graph_copies: Dict[int, bool] = field(default_factory=dict)  # bucket -> copies inside the graph
    pushed: Dict[int, bool] = field(default_factory=dict)  # bucket -> results pushed to host by the graph
    pulled: Dict[int, bool] = field(default_factory=dict)  # bucket -> input pulled from host by the graph
    native: Dict[int, tuple] = field(default_factory=dict)  # bucket -> mls_engine_launch arguments
    s_comp: Optional[torch.cuda.Stream] = None  # this slot's compute stream (concurrent mode)
    pool: Optional[tuple] = None  # this slot's graph memory pool (concurrent mode)
    ev_h2d: Optional[torch.cuda.Event] = None
    ev_comp: Optional[torch.cuda.Event] = None
    ev_done: Optional[torch.cuda.Event] = None


class Ticket:
    """Handle for an enqueued batch; :meth:`wait` returns numpy outputs trimmed to ``n`` rows."""

    __slots__ = ("engine", "slot", "bucket", "n", "t_submit", "t_arrive", "_result", "staged", "stamps", "launch_ns")

    def __init__(self, engine: "GpuEngine", slot: _Slot, bucket: int, n: int, staged: Optional["Prepared"] = None):
        self.engine = engine
        self.slot = slot
        self.bucket = bucket
        self.n = n
        self.t_submit = time.perf_counter()  # enqueue time (launch -> done: the pacing estimate)
        # when the batch's requests were handed to the engine: its staging start for a prepared
        # batch (request latency = t_arrive -> result)
        self.t_arrive = staged.t0 if staged is not None else self.t_submit
        self._result = None
        self.staged = staged  # a prepared batch's pinned buffer, returned to the pool on completion
        self.stamps = None  # submit(): perf_counter at slot wait / staged / enqueued (diagnostics)
        # native enqueue: ns spent in its H2D copy, graph launch, D2H copies and event record
        self.launch_ns: Optional[Tuple[int, ...]] = None

    def wait(self) -> Tuple[np.ndarray, ...]:
        if self._result is None:
            self._result = self.engine._finish(self)
        return self._result


class Prepared:
    """A batch staged into a spare pinned buffer (:meth:`GpuEngine.prepare`) before any slot is
    free; :meth:`GpuEngine.launch_prepared` enqueues it (H2D straight from that buffer)."""

    __slots__ = ("buf", "n", "t0", "dev")

    def __init__(self, buf: torch.Tensor, n: int, t0: Optional[float] = None):
        self.buf = buf
        self.n = n
        self.t0 = time.perf_counter() if t0 is None else t0  # prepare() start
        self.dev = None  # prepull: (device buffer, event after its pull) -- the batch already on the GPU


class GpuEngine:
    def __init__(
        self,
        forward: Callable[[torch.Tensor], Tuple[torch.Tensor, ...]],
        device,
        sample_shape: Tuple[int, ...],
        sample_dtype: torch.dtype = torch.uint8,
        buckets: Sequence[int] = (1, 2, 4, 8, 16, 32),
        inflight: int = 2,
        use_graphs: bool = True,
        name: str = "engine",
        concurrent: bool = False,
        stage_workers: Optional[int] = None,
        copies_on_slot_stream: Optional[bool] = None,
        cu_partitions: Optional[int] = None,
        spin_wait_us: Optional[float] = None,
    ):
        self.forward = forward
        self.device = torch.device(device)
        self.sample_shape = tuple(sample_shape)
        self.sample_dtype = sample_dtype
        self.buckets = sorted(set(int(b) for b in buckets))
        self.max_batch = self.buckets[-1]
        self.inflight = max(1, int(inflight))
        self.use_graphs = use_graphs
        self.concurrent = bool(concurrent) and self.inflight > 1
        # Spatial partitioning (cu_partitions / MLS_CU_PARTITION = 2, 4 or 8; 0 = off): concurrent
        # slot i's stream is CU-masked to partition i % P (ops.partition_masks, csrc/partition.hip):
        # with MLS_CU_PARTITION_MODE=intra (default) every partition holds 1 / P of the CUs of every
        # XCD (a CU mask cannot confine a queue to whole XCDs: an XCD left without mask bits runs on
        # all its CUs -- profiles/r3_cu_mask_census.txt).  Two halves x 2 batches each, unpaced:
        # ResNet-50 bs=32 54.5-55.6k vs 52.8-53.1k req/s at 200 steps, 49.3-51.4k vs 48.0-49.6k at 20,
        # p50 2.2-2.3 vs 2.55-2.8 ms (profiles/r3_cu_partition_ab.jsonl): the two batches of a half
        # co-run on 128 CUs instead of five interleaving over 256.  A masked stream holds its own
        # hardware queue, so a partitioned engine uses at most MLS_HW_QUEUES (4) masked streams --
        # 5-8 of them measured 35-44k -- and slots beyond that share them round-robin (slot i on
        # stream i % 4): their GPU work queues behind the stream-mate's while their host-side
        # phases (staging, result hand-off) overlap, which the HTTP front end needs.
        if cu_partitions is None:
            cu_partitions = int(os.environ.get("MLS_CU_PARTITION", "0"))
        self.cu_partitions = int(cu_partitions) if self.concurrent else 0
        self.part_streams = 0  # masked streams the slots are spread over
        part_masks = None
        if self.cu_partitions:
            from .. import ops

            part_masks = ops.partition_masks(self.cu_partitions, self.device,
                                             mode=os.environ.get("MLS_CU_PARTITION_MODE", "intra"))
            if part_masks is None:
                logger.warning("%s: CU partitioning unavailable (mask not verified); slots use all CUs", name)
                self.cu_partitions = 0
            else:
                hwq = int(os.environ.get("MLS_HW_QUEUES", "4"))
                n = min(self.inflight, max(hwq, self.cu_partitions))
                self.part_streams = max(self.cu_partitions, n - n % self.cu_partitions)
                try:  # create (or take from the pool) every masked stream up front
                    masked = [ops.cu_masked_stream(part_masks[si % self.cu_partitions], self.device,
                                                   key=si // self.cu_partitions) for si in range(self.part_streams)]
                except Exception as e:  # e.g. no hardware queue left for another masked stream
                    logger.warning("%s: CU-masked streams unavailable (%s); slots use all CUs", name, e)
                    part_masks, self.cu_partitions, self.part_streams = None, 0, 0
        # concurrent slots: a slot's H2D and D2H ride its own compute stream instead of the shared
        # copy streams (those share the 4 hardware queues with the slot streams).  With native
        # staging + launch pacing this is +3-4 % req/s on ResNet-50 (20 steps 47.2-48.3k vs
        # 45.9-46.3k, 300 steps 53.3k vs 51.3-51.7k; profiles/r2_hwq_slotcopies_with_pacing.jsonl);
        # MLS_SLOT_COPIES=0 restores the copy streams
        if copies_on_slot_stream is None:
            copies_on_slot_stream = os.environ.get("MLS_SLOT_COPIES", "1") == "1"
        self.copies_on_slot_stream = bool(copies_on_slot_stream) and self.concurrent
        self.graph_copies = (self.copies_on_slot_stream and use_graphs
                             and os.environ.get("MLS_GRAPH_COPIES", "0") == "1")
        # the per-batch enqueue (H2D -> graph -> D2H -> done event on the slot stream) as one native
        # call (ops/csrc/engine_launch.hip) instead of ~10 Python-level calls: 85-100 us -> a few us
        # of host time per batch.  The instrumented Python sequence runs while tracing is active.
        self.native_launch = (self.copies_on_slot_stream and use_graphs and not self.graph_copies
                              and os.environ.get("MLS_NATIVE_LAUNCH", "1") == "1")
        # SDMA-free batch I/O (MLS_PULL_H2D=<workgroups>, default 8; 0 = hipMemcpyAsync copies): the
        # slot's graph starts with a small copy kernel that pulls the pinned batch over PCIe
        # (ops.h2d_pull) and ends with one that pushes the results into the pinned output buffers
        # (ops.d2h_push).  SDMA H2D copies stalled ~6-7 ms in 8 of ~100 20-step bench runs over 6
        # boxes (hipMemcpyAsync blocked, every in-flight batch waiting on its copy); with both copies
        # as kernels 0 of 24 on a box where the SDMA arms stalled 6 of 24 (docs/PERF_NOTES.md, round 5)
        self.pull_h2d = int(os.environ.get("MLS_PULL_H2D", "8")) if (
            self.copies_on_slot_stream and use_graphs and not self.graph_copies
            and sample_dtype == torch.uint8) else 0
        # Early pull of pre-staged batches (MLS_PREPULL=1): prepare() stages a batch into a spare
        # pinned buffer while every slot is busy AND pulls it at once, on the engine's I/O stream,
        # into a spare device buffer; the slot's graph later starts with a device-to-device copy
        # (the same cell-addressed copy kernel with all MLS_PREPULL_WG workgroups, ~2-3 us) instead
        # of the ~90 us PCIe pull -- the pull leaves the batch's critical path.
        self.prepull = bool(self.pull_h2d) and os.environ.get("MLS_PREPULL", "0") == "1"
        self.pull_grid = max(self.pull_h2d, int(os.environ.get("MLS_PREPULL_WG", "64"))) if self.prepull \
            else self.pull_h2d
        # host staging (request arrays -> pinned slot): a persistent native copy pool (GIL released,
        # the submitting thread copies too); one thread's ~5-8 GB/s memcpy is not enough for a
        # 4.8 MB ResNet batch every ~0.6 ms next to the rest of the host loop
        self._stager = HostStager(stage_workers, name=name)
        self.name = name
        self._tr_stage, self._tr_h2d, self._tr_replay, self._tr_d2h, self._tr_wait = (
            f"{name}.{k}" for k in ("stage", "h2d", "replay", "d2h", "d2h_wait"))
        self._enqueue_lock = threading.Lock()
        # completion wait (Ticket.wait): poll the done event for up to spin_wait_us (MLS_EVENT_SPIN_US)
        # before the blocking (interrupt) sync -- the refill of a freed slot starts sooner; for a
        # process whose thread has nothing else to do (bench.py's closed loop), not for servers
        # whose waiter threads share the GIL with the front end (default 0 = block at once)
        env_spin = os.environ.get("MLS_EVENT_SPIN_US")
        self._spin_us = float(env_spin) if env_spin is not None else float(spin_wait_us or 0.0)
        # Launch pacing.  Batches that become ready together (a closed loop, a burst, two slots
        # freed by one clump of completions) otherwise enter the network in lock step: all in the
        # bandwidth-bound early layers at once, then all in the latency-bound late ones, and keep
        # completing in clumps.  Near saturation a launch waits until PACE x (batch latency EWMA /
        # inflight) -- Little's law: the completion interval of a full pipeline -- has passed since
        # the previous launch.  The estimate shrinks when pacing shortens the latency, so it cannot
        # run away (an estimate from observed completion intervals does: pacing stretches them).
        # MLS_LAUNCH_PACE=0 disables, MLS_LAUNCH_GAP_US=<us> fixes the gap instead.
        # (partitioned engines run unpaced unless MLS_LAUNCH_PACE says otherwise: each half holds
        # only two batches, and pacing measured level-to-worse there)
        self._pace = float(os.environ.get("MLS_LAUNCH_PACE", "0" if self.cu_partitions else "1.0"))
        self._fixed_gap_s = float(os.environ.get("MLS_LAUNCH_GAP_US", "0")) * 1e-6
        self._last_launch = 0.0
        self._lat_s = 0.0  # EWMA of launch -> done latency
        self._lat_n = 0  # completions seen
        self._pace_lock = threading.Lock()
        # pace only with at least this many other batches in flight (default: inflight - 2)
        self._pace_min_busy = int(os.environ.get("MLS_PACE_MIN_BUSY", "0")) or max(1, self.inflight - 2)
        self._free: "queue.Queue[_Slot]" = queue.Queue()
        self.slots: List[_Slot] = []
        self.batches = 0
        self.samples = 0
        self.busy_s = 0.0
        self.healthy = True
        self.last_error: Optional[str] = None
        with torch.cuda.device(self.device):
            self.s_io = torch.cuda.Stream(self.device) if self.prepull else None  # early pulls
            self.s_h2d = torch.cuda.Stream(self.device)
            self.s_comp = torch.cuda.Stream(self.device)
            self.s_d2h = torch.cuda.Stream(self.device)
            self._pool = torch.cuda.graph_pool_handle() if use_graphs else None
            for i in range(self.inflight):
                shape = (self.max_batch, *self.sample_shape)
                slot = _Slot(
                    idx=i,
                    host_in=torch.zeros(shape, dtype=sample_dtype, pin_memory=True),
                    dev_in=torch.zeros(shape, dtype=sample_dtype, device=self.device),
                    ev_h2d=torch.cuda.Event(),
                    ev_comp=torch.cuda.Event(),
                    ev_done=torch.cuda.Event(blocking=True),
                    src_cell=torch.zeros(2, dtype=torch.int64, pin_memory=True),
                )
                slot.cell_np = slot.src_cell.numpy()
                slot.cell_np[0] = slot.host_in.data_ptr()
                slot.cell_np[1] = self.pull_h2d  # workgroups that copy from host memory
                if self.concurrent:
                    if part_masks is not None:
                        # pooled per (mask, slot-in-partition): engines built one after another in a
                        # process reuse the queues; slots beyond them share round-robin
                        slot.s_comp = masked[i % self.part_streams]
                    else:
                        slot.s_comp = torch.cuda.Stream(self.device)
                    slot.pool = torch.cuda.graph_pool_handle() if use_graphs else None
                else:
                    slot.s_comp = self.s_comp
                    slot.pool = self._pool
                self.slots.append(slot)
                self._free.put(slot)
        # spare pinned input buffers for prepare() / launch_prepared(): a batch is staged while every
        # slot is still busy, so a freed slot only waits for the enqueue (the staging copy of a
        # 4.8 MB ResNet batch, 80-180 us of host time, moves off the refill path).  Allocated on the
        # first prepare(): serving engines that never pre-stage hold no extra pinned memory
        self._spare: "queue.Queue[torch.Tensor]" = queue.Queue()
        self._spare_lock = threading.Lock()
        self._spare_made = False
        self._dev_spare: "queue.Queue[tuple]" = queue.Queue()  # prepull: (device buffer, event)

    # ------------------------------------------------------------------ capture
    def warmup(self, capture: bool = True) -> None:
        """Run every bucket eagerly once (kernel load / autotune caches), then capture graphs."""
        with torch.cuda.device(self.device), torch.no_grad():
            # the model's construction (weight packing, folding) ran on the default stream; the
            # slot streams do not wait for it on their own
            torch.cuda.synchronize(self.device)
            for slot in self.slots:
                for b in self.buckets:
                    with torch.cuda.stream(slot.s_comp):
                        outs = self.forward(slot.dev_in[:b])
                    slot.s_comp.synchronize()
                    if not (self.use_graphs and capture):
                        slot.outs[b] = tuple(outs)
                    self._alloc_host_out(slot, b, outs)
            if self.use_graphs and capture:
                torch.cuda.synchronize(self.device)
                for slot in self.slots:
                    for b in self.buckets:
                        g = torch.cuda.CUDAGraph()
                        # MLS_GRAPH_COPIES=1: the slot's H2D and D2H copies ride inside its graph
                        # (memcpy nodes from / to its pinned buffers): one replay call per batch,
                        # 81 -> 45 us of host enqueue -- but the in-graph copies run slower than the
                        # stream copies (one batch alone +45 us) and the 20-step bench drops
                        # 48.3-48.6k -> 45.1-45.5k (profiles/r4_engine_graph_copies_ab.jsonl): off
                        in_graph = self.graph_copies
                        # thread_local: the RCCL watchdog thread (DP ranks keep a process group for
                        # X1 / X6) queries its events concurrently; under the default global mode
                        # that query is an illegal call during capture and aborts the process
                        with torch.cuda.graph(g, pool=slot.pool, stream=slot.s_comp,
                                              capture_error_mode="thread_local"):
                            if in_graph:
                                slot.dev_in[:b].copy_(slot.host_in[:b], non_blocking=True)
                            # the copy kernel moves whole 16-B units: other input sizes keep the copy
                            pull = (bool(self.pull_h2d) and not in_graph
                                    and (slot.host_in[:b].numel() * slot.host_in.element_size()) % 16 == 0)
                            if pull:
                                from .. import ops

                                # the source address comes from the slot's pinned cell at run time,
                                # so a pre-staged batch is pulled straight from its own buffer
                                ops.h2d_pull_cell(slot.src_cell, slot.host_in[:b].numel() * slot.host_in.element_size(),
                                                  slot.dev_in[:b], self.pull_grid)
                            outs = self.forward(slot.dev_in[:b])
                            # ... and the results pushed to the pinned host buffers by a kernel at the
                            # graph's end (no SDMA D2H either), when every output is a 16-B multiple
                            push = pull and all(
                                d.is_contiguous() and (d.numel() * d.element_size()) % 16 == 0 for d in outs)
                            if push:
                                for h, d in zip(slot.host_out[b], outs):
                                    ops.d2h_push(d, h)
                            if in_graph:
                                for h, d in zip(slot.host_out[b], outs):
                                    h.copy_(d, non_blocking=True)
                        slot.graphs[b] = g
                        slot.outs[b] = tuple(outs)
                        slot.graph_copies[b] = in_graph
                        slot.pulled[b] = pull
                        slot.pushed[b] = push
                        if self.native_launch:
                            self._prepare_native(slot, b)
                torch.cuda.synchronize(self.device)
                logger.info("%s: captured %d hipGraphs (%d slots x buckets %s)", self.name,
                            len(self.slots) * len(self.buckets), len(self.slots), self.buckets)
            self._prewarm_copies(int(os.environ.get("MLS_COPY_PREWARM", "0")))

    def _prewarm_copies(self, rounds: int) -> None:
        """``rounds`` x (H2D of every slot's whole input buffer + its D2H copies) on the slot streams
        (A/B of the copy-engine warm-up, tools/probe/r5_sdma_ab2.sh)."""
        if rounds <= 0:
            return
        with torch.cuda.device(self.device):
            for _ in range(rounds):
                for slot in self.slots:
                    with torch.cuda.stream(slot.s_comp):
                        slot.dev_in.copy_(slot.host_in, non_blocking=True)
                        for b in self.buckets:
                            for h, d in zip(slot.host_out.get(b, ()), slot.outs.get(b, ())):
                                h.copy_(d, non_blocking=True)
            torch.cuda.synchronize(self.device)

    def _prepare_native(self, slot: _Slot, b: int) -> None:
        """The mls_engine_launch argument tuple of (slot, bucket): raw stream / buffer / graph-exec /
        event handles, all persistent for the engine's lifetime (built once, reused every batch)."""
        import ctypes

        try:
            from .. import ops

            lib = ops.lib()
            # called through the CDLL handle: the GIL is released for the call, so a serving
            # process's front-end / waiter threads run meanwhile.  Round 4 held it (PyDLL) after 2
            # of 19 20-step runs stalled ~6 ms with it released; round 5 found those stalls in the
            # SDMA H2D copy itself, with the GIL held as well (docs/PERF_NOTES.md, round 5) -- the
            # engine no longer uses SDMA (pull_h2d).  MLS_ENQUEUE_HOLD_GIL=1 keeps the PyDLL form.
            hold = os.environ.get("MLS_ENQUEUE_HOLD_GIL", "0") == "1"
            fn = getattr(ctypes.PyDLL(lib._name) if hold else lib, "mls_engine_launch_after")
            fn.argtypes = lib.mls_engine_launch_after.argtypes
            fn.restype = lib.mls_engine_launch_after.restype
            exec_h = slot.graphs[b].raw_cuda_graph_exec()
            slot.ev_done.record(slot.s_comp)  # torch creates the event lazily: make it exist
            ev = slot.ev_done.cuda_event
            outs, hosts = slot.outs[b], slot.host_out[b]
            n = 0 if slot.pushed.get(b) else len(outs)  # pushed by the graph itself
            dst = (ctypes.c_void_p * max(n, 1))(*[h.data_ptr() for h in hosts[:n]])
            src = (ctypes.c_void_p * max(n, 1))(*[d.data_ptr() for d in outs[:n]])
            nb = (ctypes.c_longlong * max(n, 1))(*[d.numel() * d.element_size() for d in outs[:n]])
            h2d = slot.host_in[:b]
            t_ns = (ctypes.c_longlong * 5)()  # per-call host times of the last enqueue (diagnostics)
            h2d_bytes = 0 if slot.pulled.get(b) else h2d.numel() * h2d.element_size()  # pulled in the graph
            # (the first argument: an event the slot's stream waits for first -- a prepulled batch's pull)
            args = (None, slot.s_comp.cuda_stream, slot.dev_in.data_ptr(), slot.host_in.data_ptr(),
                    h2d_bytes, exec_h, n, dst, src, nb, ev, t_ns)
            if not exec_h or not ev:
                raise RuntimeError("graph exec / event handle unavailable")
            slot.native[b] = (fn, args, (dst, src, nb, t_ns))  # keep the arrays alive
        except Exception as e:  # noqa: BLE001 - keep the Python enqueue
            logger.warning("%s: native launch unavailable (%s); Python enqueue", self.name, e)
            self.native_launch = False
            slot.native.clear()

    def _alloc_host_out(self, slot: _Slot, b: int, outs) -> None:
        slot.host_out[b] = tuple(torch.empty(o.shape, dtype=o.dtype, pin_memory=True) for o in outs)

    # ------------------------------------------------------------------ run
    def submit(self, samples) -> Ticket:
        """Enqueue a batch.  ``samples``: a numpy array ``[n, *sample_shape]`` or a sequence of
        per-request arrays of ``sample_shape``.  Returns immediately with a :class:`Ticket`."""
        n = len(samples)
        if n == 0:
            raise ValueError("empty batch")
        pick_bucket(n, self.buckets)  # validate before taking a slot
        t0 = time.perf_counter()
        slot = self._free.get()  # blocks while `inflight` batches are outstanding
        t1 = time.perf_counter()
        try:
            with tracing.range(self._tr_stage):
                dst = slot.host_in.numpy() if self.sample_dtype != torch.bfloat16 else None
                if isinstance(samples, np.ndarray):
                    dst[:n] = samples
                elif isinstance(samples, torch.Tensor):
                    slot.host_in[:n].copy_(samples)
                elif dst is not None:
                    self._stager.gather(dst, samples)
                else:
                    for i, s in enumerate(samples):
                        dst[i] = s
        except BaseException as e:
            self._free.put(slot)
            self.last_error = f"{type(e).__name__}: {e}"
            raise
        t2 = time.perf_counter()
        tk = self.launch(slot, n)
        # host phases of this submit (slot wait, staging copy, enqueue): diagnostics for the bench's
        # ticket log (MLS_BENCH_TICKETS), e.g. to place a multi-ms host stall
        tk.stamps = (t0, t1, t2, time.perf_counter())
        return tk

    def prepare(self, samples) -> Prepared:
        """Stage a batch into a spare pinned buffer without taking a slot (blocks only while every
        spare buffer is held by an unfinished prepared batch)."""
        n = len(samples)
        if n == 0:
            raise ValueError("empty batch")
        pick_bucket(n, self.buckets)
        t0 = time.perf_counter()
        with self._spare_lock:
            if not self._spare_made:
                for _ in range(self.inflight + 1):
                    self._spare.put(torch.zeros((self.max_batch, *self.sample_shape), dtype=self.sample_dtype,
                                                pin_memory=True))
                if self.prepull:
                    for _ in range(self.inflight + 2):
                        self._dev_spare.put((torch.empty((self.max_batch, *self.sample_shape), dtype=self.sample_dtype,
                                                         device=self.device), torch.cuda.Event()))
                self._spare_made = True
        buf = self._spare.get()
        try:
            with tracing.range(self._tr_stage):
                dst = buf.numpy() if self.sample_dtype != torch.bfloat16 else None
                if isinstance(samples, np.ndarray):
                    dst[:n] = samples
                elif isinstance(samples, torch.Tensor):
                    buf[:n].copy_(samples)
                elif dst is not None:
                    self._stager.gather(dst, samples)
                else:
                    for i, x in enumerate(samples):
                        dst[i] = x
        except BaseException:
            self._spare.put(buf)
            raise
        prep = Prepared(buf, n, t0)
        if self.prepull:
            self._pull_early(prep)
        return prep

    def _pull_early(self, prep: Prepared) -> None:
        """prepull: the staged batch goes to a spare device buffer now, on the I/O stream (the
        bucket's rows: the graph copies exactly those); its event orders the slot's graph after it."""
        from .. import ops

        b = pick_bucket(prep.n, self.buckets)
        d = self._dev_spare.get()
        try:
            with torch.cuda.device(self.device), torch.cuda.stream(self.s_io):
                ops.h2d_pull(prep.buf[:b], d[0][:b], self.pull_h2d)
                d[1].record(self.s_io)
        except BaseException:
            self._dev_spare.put(d)
            raise
        prep.dev = d

    def launch_prepared(self, prep: Prepared) -> Ticket:
        """Take a free slot (blocking) and enqueue a :meth:`prepare`-d batch: H2D from its buffer."""
        slot = self._free.get()
        return self.launch(slot, prep.n, staged=prep)

    # -- zero-copy path: the caller fills the slot's pinned buffer itself (native front end) --
    def acquire(self, timeout: Optional[float] = None) -> Optional[_Slot]:
        """Take a free slot (``None`` on timeout); fill ``host_buffer(slot)[:n]`` then :meth:`launch`
        it, or hand it back with :meth:`release`."""
        try:
            return self._free.get(timeout=timeout)
        except queue.Empty:
            return None

    def release(self, slot: _Slot) -> None:
        self._free.put(slot)

    @contextlib.contextmanager
    def quiesce(self, timeout: Optional[float] = 120.0):
        """Hold every slot: in-flight batches finish first, new ones wait until the block exits
        (hot weight reload -- the captured graphs read the weights in place)."""
        held: List[_Slot] = []
        try:
            deadline = None if timeout is None else time.monotonic() + timeout
            while len(held) < len(self.slots):
                left = None if deadline is None else max(0.0, deadline - time.monotonic())
                try:
                    held.append(self._free.get(timeout=left))
                except queue.Empty:
                    raise TimeoutError(f"{self.name}: in-flight batches did not drain") from None
            torch.cuda.synchronize(self.device)
            yield
            torch.cuda.synchronize(self.device)
        finally:
            for sl in held:
                self._free.put(sl)

    @staticmethod
    def host_buffer(slot: _Slot) -> np.ndarray:
        """The slot's pinned host input as a writable numpy view ``[max_batch, *sample_shape]``."""
        return slot.host_in.numpy()

    def launch(self, slot: _Slot, n: int, staged: Optional[Prepared] = None) -> Ticket:
        """Enqueue H2D -> graph replay -> D2H for the first ``n`` rows already in the slot's pinned
        buffer (or in ``staged``'s buffer).  Consumes the slot (returned to the free list by
        :meth:`Ticket.wait`)."""
        src_host = slot.host_in if staged is None else staged.buf
        try:
            bucket = pick_bucket(n, self.buckets)
            nat = slot.native.get(bucket) if self.native_launch and not tracing.active() else None
            if nat is not None:
                pulled = slot.pulled.get(bucket)
                early = pulled and staged is not None and staged.dev is not None
                if early:  # already on the device: the graph's copy reads it there, all workgroups
                    slot.cell_np[0] = staged.dev[0].data_ptr()
                    slot.cell_np[1] = 0
                elif pulled:  # the graph pulls from the address in the slot's cell: no host copy
                    slot.cell_np[0] = src_host.data_ptr()
                    slot.cell_np[1] = self.pull_h2d
                with self._enqueue_lock:
                    self._pace_launch()
                    fn, args, _keep = nat
                    if early:  # the slot's stream first waits for the early pull
                        args = (staged.dev[1].cuda_event,) + args[1:]
                    elif staged is not None and not pulled:  # same call, H2D from the prepared buffer
                        args = args[:3] + (staged.buf.data_ptr(),) + args[4:]
                    rc = fn(*args)
                if rc != 0:
                    raise RuntimeError(f"mls_engine_launch failed (HIP error {rc})")
                tk = Ticket(self, slot, bucket, n, staged)
                t_ns = _keep[3]
                tk.launch_ns = tuple(t_ns[i + 1] - t_ns[i] for i in range(4))
                return tk
            with self._enqueue_lock, torch.cuda.device(self.device):
                self._pace_launch()
                if self.use_graphs and slot.graph_copies.get(bucket):
                    # H2D -> forward -> D2H in one replay on the slot stream (the graph reads the
                    # slot's own pinned buffer: a prepared batch is copied into it first)
                    if staged is not None:
                        slot.host_in[:n].copy_(staged.buf[:n])
                    with tracing.range(self._tr_replay), torch.cuda.stream(slot.s_comp):
                        slot.graphs[bucket].replay()
                        slot.ev_done.record(slot.s_comp)
                    return Ticket(self, slot, bucket, n, staged)
                s_h2d = slot.s_comp if self.copies_on_slot_stream else self.s_h2d
                s_d2h = slot.s_comp if self.copies_on_slot_stream else self.s_d2h
                pulled = self.use_graphs and bucket in slot.graphs and slot.pulled.get(bucket, False)
                early = pulled and staged is not None and staged.dev is not None
                if early:  # pulled to the device already: the graph copies it from there
                    slot.cell_np[0] = staged.dev[0].data_ptr()
                    slot.cell_np[1] = 0
                    slot.s_comp.wait_event(staged.dev[1])
                elif pulled:  # the graph pulls from the address in the slot's cell
                    slot.cell_np[0] = src_host.data_ptr()
                    slot.cell_np[1] = self.pull_h2d
                with tracing.range(self._tr_h2d), torch.cuda.stream(s_h2d):
                    if not pulled:
                        slot.dev_in[:bucket].copy_(src_host[:bucket], non_blocking=True)
                    slot.ev_h2d.record(s_h2d)
                slot.s_comp.wait_event(slot.ev_h2d)
                with tracing.range(self._tr_replay), torch.cuda.stream(slot.s_comp):
                    if self.use_graphs and bucket in slot.graphs:
                        slot.graphs[bucket].replay()
                        outs = slot.outs[bucket]
                    else:
                        with torch.no_grad():
                            outs = tuple(self.forward(slot.dev_in[:bucket]))
                        slot.outs[bucket] = outs
                        if bucket not in slot.host_out:
                            self._alloc_host_out(slot, bucket, outs)
                    slot.ev_comp.record(slot.s_comp)
                s_d2h.wait_event(slot.ev_comp)
                pushed = self.use_graphs and bucket in slot.graphs and slot.pushed.get(bucket, False)
                with tracing.range(self._tr_d2h), torch.cuda.stream(s_d2h):
                    if not pushed:  # a pushing graph already wrote its results to the pinned buffers
                        for h, d in zip(slot.host_out[bucket], outs):
                            h.copy_(d, non_blocking=True)
                    slot.ev_done.record(s_d2h)
        except BaseException as e:
            self._free.put(slot)
            if staged is not None:
                self._spare.put(staged.buf)
                if staged.dev is not None:
                    self._dev_spare.put(staged.dev)
            self.last_error = f"{type(e).__name__}: {e}"
            raise
        return Ticket(self, slot, bucket, n, staged)

    def _pace_launch(self) -> None:
        """Called under the enqueue lock, with this batch's slot already taken."""
        gap = self._fixed_gap_s or (self._pace * self._lat_s / self.inflight if self.inflight > 1 else 0.0)
        busy_others = self.inflight - self._free.qsize() - 1
        # only near saturation: at light load a launch never waits
        if gap > 0 and busy_others >= self._pace_min_busy:
            wait_until = self._last_launch + min(gap, 5e-3)
            while time.perf_counter() < wait_until:
                time.sleep(0)  # yield the GIL; sleeping for real overshoots by 0.1-1 ms
        self._last_launch = time.perf_counter()

    def _note_done(self, t: "Ticket") -> None:
        """Latency EWMA for pacing.  The first pipeline turn after start-up is skipped (first
        launches of freshly captured graphs can take many times the steady latency), and a
        sample counts at most twice the current estimate, so one slow batch cannot make the
        gap throttle the next dozen launches."""
        with self._pace_lock:
            lat = time.perf_counter() - t.t_submit
            self._lat_n += 1
            if self._lat_n <= self.inflight:
                return
            if self._lat_s == 0.0:
                self._lat_s = lat
            else:
                self._lat_s = 0.9 * self._lat_s + 0.1 * min(lat, 2.0 * self._lat_s)

    def _finish(self, t: Ticket) -> Tuple[np.ndarray, ...]:
        slot = t.slot
        try:
            try:
                with tracing.range(self._tr_wait):
                    if self._spin_us > 0:  # poll first: a blocking-sync wake-up costs tens of us
                        end = time.perf_counter() + self._spin_us * 1e-6
                        while not slot.ev_done.query() and time.perf_counter() < end:
                            pass
                    slot.ev_done.synchronize()
                if self._pace > 0 and self.inflight > 1:
                    self._note_done(t)
            except RuntimeError as e:  # device fault surfaced at the sync: this worker is dead
                self.healthy = False
                self.last_error = f"{type(e).__name__}: {e}"
                raise
            res = []
            for h in slot.host_out[t.bucket]:
                if h.dtype == torch.bfloat16:
                    res.append(h[: t.n].float().numpy().copy())
                else:
                    res.append(h[: t.n].numpy().copy())
            self.batches += 1
            self.samples += t.n
            self.busy_s += time.perf_counter() - t.t_submit
            return tuple(res)
        finally:
            if t.staged is not None:  # its H2D is done (the batch completed): reusable
                self._spare.put(t.staged.buf)
                if t.staged.dev is not None:
                    self._dev_spare.put(t.staged.dev)
                t.staged = None
            self._free.put(slot)

    def run(self, samples) -> Tuple[np.ndarray, ...]:
        return self.submit(samples).wait()

    def stats(self) -> dict:
        return {"name": self.name, "device": str(self.device), "batches": self.batches, "samples": self.samples,
                "inflight": self.inflight, "buckets": self.buckets, "graphs": self.use_graphs,
                "concurrent": self.concurrent, "cu_partitions": self.cu_partitions, "prepull": self.prepull,
                "native_staging": self._stager.native,
                "pace_gap_us": round(self._pace * self._lat_s / max(1, self.inflight) * 1e6, 1),
                "healthy": self.healthy, "last_error": self.last_error,
                "free_slots": self._free.qsize()}
