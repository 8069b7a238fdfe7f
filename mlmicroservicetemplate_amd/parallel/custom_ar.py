"""One-shot IPC all-reduce for tensor-parallel decode (X2).

The kernel lives in ``ops/csrc/custom_allreduce.hip``: every rank reads every peer's staging
buffer over xGMI in one hop (all 7 links at once) instead of RCCL's 2(N-1)-step ring, which
is what an 8 KiB decode message pays for.  This module does the bootstrap -- allocate, export
the IPC handle, all-gather the handles over the existing process group, open the peers -- and
a start-up self-test against the group's own all-reduce.  Anything unexpected (IPC
unavailable, a timeout, a wrong sum) leaves :attr:`CustomAllReduce.enabled` False and callers
keep RCCL.  Messages up to ``two_shot_min`` bytes take the one-shot kernel (every rank reads all
N - 1 peers' copies: (N - 1) x n bytes per rank, one synchronisation); larger ones up to ``cap2``
the two-shot kernel (reduce-scatter + all-gather in one launch: 2 (N - 1) / N x n bytes per rank,
two synchronisations) -- TP decode at 32-256 rows; beyond ``cap2`` RCCL (bandwidth-bound prefill).

``TPComm`` uses it for TP > 1 on GPUs unless ``MLS_CUSTOM_AR=0``.  Being graph-safe, it is also
what lets ``LlamaTP`` capture the TP decode step (RCCL inside graphs stays opt-in,
``MLS_TP_GRAPHS=1``).  Exercised with 8 ranks on one GPU (``tests/test_llama_tp_gpu.py``, world 8:
IPC handles, 8-peer one-shot kernel inside the captured decode graphs); the 8-GPU xGMI timing is
not measured here.
"""
from __future__ import annotations

import ctypes
import logging
import os
from typing import Optional

import torch
import torch.distributed as dist

logger = logging.getLogger("mlsamd.custom_ar")


class CustomAllReduce:
    def __init__(self, group=None, device=None, cap_bytes: int = 1 << 20, self_test: bool = True,
                 timeout_iters: Optional[int] = None, cap2_bytes: Optional[int] = None,
                 two_shot_min: Optional[int] = None):
        from ..ops import _lib

        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        dev = torch.device(device if device is not None else "cuda")
        if dev.index is None:  # "cuda" -> "cuda:<current>": eligible() compares tensor devices exactly
            dev = torch.device("cuda", torch.cuda.current_device())
        self.device = dev
        self.cap = int(cap_bytes)
        # two-shot message range (MLS_AR_TWO_SHOT_CAP=0 disables the path)
        self.cap2 = int(cap2_bytes if cap2_bytes is not None else os.environ.get("MLS_AR_TWO_SHOT_CAP", 4 << 20))
        self.two_shot_min = int(two_shot_min if two_shot_min is not None
                                else os.environ.get("MLS_AR_TWO_SHOT_MIN", 128 << 10))
        self.enabled = False
        self.reason = ""
        self._lib = _lib.lib()
        self._ctx = ctypes.c_void_p()
        # peer-wait bound in spin iterations (~1 s by default); MLS_AR_TIMEOUT_ITERS shrinks it (tests)
        self._timeout = int(timeout_iters if timeout_iters is not None
                            else os.environ.get("MLS_AR_TIMEOUT_ITERS", str(1 << 24)))
        try:
            self._setup()
            if self_test:
                self._self_test()
            self.enabled = True
        except Exception as e:  # keep RCCL
            self.reason = f"{type(e).__name__}: {e}"
            logger.warning("custom all-reduce disabled: %s", self.reason)

    def _setup(self) -> None:
        L = self._lib
        with torch.cuda.device(self.device):
            rc = L.mls_ar_create2(self.rank, self.world, self.cap, self.cap2, ctypes.byref(self._ctx))
            if rc != 0:
                raise RuntimeError(f"mls_ar_create failed ({rc})")
            self.timeout = self._timeout  # into the context too (the GEMM-fused all-reduce's bound)
            hs = L.mls_ar_handle_size()
            mine = (ctypes.c_char * hs)()
            if L.mls_ar_handle(self._ctx, ctypes.cast(mine, ctypes.c_void_p)) != 0:
                raise RuntimeError("hipIpcGetMemHandle failed")
            handles = [None] * self.world
            dist.all_gather_object(handles, bytes(mine), group=self.group)
            blob = (ctypes.c_char * (hs * self.world)).from_buffer_copy(b"".join(handles))
            if L.mls_ar_open(self._ctx, ctypes.cast(blob, ctypes.c_void_p)) != 0:
                raise RuntimeError("hipIpcOpenMemHandle failed")

    def _errors(self) -> int:
        out = ctypes.c_int(0)
        self._lib.mls_ar_error(self._ctx, ctypes.byref(out))
        return out.value

    def _self_test(self) -> None:
        g = torch.Generator().manual_seed(1234 + self.rank)
        ok = True
        sizes = [(n, False) for n in (8, 4096, 4096 * 3 + 8, self.cap // 2)]
        if self.cap2:
            sizes += [(n - n % (8 * self.world), True) for n in (8 * self.world, 100000, self.cap2 // 2)]
        for n, two in sizes:
            x = torch.randn(n, generator=g).to(torch.bfloat16)
            ref = x.float().clone()
            if dist.get_backend(self.group) == "nccl":
                ref = ref.to(self.device)
            dist.all_reduce(ref, group=self.group)  # the group's own backend (RCCL, or gloo on CPU)
            ref = ref.cpu()
            y = self._run2(x.to(self.device)) if two else self._run(x.to(self.device))
            torch.cuda.synchronize(self.device)
            err = (y.float().cpu() - ref).abs().max().item() / (ref.abs().max().item() + 1e-6)
            ok = ok and err < 2e-2
        if self._errors():
            raise RuntimeError("a peer wait timed out during the self-test")
        # every rank must agree before anyone uses the path
        flag = torch.tensor([1 if ok else 0], dtype=torch.int32)
        if dist.get_backend(self.group) == "nccl":
            flag = flag.to(self.device)
        dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=self.group)
        if not int(flag.item()):
            raise RuntimeError("self-test mismatch against the group all-reduce")

    def _run(self, t: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        out = t if out is None else out
        rc = self._lib.mls_ar_allreduce(self._ctx, t.data_ptr(), out.data_ptr(), t.numel(), self.timeout,
                                        torch.cuda.current_stream(self.device).cuda_stream)
        if rc != 0:
            raise RuntimeError(f"mls_ar_allreduce failed ({rc})")
        return out

    def _run2(self, t: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        out = t if out is None else out
        rc = self._lib.mls_ar_allreduce2(self._ctx, t.data_ptr(), out.data_ptr(), t.numel(), self.timeout,
                                         torch.cuda.current_stream(self.device).cuda_stream)
        if rc != 0:
            raise RuntimeError(f"mls_ar_allreduce2 failed ({rc})")
        return out

    def ctx_ptr(self) -> int:
        """The native context (for the GEMMs that fuse this all-reduce: ops.skinny_packed_ar)."""
        return self._ctx.value

    def fusable(self, nelems: int) -> bool:
        """May a GEMM producing ``nelems`` bf16 outputs fuse the one-shot all-reduce of them?"""
        return self.enabled and nelems % 8 == 0 and nelems * 2 <= self.cap and nelems * 2 < self.two_shot_min

    @property
    def timeout(self) -> int:
        """Peer-wait bound (spin iterations) of every one-shot / two-shot wait, the all-reduce
        fused into the decode GEMMs (``ops.skinny_packed_ar``) included."""
        return self._timeout

    @timeout.setter
    def timeout(self, iters: int) -> None:
        self._timeout = int(iters)
        if self._ctx and self._lib.mls_ar_set_timeout(self._ctx, self._timeout) != 0:
            raise RuntimeError("mls_ar_set_timeout failed")

    def errors(self) -> int:
        """Read (and clear) the peer-wait timeout word: non-zero = some one-shot collective since the
        last read completed with a peer missing (its output is partial).  A host sync."""
        return self._errors() if self.enabled or self._ctx else 0

    def error_peek(self, dst: torch.Tensor) -> None:
        """``dst`` (device int32, >= 1 element) <- the error word on the current stream, without
        clearing it: capturable, so a graph reports its collectives' peer timeouts in a read-back
        it makes anyway (the continuous engine's carried-header check)."""
        if dst.dtype != torch.int32 or not dst.is_cuda or dst.numel() < 1:
            raise ValueError("error_peek: dst must be a device int32 tensor")
        rc = self._lib.mls_ar_error_peek(self._ctx, dst.data_ptr(), torch.cuda.current_stream(self.device).cuda_stream)
        if rc != 0:
            raise RuntimeError(f"mls_ar_error_peek failed ({rc})")

    def reset(self) -> None:
        """Restart the device protocol after a timeout (per-block epochs may disagree between ranks):
        collective -- every rank calls it; process-group barriers on both sides guarantee no
        one-shot kernel of the group is in flight while the flags are cleared."""
        from . import dist as mdist

        mdist.barrier(self.group)
        rc = self._lib.mls_ar_reset(self._ctx)
        if rc != 0:
            raise RuntimeError(f"mls_ar_reset failed ({rc})")
        mdist.barrier(self.group)

    def gather_eligible(self, t: torch.Tensor) -> bool:
        nbytes = t.numel() * t.element_size()
        return self.enabled and t.is_contiguous() and t.device == self.device and nbytes % 16 == 0 and nbytes <= self.cap

    def all_gather(self, t: torch.Tensor) -> torch.Tensor:
        """X4 one-shot all-gather: ``[world, *t.shape]`` of every rank's ``t`` (graph-safe)."""
        if not self.gather_eligible(t):
            raise ValueError("tensor not eligible for the one-shot all-gather")
        out = torch.empty((self.world, *t.shape), dtype=t.dtype, device=t.device)
        rc = self._lib.mls_ar_allgather(self._ctx, t.data_ptr(), out.data_ptr(), t.numel() * t.element_size(),
                                        self.timeout, torch.cuda.current_stream(self.device).cuda_stream)
        if rc != 0:
            raise RuntimeError(f"mls_ar_allgather failed ({rc})")
        return out

    def _two_shot(self, t: torch.Tensor) -> bool:
        nbytes = t.numel() * 2
        return (self.cap2 > 0 and nbytes >= self.two_shot_min and nbytes <= self.cap2
                and t.numel() % (8 * self.world) == 0)

    def eligible(self, t: torch.Tensor) -> bool:
        if not (self.enabled and t.dtype == torch.bfloat16 and t.is_contiguous() and t.device == self.device
                and t.numel() % 8 == 0):
            return False
        return self._two_shot(t) or t.numel() * 2 <= self.cap

    def path(self, t: torch.Tensor) -> str:
        """Which kernel :meth:`all_reduce_` runs for ``t``: "two_shot", "one_shot" or "backend"."""
        if not self.eligible(t):
            return "backend"
        return "two_shot" if self._two_shot(t) else "one_shot"

    def all_reduce_(self, t: torch.Tensor) -> torch.Tensor:
        """In-place sum across the group: one-shot for small messages, two-shot for the mid range,
        else the group's backend."""
        p = self.path(t)
        if p == "two_shot":
            return self._run2(t)
        if p == "one_shot":
            return self._run(t)
        dist.all_reduce(t, group=self.group)
        return t

    def close(self) -> None:
        if self._ctx:
            self._lib.mls_ar_destroy(self._ctx)
            self._ctx = ctypes.c_void_p()
            self.enabled = False
