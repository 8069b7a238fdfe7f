"""CU-masked streams and the spatial partitions of the in-flight batches (census-verified masks)."""
from __future__ import annotations

import ctypes
from typing import Dict, List, Optional, Sequence

import torch

from ._lib import check, lib


MASK_WORDS = 8  # 256 CUs


_MASKED_STREAMS: Dict[tuple, torch.cuda.ExternalStream] = {}


_MASKED_LOCK = __import__("threading").Lock()
_ATEXIT_SET = False


def release_masked_streams(key=None) -> None:
    """Synchronize and destroy the pooled CU-masked streams (all of them, or those created with
    ``key``); registered with ``atexit`` when the first one is created: the HIP runtime otherwise
    tears them down in its static destructors, after a profiler's tool library has finalized --
    ``rocprofv3`` runs of the partitioned bench segfaulted in ``__cxa_finalize`` after writing their
    output (rc 0 with this; ``tools/probe/r5_exit.sh``).  Engines still holding a released stream
    must not run again."""
    with _MASKED_LOCK:
        ks = [k for k in _MASKED_STREAMS if key is None or k[2] == key]
        streams = [_MASKED_STREAMS.pop(k) for k in ks]
    for st in streams:
        try:
            st.synchronize()
            lib().mls_stream_destroy(st.cuda_stream)
        except Exception:  # noqa: BLE001 -- best effort at interpreter exit
            pass


def cu_masked_stream(mask: Sequence[int], device=None, key=0) -> torch.cuda.ExternalStream:
    """The HIP stream restricted to the CUs whose bits are set in ``mask`` (``MASK_WORDS`` uint32
    words; csrc/partition.hip) -- one per (device, mask, ``key``), created on first use and kept
    for the process.  Every masked stream holds a hardware queue of its own, so they are pooled:
    engines built one after another reuse them (``key`` tells apart the streams one engine needs
    on the same mask) instead of piling up queues until queue creation fails."""
    import ctypes

    dev = torch.device(device if device is not None else "cuda")
    if dev.index is None:
        dev = torch.device("cuda", torch.cuda.current_device())
    ck = (dev.index, tuple(int(m) & 0xFFFFFFFF for m in mask), key)
    with _MASKED_LOCK:
        st = _MASKED_STREAMS.get(ck)
        if st is None:
            words = (ctypes.c_uint32 * len(mask))(*ck[1])
            out = ctypes.c_void_p()
            with torch.cuda.device(dev):
                check(lib().mls_stream_create_cumask(ctypes.cast(words, ctypes.c_void_p), len(mask),
                                                     ctypes.byref(out)), "mls_stream_create_cumask")
            st = _MASKED_STREAMS[ck] = torch.cuda.ExternalStream(out.value, device=dev)
            global _ATEXIT_SET
            if not _ATEXIT_SET:
                import atexit

                atexit.register(release_masked_streams)
                _ATEXIT_SET = True
        return st


class _TempMaskedStream:
    """A CU-masked stream for one census only: created outside the serving pool and destroyed
    (``mls_stream_destroy``) when the census is done, so a partitioned process keeps only the
    engine's masked streams (each holds one of the 4 hardware queues)."""

    def __init__(self, mask: Sequence[int], dev: torch.device):
        import ctypes

        words = (ctypes.c_uint32 * len(mask))(*[int(m) & 0xFFFFFFFF for m in mask])
        out = ctypes.c_void_p()
        with torch.cuda.device(dev):
            check(lib().mls_stream_create_cumask(ctypes.cast(words, ctypes.c_void_p), len(mask), ctypes.byref(out)),
                  "mls_stream_create_cumask")
        self.handle = out.value
        self.stream = torch.cuda.ExternalStream(out.value, device=dev)

    def __enter__(self) -> torch.cuda.ExternalStream:
        return self.stream

    def __exit__(self, *exc) -> None:
        self.stream.synchronize()
        check(lib().mls_stream_destroy(self.handle), "mls_stream_destroy")


def cu_census(stream: torch.cuda.Stream, blocks: int = 2048, spin: int = 64) -> torch.Tensor:
    """(XCC_ID, HW_ID) of the CU each of ``blocks`` blocks ran on, launched on ``stream``: int32 [blocks, 2]."""
    out = torch.full((blocks, 2), -1, device=stream.device, dtype=torch.int32)
    with torch.cuda.stream(stream):
        check(lib().mls_cu_census(out.data_ptr(), blocks, spin, stream.cuda_stream), "mls_cu_census")
    stream.synchronize()
    return out.cpu()


_XCD_MASKS: Dict[int, Optional[List[List[int]]]] = {}


def xcd_cu_masks(device=None) -> Optional[List[List[int]]]:
    """Per XCD, the CU-mask words that select exactly that XCD's CUs, verified on the device with
    :func:`cu_census` (every block of a masked stream must report one XCC id, and the 8 masks 8
    distinct ids).  Logical mask bit ``b`` is tried as XCD ``b % 8`` (round-robin) and as
    ``b // 32`` (contiguous); ``None`` when neither layout verifies."""
    dev = torch.device(device if device is not None else "cuda")
    key = dev.index if dev.index is not None else torch.cuda.current_device()
    if key in _XCD_MASKS:
        return _XCD_MASKS[key]
    ncu = torch.cuda.get_device_properties(dev).multi_processor_count
    result = None
    if ncu == 256:
        for layout in ("roundrobin", "contiguous"):
            masks = []
            for x in range(8):
                bits = [b for b in range(ncu) if (b % 8 if layout == "roundrobin" else b // 32) == x]
                w = [0] * MASK_WORDS
                for b in bits:
                    w[b // 32] |= 1 << (b % 32)
                masks.append(w)
            ids = []
            for w in masks:
                with _TempMaskedStream(w, dev) as st:
                    c = cu_census(st, blocks=256)
                ids.append(set(c[:, 0].tolist()))
            if all(len(s) == 1 for s in ids) and len(set().union(*ids)) == 8:
                result = masks
                break
    _XCD_MASKS[key] = result
    return result


def census_cus(c: torch.Tensor) -> set:
    """Distinct physical CUs in a :func:`cu_census` result: (XCC, SE, SH, CU) from HW_ID bits 8-15."""
    return {(int(x), (int(h) >> 8) & 0xFF) for x, h in c.tolist()}


def intra_partition_words(parts: int, ncu: int = 256, mode: str = "intra", xccs: int = 8) -> List[List[int]]:
    """The CU-mask words of ``parts`` intra-XCD partitions (pure; verified on the device by
    :func:`partition_masks`).  Mask bit ``b`` is CU ``b // xccs`` of XCC ``b % xccs`` (census:
    profiles/r3_cu_mask_census.txt); an XCC left without a bit runs on ALL its CUs, so every
    partition keeps ``ncu / xccs / parts`` CUs on every XCC: CU ``c`` goes to partition ``c %
    parts`` (``"intra"``) or ``c // (ncu / xccs / parts)`` (``"intra_contig"``)."""
    per_xcc = ncu // xccs
    if parts <= 0 or per_xcc % parts or mode not in ("intra", "intra_contig"):
        raise ValueError(f"{parts} {mode} partitions of {per_xcc} CUs per XCC")
    out = []
    for p in range(parts):
        w = [0] * max(MASK_WORDS, (ncu + 31) // 32)
        for b in range(ncu):
            c = b // xccs
            if (c % parts if mode == "intra" else c // (per_xcc // parts)) == p:
                w[b // 32] |= 1 << (b % 32)
        out.append(w)
    return out


_PARTITION_MASKS: Dict[tuple, Optional[List[List[int]]]] = {}


def partition_masks(parts: int, device=None, mode: str = "xcd") -> Optional[List[List[int]]]:
    """Cached :func:`_partition_masks` (the census verification runs once per device / mode / parts)."""
    dev = torch.device(device if device is not None else "cuda")
    ck = (dev.index if dev.index is not None else torch.cuda.current_device(), parts, mode)
    if ck not in _PARTITION_MASKS:
        _PARTITION_MASKS[ck] = _partition_masks(parts, dev, mode)
    return _PARTITION_MASKS[ck]


def _partition_masks(parts: int, device=None, mode: str = "xcd") -> Optional[List[List[int]]]:
    """``parts`` (1, 2, 4 or 8) CU masks.  ``mode="xcd"``: each the union of 8 / parts whole XCDs
    (needs :func:`xcd_cu_masks`).  ``mode="intra"``: each a 1 / parts share of the CUs of EVERY
    XCD (CU ``c`` of every XCC with ``c % parts == p``; ``"intra_contig"``: ``c // (32 / parts) ==
    p``), verified by census to select disjoint CU sets of the expected size."""
    if parts not in (1, 2, 4, 8):
        raise ValueError("parts must be 1, 2, 4 or 8")
    if mode in ("intra", "intra_contig"):
        dev = torch.device(device if device is not None else "cuda")
        ncu = torch.cuda.get_device_properties(dev).multi_processor_count
        out, seen = [], set()
        for p, w in enumerate(intra_partition_words(parts, ncu, mode)):
            with _TempMaskedStream(w, dev) as st:
                cus = census_cus(cu_census(st, blocks=4096))
            if len(cus) > ncu // parts or cus & seen:
                return None
            seen |= cus
            out.append(w)
        return out
    xm = xcd_cu_masks(device)
    if xm is None:
        return None
    per = 8 // parts
    out = []
    for p in range(parts):
        w = [0] * MASK_WORDS
        for x in range(p * per, (p + 1) * per):
            w = [a | b for a, b in zip(w, xm[x])]
        out.append(w)
    return out
