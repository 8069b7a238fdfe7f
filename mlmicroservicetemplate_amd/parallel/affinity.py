"""Bind a GPU worker process to the CPUs of its GPU's NUMA node.

One process per GPU on a 2-socket MI355X node: the engine's host side (pinned staging slots,
the request memcpy threads, H2D submission) should live on the socket the GPU's PCIe root hangs
off, or every batch's 4.8 MB of pixels crosses the inter-socket link twice (memcpy into the
pinned slot, then the H2D DMA).  torchrun does not pin; this reads the GPU's PCI address from the
runtime, the node's CPU list from sysfs, and restricts the calling thread (threads created later
-- the engine's staging pool -- inherit it) to that list intersected with the CPUs the process
may use.  Call before allocating pinned memory so first-touch places it on the local node.

``MLS_NUMA_BIND=0`` disables, ``=1`` forces it.  By default every rank binds -- a single-rank
run too, provided the GPU-local CPUs it may use number at least :data:`SINGLE_RANK_MIN_CPUS` (or
all it may use), so a small CPU share on the far socket is not shrunk further.  Single-rank A/B
on one MI355X (profiles/r6_numa_bind_single_rank_ab.jsonl): bound 53.1k vs 52.7k req/s mean over
5 paired 20-step runs (4 of 5 pairs ahead), 57.1k vs 56.8k at 200 steps.

Host-thread budget: on an 8-GPU node four ranks share each socket's CPUs, and every rank's
engine would otherwise start 4 staging copy threads regardless (plus the submitting thread, the
Python loop and HIP's own threads).  :func:`bind_to_gpu` also records how many CPUs this rank
may use and how many local ranks share them; :func:`stage_threads_hint` turns that into the
engine's copy-thread count (``engine/staging.HostStager``'s default).
"""
from __future__ import annotations

import logging
import os
from typing import List, Optional, Set

logger = logging.getLogger("mlsamd.affinity")


def parse_cpulist(text: str) -> List[int]:
    """``"0-3,8,10-11"`` -> ``[0, 1, 2, 3, 8, 10, 11]``."""
    cpus: List[int] = []
    for part in text.strip().split(","):
        part = part.strip()
        if not part:
            continue
        if "-" in part:
            lo, hi = part.split("-", 1)
            cpus.extend(range(int(lo), int(hi) + 1))
        else:
            cpus.append(int(part))
    return cpus


def pci_address(device_index: int) -> Optional[str]:
    try:
        import torch

        p = torch.cuda.get_device_properties(device_index)
        return f"{int(p.pci_domain_id):04x}:{int(p.pci_bus_id):02x}:{int(p.pci_device_id):02x}.0"
    except Exception:
        return None


def gpu_local_cpus(pci_addr: str, sysfs_root: str = "/sys") -> Optional[Set[int]]:
    base = os.path.join(sysfs_root, "bus", "pci", "devices", pci_addr)
    try:
        with open(os.path.join(base, "local_cpulist")) as f:
            cpus = set(parse_cpulist(f.read()))
    except OSError:
        return None
    return cpus or None


SINGLE_RANK_MIN_CPUS = 8  # a default single-rank bind keeps at least this many CPUs (or all allowed)
STAGE_THREADS_CAP = 4  # copy threads that saturate one batch's memcpy (docs/PERF_NOTES.md, round 2)
# a copy thread's memcpy rate into pinned memory with 8 ranks copying at once: the 8-process CPU
# staging test measured 3.5-8.7 GB/s per instance (profiles/r4_staging_8_rank_processes_cpu.txt);
# the plan below budgets the low end per thread
COPY_GBPS_PER_THREAD = 3.5
_hint: Optional[int] = None
_plan: Optional[dict] = None


def stage_thread_budget(n_cpus: int, ranks_sharing: int, cap: int = STAGE_THREADS_CAP) -> int:
    """Staging copy threads for one rank: its share of the CPUs it may use (``n_cpus`` shared by
    ``ranks_sharing`` local ranks) minus one for the submitting thread (which copies too), at
    least 1 and at most ``cap``."""
    share = max(1, int(n_cpus)) // max(1, int(ranks_sharing))
    return max(1, min(int(cap), share - 1))


def ranks_sharing_cpus(device_index: int, local_world: int, sysfs_root: str = "/sys",
                       pci_of=None) -> int:
    """How many of the node's ``local_world`` ranks (rank r drives GPU ``r % ngpus``) have
    their GPU on the same NUMA node as ``device_index`` -- i.e. share its local CPU list.  Unknown
    topology: all of them."""
    pci_of = pci_of or pci_address
    mine_addr = pci_of(device_index)
    mine = gpu_local_cpus(mine_addr, sysfs_root) if mine_addr else None
    if not mine:
        return max(1, local_world)
    try:
        import torch

        ngpu = max(1, torch.cuda.device_count())
    except Exception:
        ngpu = 1
    if pci_of is not pci_address:  # an explicit map (tests): one GPU per local rank
        ngpu = max(1, local_world)
    n = 0
    for r in range(max(1, local_world)):
        addr = pci_of(r % ngpu)
        cpus = gpu_local_cpus(addr, sysfs_root) if addr else None
        n += 1 if cpus == mine else 0
    return max(1, n)


def stage_threads_hint() -> Optional[int]:
    """The copy-thread budget :func:`bind_to_gpu` computed for this process (None: not computed)."""
    return _hint


def host_plan(n_cpus: int, ranks_sharing: int, bytes_per_sample: int = 224 * 224 * 3,
              target_samples_per_s: float = 60000.0, numa_bound: bool = False) -> dict:
    """This rank's host-side budget: staging copy threads from its CPU share, the memcpy rate they
    give at :data:`COPY_GBPS_PER_THREAD` each (the submitting thread copies too), against what the
    GPU needs at ``target_samples_per_s`` (ResNet-50 bs=32 on one MI355X: 57k req/s measured x
    150 KB per image = 8.6 GB/s).  ``headroom`` < 1 means the host, not the GPU, would bound this
    rank."""
    threads = stage_thread_budget(n_cpus, ranks_sharing)
    copy = (threads + 1) * COPY_GBPS_PER_THREAD
    need = bytes_per_sample * target_samples_per_s / 1e9
    return {"cpus": int(n_cpus), "ranks_sharing_cpus": int(ranks_sharing), "cpus_per_rank": int(n_cpus) // max(1, int(ranks_sharing)),
            "stage_threads": threads, "copy_gbps_budget": round(copy, 1), "need_gbps": round(need, 2),
            "headroom": round(copy / need, 2) if need > 0 else None, "numa_bound": bool(numa_bound)}


def host_plan_hint() -> Optional[dict]:
    """The plan :func:`bind_to_gpu` computed for this process (None: single rank)."""
    return _plan


def bind_to_gpu(device_index: int, world_size: int = 1, sysfs_root: str = "/sys",
                pci_addr: Optional[str] = None, local_world: Optional[int] = None,
                pci_of=None) -> Optional[List[int]]:
    """Restrict this process's (calling thread's) CPU affinity to the GPU's local CPUs.
    Returns the CPU list applied, or None when binding is disabled / impossible.  With several
    ranks it also sets :func:`stage_threads_hint` from the CPUs left to this rank."""
    global _hint, _plan
    if world_size > 1:
        lw = int(local_world or os.environ.get("LOCAL_WORLD_SIZE", world_size))
        try:
            allowed0 = os.sched_getaffinity(0)
        except (AttributeError, OSError):
            allowed0 = set(range(os.cpu_count() or 1))
        pci_of = pci_of or pci_address
        addr0 = pci_addr or pci_of(device_index)
        local0 = gpu_local_cpus(addr0, sysfs_root) if addr0 else None
        usable = (local0 & allowed0) if local0 and (local0 & allowed0) else allowed0
        sharing = ranks_sharing_cpus(device_index, lw, sysfs_root, pci_of=pci_of) if local0 else lw
        _hint = stage_thread_budget(len(usable), sharing)
        _plan = host_plan(len(usable), sharing, numa_bound=bool(local0 and (local0 & allowed0)))
        logger.info("GPU %d: %d usable CPUs shared by %d local ranks -> %d staging threads (%s)", device_index,
                    len(usable), sharing, _hint, _plan)
    mode = os.environ.get("MLS_NUMA_BIND", "")
    if mode == "0":
        return None
    addr = pci_addr or (pci_of or pci_address)(device_index)
    if addr is None:
        return None
    local = gpu_local_cpus(addr, sysfs_root)
    if not local:
        return None
    try:
        allowed = os.sched_getaffinity(0)
    except (AttributeError, OSError):
        return None
    cpus = sorted(local & allowed)
    if not cpus or set(cpus) == allowed:
        return None
    if mode != "1" and world_size <= 1 and len(cpus) < min(SINGLE_RANK_MIN_CPUS, len(allowed)):
        logger.info("GPU %d: only %d of %d allowed CPUs are local; not binding a single rank", device_index,
                    len(cpus), len(allowed))
        return None
    try:
        os.sched_setaffinity(0, cpus)
    except OSError as e:
        logger.warning("could not bind to GPU %d's CPUs: %s", device_index, e)
        return None
    logger.info("GPU %d (%s): bound to %d local CPUs", device_index, addr, len(cpus))
    return cpus
