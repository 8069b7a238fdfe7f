"""Bind a GPU worker process to the CPUs of its GPU's NUMA node.

One process per GPU on a 2-socket MI355X node: the engine's host side (pinned staging slots,
the request memcpy threads, H2D submission) should live on the socket the GPU's PCIe root hangs
off, or every batch's 4.8 MB of pixels crosses the inter-socket link twice (memcpy into the
pinned slot, then the H2D DMA).  torchrun does not pin; this reads the GPU's PCI address from the
runtime, the node's CPU list from sysfs, and restricts the calling thread (threads created later
-- the engine's staging pool -- inherit it) to that list intersected with the CPUs the process
may use.  Call before allocating pinned memory so first-touch places it on the local node.

``MLS_NUMA_BIND=0`` disables; ``=1`` forces it for single-process runs (default: only with
several ranks, where it matters).
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


def bind_to_gpu(device_index: int, world_size: int = 1, sysfs_root: str = "/sys",
                pci_addr: Optional[str] = None) -> Optional[List[int]]:
    """Restrict this process's (calling thread's) CPU affinity to the GPU's local CPUs.
    Returns the CPU list applied, or None when binding is disabled / impossible."""
    mode = os.environ.get("MLS_NUMA_BIND", "")
    if mode == "0" or (mode != "1" and world_size <= 1):
        return None
    addr = pci_addr or pci_address(device_index)
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
    try:
        os.sched_setaffinity(0, cpus)
    except OSError as e:
        logger.warning("could not bind to GPU %d's CPUs: %s", device_index, e)
        return None
    logger.info("GPU %d (%s): bound to %d local CPUs", device_index, addr, len(cpus))
    return cpus
