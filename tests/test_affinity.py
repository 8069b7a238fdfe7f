"""NUMA binding of GPU worker processes (parallel/affinity.py) against a fake sysfs."""
import os

import pytest

from mlmicroservicetemplate_amd.parallel.affinity import bind_to_gpu, gpu_local_cpus, parse_cpulist


def test_parse_cpulist():
    assert parse_cpulist("0-3,8,10-11\n") == [0, 1, 2, 3, 8, 10, 11]
    assert parse_cpulist("") == []


def _fake_sysfs(tmp_path, addr, cpulist):
    d = tmp_path / "bus" / "pci" / "devices" / addr
    d.mkdir(parents=True)
    (d / "local_cpulist").write_text(cpulist)
    return str(tmp_path)


def test_gpu_local_cpus(tmp_path):
    root = _fake_sysfs(tmp_path, "0000:05:00.0", "0-1")
    assert gpu_local_cpus("0000:05:00.0", root) == {0, 1}
    assert gpu_local_cpus("0000:06:00.0", root) is None


@pytest.mark.skipif(not hasattr(os, "sched_getaffinity") or len(os.sched_getaffinity(0)) < 2,
                    reason="needs >= 2 usable CPUs")
def test_bind_to_gpu_restricts_and_respects_switches(tmp_path, monkeypatch):
    allowed = sorted(os.sched_getaffinity(0))
    root = _fake_sysfs(tmp_path, "0000:05:00.0", str(allowed[0]))
    monkeypatch.delenv("MLS_NUMA_BIND", raising=False)
    # single rank by default: binds only when it keeps enough CPUs (one local CPU of several: no)
    assert bind_to_gpu(0, world_size=1, sysfs_root=root, pci_addr="0000:05:00.0") is None
    monkeypatch.setenv("MLS_NUMA_BIND", "0")
    assert bind_to_gpu(0, world_size=8, sysfs_root=root, pci_addr="0000:05:00.0") is None
    monkeypatch.delenv("MLS_NUMA_BIND")
    try:
        got = bind_to_gpu(0, world_size=8, sysfs_root=root, pci_addr="0000:05:00.0")
        assert got == [allowed[0]] and sorted(os.sched_getaffinity(0)) == [allowed[0]]
    finally:
        os.sched_setaffinity(0, allowed)


@pytest.mark.skipif(not hasattr(os, "sched_getaffinity") or len(os.sched_getaffinity(0)) < 2,
                    reason="needs >= 2 usable CPUs")
def test_single_rank_binds_by_default_when_enough_cpus_are_local(tmp_path, monkeypatch):
    from mlmicroservicetemplate_amd.parallel import affinity

    allowed = sorted(os.sched_getaffinity(0))
    half = allowed[: max(1, len(allowed) // 2)]
    root = _fake_sysfs(tmp_path, "0000:05:00.0", ",".join(map(str, half)))
    monkeypatch.delenv("MLS_NUMA_BIND", raising=False)
    monkeypatch.setattr(affinity, "SINGLE_RANK_MIN_CPUS", len(half))
    try:
        assert bind_to_gpu(0, world_size=1, sysfs_root=root, pci_addr="0000:05:00.0") == half
        assert sorted(os.sched_getaffinity(0)) == half
    finally:
        os.sched_setaffinity(0, allowed)
    monkeypatch.setattr(affinity, "SINGLE_RANK_MIN_CPUS", len(half) + 1)
    assert bind_to_gpu(0, world_size=1, sysfs_root=root, pci_addr="0000:05:00.0") is None  # too few local
    monkeypatch.setenv("MLS_NUMA_BIND", "1")  # forced: binds regardless
    try:
        assert bind_to_gpu(0, world_size=1, sysfs_root=root, pci_addr="0000:05:00.0") == half
    finally:
        os.sched_setaffinity(0, allowed)


def test_host_plan_8_ranks_on_2_sockets(tmp_path, monkeypatch):
    """An 8-GPU node with 2 x 64-CPU sockets, GPUs 0-3 on socket 0 and 4-7 on socket 1: every rank
    shares its socket's 64 CPUs with 3 others -> 16 CPUs each, the 4-thread staging cap, a copy
    budget that covers one MI355X's ResNet-50 input rate; the plan is what bind_to_gpu records
    for the bench JSON (bench.py host_plan_rank0)."""
    from mlmicroservicetemplate_amd.parallel import affinity

    addrs = [f"0000:{0x10 * (g + 1):02x}:00.0" for g in range(8)]
    for g, a in enumerate(addrs):
        d = tmp_path / "bus" / "pci" / "devices" / a
        d.mkdir(parents=True)
        (d / "local_cpulist").write_text("0-63" if g < 4 else "64-127")
    root = str(tmp_path)
    pci_of = lambda i: addrs[i]  # noqa: E731
    for g in range(8):
        assert affinity.ranks_sharing_cpus(g, 8, root, pci_of=pci_of) == 4
    plan = affinity.host_plan(64, 4)
    assert plan["cpus_per_rank"] == 16 and plan["stage_threads"] == affinity.STAGE_THREADS_CAP
    assert plan["headroom"] >= 1.0, plan  # 5 copying threads x 3.5 GB/s >= 60k img/s x 150 KB
    # a rank whose process may only use 8 CPUs of its socket (a container): 2 each, 1 copy thread
    small = affinity.host_plan(8, 4)
    assert small["stage_threads"] == 1 and small["headroom"] < 1.0, small
    # bind_to_gpu records the plan with the process's real CPU set (the fake sockets are not ours,
    # so binding falls back to the allowed CPUs) without changing the affinity here
    monkeypatch.setenv("MLS_NUMA_BIND", "0")
    bind_to_gpu(5, world_size=8, sysfs_root=root, pci_of=pci_of, local_world=8)
    got = affinity.host_plan_hint()
    assert got is not None and got["ranks_sharing_cpus"] == 4
    assert got["stage_threads"] == affinity.stage_threads_hint()
