"""Per-replica host CPU placement (omnia_amd/utils/affinity.py) on a fake sysfs
tree shaped like an 8-GPU MI355X node: 2 sockets / NUMA nodes of 64 CPUs,
GPUs 0-3 on node 0 and 4-7 on node 1 (PCI addresses in KFD node order)."""
import os

import pytest

from omnia_amd.utils import affinity


def _fake_node(tmp_path, gpus_per_node=4, cpus_per_node=64, nodes=2, numa=None):
    root = tmp_path
    kfd = root / "sys/class/kfd/kfd/topology/nodes"
    # KFD: CPU nodes first, then GPU nodes (simd_count > 0)
    idx = 0
    for n in range(nodes):
        d = kfd / str(idx)
        d.mkdir(parents=True)
        (d / "properties").write_text(f"cpu_cores_count {cpus_per_node}\nsimd_count 0\n")
        idx += 1
    g = 0
    for n in range(nodes):
        for k in range(gpus_per_node):
            d = kfd / str(idx)
            d.mkdir(parents=True)
            bus = 0x05 + 0x20 * g
            (d / "properties").write_text(
                f"cpu_cores_count 0\nsimd_count 1024\ndomain 0\nlocation_id {bus << 8}\n")
            pci = root / f"sys/bus/pci/devices/0000:{bus:02x}:00.0"
            pci.mkdir(parents=True)
            node = numa[g] if numa is not None else n
            (pci / "numa_node").write_text(f"{node}\n")
            idx += 1
            g += 1
    for n in range(nodes):
        d = root / f"sys/devices/system/node/node{n}"
        d.mkdir(parents=True)
        lo = n * cpus_per_node
        (d / "cpulist").write_text(f"{lo}-{lo + cpus_per_node - 1}\n")
    return str(root)


def test_parse_cpulist():
    assert affinity.parse_cpulist("0-3,8,10-11\n") == [0, 1, 2, 3, 8, 10, 11]
    assert affinity.parse_cpulist("") == []


def test_gpu_numa_nodes_from_kfd_and_pci(tmp_path):
    root = _fake_node(tmp_path)
    addrs = affinity.gpu_pci_addresses(root)
    assert len(addrs) == 8 and addrs[0] == "0000:05:00.0"
    assert [affinity.gpu_numa_node(g, root) for g in range(8)] == [0] * 4 + [1] * 4
    assert affinity.gpu_numa_node(9, root) == 0  # unknown -> node 0


def test_eight_replicas_get_disjoint_numa_local_sets(tmp_path):
    root = _fake_node(tmp_path)
    plan = affinity.plan(list(range(8)), root, allowed=set(range(128)))
    assert all(len(p) == 16 for p in plan)
    flat = [c for p in plan for c in p]
    assert len(flat) == len(set(flat))  # disjoint
    for g, p in enumerate(plan):
        node = 0 if g < 4 else 1
        assert all(node * 64 <= c < (node + 1) * 64 for c in p), (g, p)


def test_plan_respects_container_cpuset_and_oversubscription(tmp_path):
    root = _fake_node(tmp_path)
    # a cpuset of 8 CPUs on node 0 and 2 on node 1
    allowed = set(range(8)) | {64, 65}
    plan = affinity.plan(list(range(8)), root, allowed=allowed)
    assert [len(p) for p in plan[:4]] == [2, 2, 2, 2]
    assert len({c for p in plan[:4] for c in p}) == 8
    # node 1 has 2 CPUs for 4 replicas: one each, shared round-robin, never node 0
    assert all(len(p) == 1 and p[0] in (64, 65) for p in plan[4:])


def test_no_sysfs_falls_back_to_an_even_split(tmp_path):
    plan = affinity.plan([0, 1, 2, 3], str(tmp_path), allowed=set(range(8)))
    assert plan == [[0, 1], [2, 3], [4, 5], [6, 7]]


def test_pin_sets_this_process_affinity():
    before = os.sched_getaffinity(0)
    try:
        cpu = min(before)
        assert affinity.pin([cpu])
        assert os.sched_getaffinity(0) == {cpu}
    finally:
        os.sched_setaffinity(0, before)
    assert not affinity.pin([])


def test_device_allocator_pins_pods_to_their_gpus_slices(monkeypatch, tmp_path):
    from omnia_amd.operator.launcher import DeviceAllocator

    monkeypatch.setattr(affinity, "plan", lambda devs, root="/": [[2 * d, 2 * d + 1]
                                                                  for d in devs])
    a = DeviceAllocator(4)
    assert a.cpus_for([1]) is None  # 2-CPU slices: oversubscribed, left unpinned
    monkeypatch.setattr(affinity, "plan", lambda devs, root="/": [list(range(4 * d, 4 * d + 4))
                                                                  for d in devs])
    a = DeviceAllocator(4)
    assert a.cpus_for([1]) == [4, 5, 6, 7]
    assert a.cpus_for([2, 3]) == list(range(8, 16))  # a TP pod: its GPUs' slices
    assert DeviceAllocator(1).cpus_for([0]) is None
    monkeypatch.setenv("OMNIA_PIN_CPUS", "0")
    assert DeviceAllocator(4).cpus_for([0]) is None


@pytest.mark.skipif(len(os.sched_getaffinity(0)) < 2, reason="needs 2 CPUs")
def test_process_pod_children_inherit_the_pin(tmp_path):
    """A pod's processes run inside its CPU set (checked on a real child)."""
    import subprocess
    import sys

    from omnia_amd.operator.pods import ProcessPod

    cpu = min(os.sched_getaffinity(0))
    pod = ProcessPod("t", {}, {}, log_dir=str(tmp_path), cpus=[cpu])
    p = pod._spawn("json.tool", {}, "probe")  # any module: we only read its affinity
    try:
        assert os.sched_getaffinity(p.pid) == {cpu}
    finally:
        p.kill()
        p.wait()
    out = subprocess.run([sys.executable, "-c", "import os;print(sorted(os.sched_getaffinity(0)))"],
                         capture_output=True, text=True)
    assert out.returncode == 0
