"""Host-CPU placement of per-GPU serving replicas (SURVEY §2.3 DP row).

On an 8-GPU MI355X node every replica's serving tree -- bench/WS client,
facade, runtime, engine-core -- keeps ~2.5 host cores busy
(``profiles/r4/hostpath``).  Left to the scheduler, the eight trees migrate
across sockets: the engine-core that feeds GPU g ends up on the far NUMA node,
its pinned staging buffers and the step-launch path cross the socket
interconnect, and trees steal each other's cores.  This module computes one
DISJOINT CPU set per replica, preferring CPUs on the NUMA node of the
replica's GPU, and pins a process (which its children inherit) -- without
touching the GPU, so a parent that later forks GPU workers stays safe.

GPU -> NUMA node, read from sysfs only:
  1. the KFD topology (``/sys/class/kfd/kfd/topology/nodes/N/properties``):
     GPU nodes (``simd_count > 0``) in node order are the HIP device indices;
     their ``domain`` + ``location_id`` give the PCI address;
  2. ``/sys/bus/pci/devices/<bdf>/numa_node`` (``-1`` = no affinity -> node 0).
CPUs of a node: ``/sys/devices/system/node/nodeN/cpulist``, intersected with
this process's allowed set (a container cpuset).  Every reader takes a
``root`` so tests can point it at a fake tree.
"""
from __future__ import annotations

import logging
import os

log = logging.getLogger("omnia.affinity")

# below this many CPUs per replica, automatic pinning is skipped: a serving tree
# keeps ~2.5 cores busy with bursts above that (profiles/r4/hostpath), and a
# hard slice that small starves it -- on an oversubscribed host the replicas
# are better off sharing every CPU (profiles/r5/hostpath)
MIN_AUTO_PIN_CPUS = 4


def parse_cpulist(s: str) -> list[int]:
    """``"0-3,8,10-11"`` -> ``[0, 1, 2, 3, 8, 10, 11]``."""
    out: list[int] = []
    for part in s.strip().split(","):
        part = part.strip()
        if not part:
            continue
        if "-" in part:
            a, b = part.split("-", 1)
            out.extend(range(int(a), int(b) + 1))
        else:
            out.append(int(part))
    return out


def _read(path: str) -> str | None:
    try:
        with open(path) as f:
            return f.read()
    except OSError:
        return None


def gpu_pci_addresses(root: str = "/") -> list[str]:
    """PCI addresses of the GPUs in HIP device-index order (KFD node order)."""
    base = os.path.join(root, "sys/class/kfd/kfd/topology/nodes")
    try:
        nodes = sorted(int(n) for n in os.listdir(base) if n.isdigit())
    except OSError:
        return []
    out = []
    for n in nodes:
        txt = _read(os.path.join(base, str(n), "properties"))
        if not txt:
            continue
        props = {}
        for line in txt.splitlines():
            k, _, v = line.partition(" ")
            if v.strip().lstrip("-").isdigit():
                props[k] = int(v)
        if props.get("simd_count", 0) <= 0:
            continue  # a CPU node
        loc, dom = props.get("location_id", 0), props.get("domain", 0)
        out.append(f"{dom:04x}:{(loc >> 8) & 0xff:02x}:{(loc >> 3) & 0x1f:02x}.{loc & 0x7}")
    return out


def gpu_numa_node(index: int, root: str = "/") -> int:
    """NUMA node of HIP device ``index`` (0 when unknown)."""
    addrs = gpu_pci_addresses(root)
    if index >= len(addrs):
        return 0
    txt = _read(os.path.join(root, "sys/bus/pci/devices", addrs[index], "numa_node"))
    try:
        n = int((txt or "0").strip())
    except ValueError:
        return 0
    return max(0, n)


def node_cpus(root: str = "/") -> dict[int, list[int]]:
    """NUMA node -> its CPUs (one pseudo-node 0 with every CPU if sysfs has none)."""
    base = os.path.join(root, "sys/devices/system/node")
    out = {}
    try:
        names = os.listdir(base)
    except OSError:
        names = []
    for name in names:
        if name.startswith("node") and name[4:].isdigit():
            txt = _read(os.path.join(base, name, "cpulist"))
            if txt:
                out[int(name[4:])] = parse_cpulist(txt)
    if not out:
        out[0] = list(range(os.cpu_count() or 1))
    return out


def plan(devices: list[int], root: str = "/", allowed: set[int] | None = None,
         reserve: int = 0) -> list[list[int]]:
    """One disjoint CPU list per replica (``devices[i]`` = replica i's GPU).

    Replicas whose GPUs share a NUMA node split that node's allowed CPUs into
    equal contiguous slices (the first ``reserve`` CPUs of each node are left
    to the system).  A node with fewer CPUs than replicas gives each replica at
    least one CPU, shared round-robin -- still never a CPU of another node.  A
    GPU whose node has no allowed CPUs falls back to the whole allowed set
    split among all such replicas."""
    allowed = set(allowed if allowed is not None else os.sched_getaffinity(0))
    cpus_of = {n: [c for c in cs if c in allowed] for n, cs in node_cpus(root).items()}
    node_of = [gpu_numa_node(d, root) for d in devices]
    by_node: dict[int, list[int]] = {}
    orphans = []
    for i, n in enumerate(node_of):
        if cpus_of.get(n):
            by_node.setdefault(n, []).append(i)
        else:
            orphans.append(i)
    out: list[list[int]] = [[] for _ in devices]

    def split(cpus: list[int], members: list[int]):
        k = len(members)
        if len(cpus) >= k:
            per = len(cpus) // k
            for j, i in enumerate(members):
                lo = j * per
                out[i] = cpus[lo:lo + per] if j < k - 1 else cpus[lo:]
        else:
            for j, i in enumerate(members):
                out[i] = [cpus[j % len(cpus)]]

    for n, members in by_node.items():
        cs = cpus_of[n]
        split(cs[reserve:] if len(cs) - reserve >= len(members) else cs, members)
    if orphans:
        split(sorted(allowed), orphans)
    return out


def pin(cpus: list[int], pid: int = 0) -> bool:
    """Pin ``pid`` (0 = this process; children inherit it) to ``cpus``."""
    if not cpus:
        return False
    try:
        os.sched_setaffinity(pid, set(cpus))
    except (OSError, AttributeError) as e:
        log.warning("cannot pin to CPUs %s: %s", cpus, e)
        return False
    return True


def replica_cpus(rank: int, world: int, devices: list[int] | None = None,
                 root: str = "/") -> list[int]:
    """This replica's slice of :func:`plan` (``devices`` default: rank = GPU)."""
    devs = devices if devices is not None else list(range(world))
    return plan(devs, root)[rank]
