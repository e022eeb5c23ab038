"""Rank layout and GPU-link topology of one MI355X node.

qmx runs one rank process per GPU (data-parallel session sharding over one SO_REUSEPORT
port; optional expert-parallel-style backend-stream placement, see :mod:`.exchange`).
The reference has no distributed layer at all (a single asyncio
process, ``oai_proxy.py:547-550`` fan-out); this module is new.

* :class:`RankEnv` — rank / world / local rank / device from the launcher's environment
  (``torch.distributed.run``: RANK, WORLD_SIZE, LOCAL_RANK; ``qmx serve --gpus N``:
  QMX_RANK, QMX_WORLD).
* :func:`gpu_links` — the xGMI / PCIe links between GPUs from the KFD topology in sysfs
  (``/sys/class/kfd/kfd/topology/nodes/*/io_links/*/properties``).  On an 8× MI355X node
  every GPU has 7 direct xGMI links (one per peer): a ring collective is bound by ONE
  link per step, so the exchange batches every session finalised in a round into a single
  all-gather (latency-bound KB payloads) instead of per-session collectives.
"""
from __future__ import annotations

import os
from dataclasses import dataclass
from pathlib import Path
from typing import Dict, List, Mapping, Optional

# QMX_SYSFS_ROOT: read the topology from a copy of /sys (tests and `bench.py --plan` on a
# fake 8-GPU node); set before this module is imported
SYSFS = Path(os.environ.get("QMX_SYSFS_ROOT", "/sys"))
KFD_TOPOLOGY = SYSFS / "class/kfd/kfd/topology/nodes"
# KFD io_link "type" values (kfd_topology.h: CRAT_IOLINK_TYPE_*)
LINK_TYPES = {1: "hypertransport", 2: "pcie", 11: "xgmi"}


@dataclass(frozen=True)
class RankEnv:
    rank: int = 0
    world: int = 1
    local_rank: int = 0

    @classmethod
    def from_env(cls, env: Optional[Mapping[str, str]] = None) -> "RankEnv":
        """qmx's own launcher (QMX_*) wins over torch.distributed.run's variables."""
        e = os.environ if env is None else env
        rank = int(e.get("QMX_RANK", e.get("RANK", "0")))
        world = int(e.get("QMX_WORLD", e.get("WORLD_SIZE", "1")))
        local = int(e.get("LOCAL_RANK", str(rank)))
        if not (0 <= rank < world):
            raise ValueError(f"rank {rank} outside world {world}")
        return cls(rank, world, local)

    def device(self, n_devices: int) -> int:
        """One rank per GPU: the local rank's GPU (wrapping only when ranks > GPUs, as in CPU
        rehearsals; a real node launches exactly one rank per device)."""
        return self.local_rank % max(n_devices, 1)

    @property
    def distributed(self) -> bool:
        return self.world > 1


@dataclass(frozen=True)
class Link:
    src: int  # GPU index (order of KFD GPU nodes = HIP device order)
    dst: int
    kind: str
    weight: int
    max_bandwidth: int  # MB/s as reported by KFD (0 = not reported)


def _props(path: Path) -> Dict[str, int]:
    out: Dict[str, int] = {}
    try:
        for ln in path.read_text().splitlines():
            k, _, v = ln.strip().partition(" ")
            try:
                out[k] = int(v.strip())
            except ValueError:
                pass
    except OSError:
        pass
    return out


def _gpu_nodes(root: Path) -> Dict[int, int]:
    """KFD node id -> GPU index (KFD node order = HIP device order; CPU nodes have no SIMDs)."""
    if not root.is_dir():
        return {}
    nodes = sorted((p for p in root.iterdir() if p.name.isdigit()), key=lambda p: int(p.name))
    gpu_of: Dict[int, int] = {}
    for p in nodes:
        if _props(p / "properties").get("simd_count", 0) > 0:
            gpu_of[int(p.name)] = len(gpu_of)
    return gpu_of


def gpu_count(root: Path = KFD_TOPOLOGY) -> int:
    return len(_gpu_nodes(root))


def gpu_links(root: Path = KFD_TOPOLOGY) -> List[Link]:
    """Direct GPU↔GPU links (CPU nodes and GPU↔CPU links are left out)."""
    gpu_of = _gpu_nodes(root)
    if not gpu_of:
        return []
    nodes = sorted((p for p in root.iterdir() if p.name.isdigit()), key=lambda p: int(p.name))
    links: List[Link] = []
    for p in nodes:
        src = int(p.name)
        if src not in gpu_of:
            continue
        io = p / "io_links"
        if not io.is_dir():
            continue
        for lp in sorted(io.iterdir(), key=lambda q: int(q.name) if q.name.isdigit() else 0):
            pr = _props(lp / "properties")
            dst = pr.get("node_to", -1)
            if dst not in gpu_of:
                continue
            links.append(Link(gpu_of[src], gpu_of[dst], LINK_TYPES.get(pr.get("type", 0), str(pr.get("type", 0))),
                              pr.get("weight", 0), pr.get("max_bandwidth", 0)))
    return links


def summary(links: Optional[List[Link]] = None, n_gpus: Optional[int] = None,
            root: Path = KFD_TOPOLOGY) -> Dict[str, object]:
    """GPU count, per-GPU direct-link counts by kind, and whether the GPUs form a full xGMI
    mesh (a single GPU trivially does)."""
    links = gpu_links(root) if links is None else links
    if n_gpus is None:
        n_gpus = gpu_count(root) if root.is_dir() else len({x.src for x in links} | {x.dst for x in links})
    per: Dict[int, Dict[str, int]] = {g: {} for g in range(n_gpus)}
    for x in links:
        per.setdefault(x.src, {})
        per[x.src][x.kind] = per[x.src].get(x.kind, 0) + 1
    full = n_gpus > 0 and all(per[g].get("xgmi", 0) >= n_gpus - 1 for g in range(n_gpus))
    return {"gpus": n_gpus, "links_per_gpu": per, "full_xgmi_mesh": full}


# ---- NUMA placement of a rank's host threads ------------------------------------------
# On an 8-GPU node each GPU hangs off one socket's PCIe root; a rank's io loops, tick lanes
# (which poll the GPU's mapped result records) and — in bench.py — its load generator and
# mock backends talk over loopback TCP, so keeping them on the GPU's NUMA node keeps both
# the socket traffic and the mapped-memory polling socket-local.
PCI_DEVICES = SYSFS / "bus/pci/devices"
NUMA_NODES = SYSFS / "devices/system/node"
CPU_DEVICES = SYSFS / "devices/system/cpu"


def all_node_cpus(root: Path = NUMA_NODES) -> List[int]:
    """Every CPU of every NUMA node (the machine's CPUs as the topology reports them)."""
    out: List[int] = []
    if root.is_dir():
        for p in sorted(root.iterdir()):
            if p.name.startswith("node") and p.name[4:].isdigit():
                out.extend(node_cpus(int(p.name[4:]), root))
    return sorted(set(out))


def parse_cpulist(s: str) -> List[int]:
    """``0-3,8,10-11`` -> [0, 1, 2, 3, 8, 10, 11]."""
    out: List[int] = []
    for part in s.strip().split(","):
        if not part:
            continue
        a, _, b = part.partition("-")
        out.extend(range(int(a), int(b or a) + 1))
    return out


def pci_numa_node(domain: int, bus: int, device: int, function: int = 0, root: Path = PCI_DEVICES) -> int:
    """NUMA node of a PCI function (-1 when unknown or single-node)."""
    try:
        return int((root / f"{domain:04x}:{bus:02x}:{device:02x}.{function}" / "numa_node").read_text().strip())
    except (OSError, ValueError):
        return -1


def node_cpus(node: int, root: Path = NUMA_NODES) -> List[int]:
    try:
        return parse_cpulist((root / f"node{node}" / "cpulist").read_text())
    except (OSError, ValueError):
        return []


def _core_key(cpu: int, root: Path) -> tuple:
    t = root / f"cpu{cpu}" / "topology"
    try:
        return (int((t / "physical_package_id").read_text()), int((t / "core_id").read_text()))
    except (OSError, ValueError):
        return (-1, cpu)


def rank_cpus(gpu_nodes: List[int], local_rank: int, allowed: Optional[List[int]] = None,
              node_root: Path = NUMA_NODES, cpu_root: Path = CPU_DEVICES) -> Optional[List[int]]:
    """CPUs for ``local_rank`` given the NUMA node of every local rank's GPU: the ranks whose
    GPUs share a node split that node's allowed CPUs by whole physical cores (SMT siblings
    stay together), in rank order.  None when the node is unknown or has too few cores."""
    node = gpu_nodes[local_rank] if 0 <= local_rank < len(gpu_nodes) else -1
    if node < 0:
        return None
    ok = set(allowed) if allowed is not None else None
    cpus = [c for c in node_cpus(node, node_root) if ok is None or c in ok]
    peers = [r for r, n in enumerate(gpu_nodes) if n == node]
    cores: Dict[tuple, List[int]] = {}
    for c in cpus:
        cores.setdefault(_core_key(c, cpu_root), []).append(c)
    keys = sorted(cores, key=lambda k: min(cores[k]))
    if len(keys) < len(peers):
        return None
    k = peers.index(local_rank)
    lo, hi = k * len(keys) // len(peers), (k + 1) * len(keys) // len(peers)
    return sorted(c for key in keys[lo:hi] for c in cores[key])


def _llc_key(cpu: int, root: Path) -> str:
    try:
        return (root / f"cpu{cpu}" / "cache" / "index3" / "shared_cpu_list").read_text().strip()
    except OSError:
        return ""


def llc_cpus(node: int, node_root: Path = NUMA_NODES, cpu_root: Path = CPU_DEVICES) -> int:
    """Hardware threads sharing the last-level cache with the node's first CPU (0: unknown)."""
    cpus = node_cpus(node, node_root)
    if not cpus:
        return 0
    k = _llc_key(cpus[0], cpu_root)
    return len(parse_cpulist(k)) if k else 0


def cpu_busy(interval: float = 0.2, stat: Path = Path("/proc/stat")) -> Dict[int, float]:
    """Per-CPU busy fraction over ``interval`` seconds (/proc/stat; {} when unreadable)."""
    import time

    def read() -> Dict[int, tuple]:
        out = {}
        try:
            for line in stat.read_text().splitlines():
                f = line.split()
                if f and f[0].startswith("cpu") and f[0] != "cpu":
                    v = [int(x) for x in f[1:]]
                    idle = v[3] + (v[4] if len(v) > 4 else 0)
                    out[int(f[0][3:])] = (sum(v), idle)
        except (OSError, ValueError):
            return {}
        return out

    a = read()
    time.sleep(interval)
    b = read()
    busy = {}
    for c, (t1, i1) in b.items():
        t0, i0 = a.get(c, (t1, i1))
        busy[c] = 1.0 - (i1 - i0) / (t1 - t0) if t1 > t0 else 0.0
    return busy


def compact_cpus(n: int, node: int, allowed: Optional[List[int]] = None, smt: bool = False,
                 node_root: Path = NUMA_NODES, cpu_root: Path = CPU_DEVICES,
                 busy: Optional[Dict[int, float]] = None) -> Optional[List[int]]:
    """``n`` CPUs of NUMA node ``node`` packed into as few last-level caches (CCDs) as they
    fit: one hardware thread per physical core (``smt``: both siblings of n / 2 cores), cores
    in LLC order.  A single-rank bench whose job quota is ``n`` CPUs on a many-core box then
    keeps its proxy, mocks and load generator — loopback TCP peers — on shared L3s instead of
    wherever the scheduler scatters them.  ``busy`` (cpu_busy: other tenants' load on a shared
    host) orders the L3s least-loaded first.  None when the node has too few cores."""
    ok = set(allowed) if allowed is not None else None
    cpus = [c for c in node_cpus(node, node_root) if ok is None or c in ok]
    cores: Dict[tuple, List[int]] = {}
    for c in cpus:
        cores.setdefault(_core_key(c, cpu_root), []).append(c)
    def llc_of(cpu: int) -> List[int]:
        k = _llc_key(cpu, cpu_root)
        return parse_cpulist(k) if k else [cpu]

    def llc_rank(cpu: int) -> tuple:  # an L3 by its load, then by its lowest CPU
        members = llc_of(cpu)
        load = round(sum((busy or {}).get(c, 0.0) for c in members), 1)
        return (load, min(members))

    keys = sorted(cores, key=lambda k: (llc_rank(min(cores[k])), min(cores[k])))
    out: List[int] = []
    for k in keys:
        if len(out) >= n:
            break
        out.extend(sorted(cores[k]) if smt else [min(cores[k])])
    if len(out) < n:
        return None
    return sorted(out[:n])


def rank_llc_cpus(gpu_nodes: List[int], local_rank: int, per_rank: int, allowed: Optional[List[int]] = None,
                  node_root: Path = NUMA_NODES, cpu_root: Path = CPU_DEVICES) -> Optional[List[int]]:
    """``local_rank``'s compact CPU set: whole last-level caches (both SMT threads of their
    cores) of its GPU's NUMA node, ``per_rank`` CPUs rounded up to whole L3s; the ranks whose
    GPUs share the node take consecutive L3s in CPU order (every rank computes the same,
    disjoint split without talking to the others).  None when the node is unknown or has too
    few L3s for its ranks."""
    node = gpu_nodes[local_rank] if 0 <= local_rank < len(gpu_nodes) else -1
    if node < 0 or per_rank <= 0:
        return None
    ok = set(allowed) if allowed is not None else None
    cpus = [c for c in node_cpus(node, node_root) if ok is None or c in ok]
    groups: Dict[str, List[int]] = {}
    for c in cpus:
        groups.setdefault(_llc_key(c, cpu_root) or f"cpu{c}", []).append(c)
    order = sorted(groups.values(), key=min)
    if not order:
        return None
    llc = max(len(g) for g in order)
    k = max(1, -(-per_rank // llc))
    peers = [r for r, n in enumerate(gpu_nodes) if n == node]
    p = peers.index(local_rank)
    if (p + 1) * k > len(order):
        return None
    return sorted(c for g in order[p * k:(p + 1) * k] for c in g)


def gpu_numa_nodes(root: Path = KFD_TOPOLOGY, pci_root: Path = PCI_DEVICES) -> List[int]:
    """NUMA node of every GPU in KFD order, from the KFD node's PCI address (``domain`` +
    ``location_id`` = bus << 8 | devfn) — no HIP call, so a launcher can plan before any
    rank touches the GPU.  -1 where unknown."""
    out: List[int] = []
    gpu_of = _gpu_nodes(root)
    for node in sorted(gpu_of, key=gpu_of.get):
        pr = _props(root / str(node) / "properties")
        loc = pr.get("location_id", -1)
        out.append(pci_numa_node(pr.get("domain", 0), loc >> 8, (loc >> 3) & 31, loc & 7, pci_root)
                   if loc >= 0 else -1)
    return out


def plan_rank_cpus(gpu_nodes: List[int], allowed: List[int], min_cover: float = 0.9,
                   node_root: Path = NUMA_NODES, cpu_root: Path = CPU_DEVICES) -> Optional[List[List[int]]]:
    """Every local rank's CPU set (see :func:`rank_cpus`), or None when any rank's node is
    unknown or the sets would leave more than ``1 - min_cover`` of the allowed CPUs idle
    (e.g. firmware reporting every GPU on node 0 of a two-socket box): pinning must never
    strand cores the unpinned scheduler would use."""
    sets = [rank_cpus(gpu_nodes, r, allowed, node_root, cpu_root) for r in range(len(gpu_nodes))]
    if not sets or any(s is None for s in sets):
        return None
    if sum(len(s) for s in sets) < min_cover * len(allowed):
        return None
    return sets
