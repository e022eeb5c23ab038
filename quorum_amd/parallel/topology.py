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

KFD_TOPOLOGY = Path("/sys/class/kfd/kfd/topology/nodes")
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
