"""Cross-rank settings of the native exchange (SURVEY §2.3 R1, §2.4 EP, §5.8).

With ``runtime.placement: spread`` a session's N backend streams run on ranks
owner..owner+N-1 (mod world) — the expert-parallel analog of quorum's backend fan-out
(``oai_proxy.py:547-550``).  The exchange (``csrc/qmx_exchange.cpp``) has two planes, both
event-driven (an idle node exchanges nothing):

* mesh: one TCP connection per rank pair (rank r listens on ``QMX_XCHG_PORT + r``) for
  control messages and the encoded SSE deltas — point to point, never on a collective,
  because they sit on the TTFT path; a restarted rank re-joins by redialling;
* bulk (``rccl``): each stream's final text moves from the worker's HBM content arena into
  the owner's HBM shadow slot with ``ncclSend``/``ncclRecv`` over xGMI, in rounds rank 0
  orders (so both ends of every pair post matching operations), and the owner's fused
  finalize kernel merges remote and local texts.  ``tcpbulk`` runs the very same rounds,
  epochs and fallbacks with a socket per rank pair as the executor (CPU hosts, and rank
  rehearsals sharing one GPU, where RCCL cannot form).  ``tcp`` moves the bytes over the
  mesh, as do the others while their communicator is (re)forming.

Every rank must agree on the transport and the mesh base port: :func:`exchange_env` builds
them once (launcher / bench) and :func:`cluster_config` turns them into the native
server's settings.
"""
from __future__ import annotations

import os
import time
from typing import Any, Dict, Mapping, Optional

from .topology import RankEnv


def exchange_env(rank: int, world: int, port: int, nonce: Optional[str] = None) -> Dict[str, str]:
    """Environment for rank ``rank`` of a ``world``-rank node serving on ``port``: the mesh
    listens on ``port + 7 + rank``.  The nonce names the deployment (all ranks of one
    deployment get the same one)."""
    return {"QMX_RANK": str(rank), "QMX_WORLD": str(world), "QMX_XCHG_NONCE": nonce or str(time.time_ns()),
            "QMX_XCHG_PORT": str(port + 7)}


def cluster_config(placement: str, exchange: str, round_us: int, timeout: float, port: int, engine: str,
                   env: Optional[Mapping[str, str]] = None, eager_bytes: int = 4096) -> Dict[str, Any]:
    """Rank / placement / exchange settings of the native server (env wins: QMX_RANK,
    QMX_WORLD, QMX_XCHG_*).  ``exchange: auto`` = RCCL with the HIP engine, else TCP."""
    e = os.environ if env is None else env
    r = RankEnv.from_env(e)
    xchg = e.get("QMX_XCHG", exchange)
    if xchg == "auto":
        xchg = "rccl" if engine == "hip" else "tcp"
    if xchg not in ("rccl", "tcp", "tcpbulk"):
        raise ValueError(f"runtime.exchange {xchg!r}: expected 'auto', 'rccl', 'tcpbulk' or 'tcp'")
    if placement not in ("local", "spread"):
        raise ValueError(f"runtime.placement {placement!r}: expected 'local' or 'spread'")
    nonce = e.get("QMX_XCHG_NONCE", "0")
    return {
        "rank": r.rank, "world": r.world, "placement": placement, "xchg": xchg,
        "xchg_addr": e.get("QMX_XCHG_ADDR", "127.0.0.1"),
        "xchg_port": int(e.get("QMX_XCHG_PORT", str(port + 7))),
        # tcpbulk: the round executor's sockets (rank r listens on this + r; 0 = mesh port + world)
        "xchg_bulk_port": int(e.get("QMX_XCHG_BULK_PORT", "0")),
        "xchg_id_file": "",  # the RCCL unique id travels over the mesh (rank 0 → all)
        # rank 0 batches bulk announcements arriving within this window into one round
        "xchg_round_us": int(e.get("QMX_XCHG_ROUND_US", str(round_us))),
        "xchg_timeout": float(e.get("QMX_XCHG_TIMEOUT", str(timeout))),
        # final texts up to this size ride the mesh behind their deltas (eager, no round)
        "xchg_eager_bytes": int(e.get("QMX_XCHG_EAGER_BYTES", str(eager_bytes))),
        # per-loop links: io loop l of each rank pair on a connection of its own (0: the mesh
        # thread carries every session message)
        "xchg_links": int(e.get("QMX_XCHG_LINKS", "1")),
    }
