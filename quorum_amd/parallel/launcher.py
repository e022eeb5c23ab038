"""Node launcher: one rank (supervisor + native worker) per GPU on one shared port.

    python -m quorum_amd.serve --impl native --gpus 8 --config config.yaml --port 8000

Data parallelism is session sharding: every rank's io loops bind the same SO_REUSEPORT
port, so the kernel hashes client connections (sessions) across the node's GPUs.  With
``runtime.placement: spread`` the ranks also exchange backend streams (see
:mod:`.exchange`).  SIGHUP (rolling reload) and SIGTERM (drain) are forwarded to every
rank's supervisor.  ``torch.distributed.run`` is the other supported launcher (bench.py):
both set the same rank variables (:class:`.topology.RankEnv`).

Reference counterpart: none — quorum is one uvicorn process (Makefile:4-7).
"""
from __future__ import annotations

import logging
import os
import signal
import subprocess
import sys
import time
from typing import List, Sequence

from .exchange import exchange_env
from .topology import gpu_numa_nodes, plan_rank_cpus, summary

log = logging.getLogger("qmx.launcher")


def rank_commands(argv: Sequence[str], gpus: int, bind_devices: bool, port: int, nonce: str):
    """(cmd, env) per rank: the same ``serve`` command line re-run with the rank variables
    (and ``--device r`` unless the caller pinned a device)."""
    out = []
    for r in range(gpus):
        xe = exchange_env(r, gpus, port, nonce)
        if "QMX_XCHG_PORT" in os.environ:  # an explicit rendezvous port wins
            xe.pop("QMX_XCHG_PORT")
        env = dict(os.environ, LOCAL_RANK=str(r), **xe)
        cmd = [sys.executable, "-m", "quorum_amd.serve"] + list(argv)
        if bind_devices:
            cmd += ["--device", str(r)]
        out.append((cmd, env))
    return out


def launch_ranks(argv: Sequence[str], gpus: int, bind_devices: bool, port: int) -> int:
    topo = summary()
    if topo["gpus"]:
        log.info("GPU links: %s (full xGMI mesh: %s)", topo["links_per_gpu"], topo["full_xgmi_mesh"])
    nonce = str(time.time_ns())
    # bind each rank to its GPU's NUMA node when the KFD/PCI topology says where it is
    # (QMX_PIN=0 disables; device-pinned or rehearsal launches are left alone)
    plan = None
    if bind_devices and os.environ.get("QMX_PIN", "1") != "0":
        nodes = gpu_numa_nodes()
        if len(nodes) >= gpus:
            plan = plan_rank_cpus(nodes[:gpus], sorted(os.sched_getaffinity(0)))
    if plan:
        log.info("rank CPU sets: %s", [len(c) for c in plan])
    procs: List[subprocess.Popen] = []
    for r, (cmd, env) in enumerate(rank_commands(argv, gpus, bind_devices, port, nonce)):
        cpus = plan[r] if plan else None
        pre = (lambda c=cpus: os.sched_setaffinity(0, c)) if cpus else None
        procs.append(subprocess.Popen(cmd, env=env, start_new_session=True, preexec_fn=pre))

    def fwd(sig, _frame):
        for p in procs:
            try:
                os.kill(p.pid, sig)
            except OSError:
                pass

    for sig in (signal.SIGHUP, signal.SIGTERM, signal.SIGINT):
        signal.signal(sig, fwd)
    rc = 0
    for p in procs:
        rc = p.wait() or rc
    return rc
