"""``qmx serve`` — run the proxy: W worker processes per rank on one SO_REUSEPORT port.

    python -m quorum_amd.serve --config config.yaml --port 8000 --workers 4 [--device 0]
                               [--engine hip|cpu|python|auto] [--impl python|native]

Each worker owns its own stream engine (for ``hip``: its own HIP stream, device-resident
slot arena and pinned arenas on the rank's GPU).  The kernel's SO_REUSEPORT hashing
shards client connections (sessions) across workers — and, when several ranks bind the
same port, across the node's GPUs.

``--impl native`` runs the C++ epoll data plane (quorum_amd/csrc/qmx_server.cpp) instead
of uvicorn/FastAPI; same config, same semantics.
"""
from __future__ import annotations

import argparse
import logging
import os
import signal
import socket
import subprocess
import sys
import time
from typing import List, Optional


def reuseport_socket(host: str, port: int) -> socket.socket:
    s = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
    s.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
    s.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEPORT, 1)
    s.bind((host, port))
    s.listen(4096)
    s.set_inheritable(True)
    return s


def run_worker(config: str, host: str, port: int, engine: str, device: Optional[int]) -> None:
    import uvicorn

    from .server.app import create_app
    from .utils.config import RuntimeConfig, load_config

    cfg = load_config(config)
    rt = RuntimeConfig.from_config(cfg)
    if engine:
        rt.engine = engine
    if device is not None:
        rt.device = device
    app = create_app(lambda: cfg, runtime=rt)
    sock = reuseport_socket(host, port)
    ucfg = uvicorn.Config(app, log_level="warning", access_log=False, lifespan="off", http="h11",
                          loop="asyncio", timeout_keep_alive=60, backlog=4096)
    uvicorn.Server(ucfg).run(sockets=[sock])


def spawn_workers(config: str, host: str, port: int, workers: int, engine: str, device: Optional[int],
                  impl: str = "python", threads: int = 2, env: Optional[dict] = None) -> List[subprocess.Popen]:
    procs = []
    e = dict(os.environ if env is None else env)
    e.setdefault("PYTHONUNBUFFERED", "1")
    for _ in range(workers if impl == "python" else 1):
        if impl == "native":
            cmd = [sys.executable, "-m", "quorum_amd.serve", "--native-worker", "--config", config, "--host", host,
                   "--port", str(port), "--engine", engine, "--threads", str(threads)]
        else:
            cmd = [sys.executable, "-m", "quorum_amd.serve", "--worker", "--config", config, "--host", host,
                   "--port", str(port), "--engine", engine]
        if device is not None:
            cmd += ["--device", str(device)]
        procs.append(subprocess.Popen(cmd, env=e, start_new_session=True))
    return procs


def wait_healthy(host: str, port: int, timeout: float = 120.0) -> bool:
    import http.client

    t0 = time.time()
    while time.time() - t0 < timeout:
        try:
            c = http.client.HTTPConnection(host, port, timeout=2)
            c.request("GET", "/health")
            if c.getresponse().status == 200:
                return True
        except OSError:
            pass
        time.sleep(0.2)
    return False


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="qmx serve")
    ap.add_argument("--config", default=None)
    ap.add_argument("--host", default="127.0.0.1")
    ap.add_argument("--port", type=int, default=8000)
    ap.add_argument("--workers", type=int, default=1)
    ap.add_argument("--threads", type=int, default=2)
    ap.add_argument("--engine", default="auto")
    ap.add_argument("--device", type=int, default=None)
    ap.add_argument("--impl", default="python", choices=["python", "native"])
    ap.add_argument("--worker", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--native-worker", action="store_true", help=argparse.SUPPRESS)
    args = ap.parse_args(argv)
    logging.basicConfig(level=logging.WARNING)
    config = args.config or os.environ.get("QMX_CONFIG") or "config.yaml"
    if args.worker:
        run_worker(config, args.host, args.port, args.engine, args.device)
        return 0
    if args.native_worker:
        from .runtime.native_server import run_native

        return run_native(config, args.host, args.port, args.engine, args.device, args.threads)
    procs = spawn_workers(config, args.host, args.port, args.workers, args.engine, args.device, args.impl,
                          args.threads)

    def stop(*_):
        for p in procs:
            try:
                os.killpg(p.pid, signal.SIGTERM)
            except OSError:
                pass

    signal.signal(signal.SIGTERM, stop)
    signal.signal(signal.SIGINT, stop)
    rc = 0
    for p in procs:
        rc = p.wait() or rc
    return rc


if __name__ == "__main__":
    sys.exit(main())
