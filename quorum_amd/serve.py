"""``qmx serve`` — run the proxy: W worker processes per rank on one SO_REUSEPORT port.

    python -m quorum_amd.serve --config config.yaml --port 8000 --workers 4 [--device 0]
                               [--engine hip|cpu|python|auto] [--impl python|native]
                               [--gpus N]     # one rank (supervisor + workers) per GPU

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
    from .utils.logging_setup import from_env, set_log_content

    from_env()
    cfg = load_config(config)
    rt = RuntimeConfig.from_config(cfg)
    if rt.log_content:
        set_log_content(True)
    if engine:
        rt.engine = engine
    if device is not None:
        rt.device = device
    app = create_app(lambda: cfg, runtime=rt)
    sock = reuseport_socket(host, port)
    ucfg = uvicorn.Config(app, log_level="warning", access_log=False, lifespan="off", http="h11",
                          loop="asyncio", timeout_keep_alive=60, backlog=4096,
                          timeout_graceful_shutdown=int(rt.drain_timeout))
    ready = os.environ.get("QMX_READY_FILE")
    if ready:
        with open(ready + f".{os.getpid()}", "w") as f:
            f.write(str(os.getpid()))
    uvicorn.Server(ucfg).run(sockets=[sock])


def spawn_workers(config: str, host: str, port: int, workers: int, engine: str, device: Optional[int],
                  impl: str = "python", threads: int = 2, env: Optional[dict] = None) -> List[subprocess.Popen]:
    procs = []
    e = dict(os.environ if env is None else env)
    e.setdefault("PYTHONUNBUFFERED", "1")
    # workers run `python -m quorum_amd.serve`: the package must import from any cwd
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    e["PYTHONPATH"] = os.pathsep.join([root] + [x for x in e.get("PYTHONPATH", "").split(os.pathsep) if x])
    # per-loop engines (runtime.shared_engine: false) each own a HIP stream: give them
    # hardware queues of their own (HIP defaults to 4)
    e.setdefault("GPU_MAX_HW_QUEUES", str(min(16, max(4, threads))))
    # the HIP engine's latency mode: on an idle loop (no tick on the GPU, <= 2 sessions at a
    # time lately) a session's streams run on the host path — p50 TTFT 0.040 -> 0.018 ms at one
    # connection, neutral at the headline's load (profiles/r6/lowload/light_host).  bench.py
    # and in-process servers leave it off: they measure / test the GPU path itself
    e.setdefault("QMX_LIGHT_HOST", "2")
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


class Supervisor:
    """Per-rank process supervisor: worker generations, rolling reload, restart on crash.

    * SIGHUP  — re-read and validate the config; start a new generation of workers on the
      same SO_REUSEPORT port; once every new worker reports ready (ready file), SIGTERM
      the old generation, which drains (no new connections, in-flight sessions finish).
      An invalid config is rejected and the running generation keeps serving.
    * SIGTERM / SIGINT — drain and stop every worker, then exit.
    * A worker of the current generation that dies unexpectedly is restarted (the
      surviving workers / ranks keep serving meanwhile) with exponential backoff.
    * ``runtime.watch_config`` / ``--watch-config``: the config file is polled (mtime, size,
      then content hash) and a change triggers the same rolling reload as SIGHUP.  A file
      that fails validation is reported once and not retried until it changes again.
    Reference counterpart: ``uvicorn --reload --reload-include "*.yaml"`` (Makefile:4), which
    restarts the single process and drops its in-flight requests.
    """

    def __init__(self, args, config: str):
        import tempfile

        self.args = args
        self.config = config
        self.tmp = tempfile.mkdtemp(prefix="qmx_sup_")
        self.gen = 0
        self.current: List[subprocess.Popen] = []
        self.retiring: List[subprocess.Popen] = []
        self.stop_requested = False
        self.reload_requested = False
        self.restarts = 0
        self.backoff = 0.5
        self.active = config  # config the current generation runs (restarts reuse it)
        self.watch_interval = 1.0
        self.watch = self._runtime_watch() or bool(getattr(args, "watch_config", False))
        self.reloads = 0
        self._stamp = self._file_stamp()
        self._next_watch = 0.0

    def _runtime_watch(self) -> bool:
        try:
            import yaml

            from .utils.config import RuntimeConfig

            with open(self.config) as f:
                rt = RuntimeConfig.from_config(yaml.safe_load(f) or {})
            self.watch_interval = max(0.05, float(rt.watch_interval))
            return bool(rt.watch_config)
        except Exception:  # noqa: BLE001 - an unreadable config is reported by validate()
            return False

    def _file_stamp(self):
        """(mtime_ns, size, sha256) of the config file, None when it cannot be read."""
        import hashlib

        try:
            st = os.stat(self.config)
            with open(self.config, "rb") as f:
                return (st.st_mtime_ns, st.st_size, hashlib.sha256(f.read()).hexdigest())
        except OSError:
            return None

    def poll_config(self) -> bool:
        """Watch mode: True when the config's content changed since the last look (an mtime
        touch with identical bytes is not a change)."""
        now = time.time()
        if not self.watch or now < self._next_watch:
            return False
        self._next_watch = now + self.watch_interval
        try:
            st = os.stat(self.config)
        except OSError:
            return False
        old = self._stamp
        if old is not None and (st.st_mtime_ns, st.st_size) == old[:2]:
            return False
        new = self._file_stamp()
        self._stamp = new
        return new is not None and (old is None or new[2] != old[2])

    def validate(self) -> Optional[str]:
        import yaml

        from .utils.config import validate_config

        try:  # strict: a reload never falls back to the built-in default config
            with open(self.config) as f:
                cfg = yaml.safe_load(f)
            validate_config(cfg)
            if self.args.impl == "native":
                from .runtime.native_server import native_config

                native_config(cfg, self.args.host, self.args.port, self.args.engine, self.args.device,
                              self.args.threads)
        except Exception as e:  # noqa: BLE001
            logging.getLogger("qmx.serve").error("config %s rejected: %s", self.config, e)
            return None
        snap = os.path.join(self.tmp, f"config.gen{self.gen + 1}.yaml")  # immutable snapshot
        with open(snap, "w") as f:
            yaml.safe_dump(cfg, f)
        return snap

    def spawn(self, n: Optional[int] = None, config: Optional[str] = None) -> List[subprocess.Popen]:
        self.gen += 1
        ready = os.path.join(self.tmp, f"gen{self.gen}")
        env = dict(os.environ)
        env["QMX_READY_FILE"] = ready
        procs = spawn_workers(config or self.active, self.args.host, self.args.port, n or self.args.workers, self.args.engine,
                              self.args.device, self.args.impl, self.args.threads, env=env)
        for p in procs:
            p.ready_file = f"{ready}.{p.pid}"  # type: ignore[attr-defined]  (written by the worker)
        return procs

    def wait_ready(self, procs, timeout: float = 120.0) -> bool:
        t0 = time.time()
        while time.time() - t0 < timeout:
            if any(p.poll() is not None for p in procs):
                return False
            if all(os.path.exists(p.ready_file) for p in procs):  # type: ignore[attr-defined]
                return True
            time.sleep(0.05)
        return False

    @staticmethod
    def term(procs) -> None:
        for p in procs:
            try:
                os.killpg(p.pid, signal.SIGTERM)
            except OSError:
                pass

    def reload(self) -> None:
        snap = self.validate()
        if snap is None:
            return
        self.reloads += 1
        new = self.spawn(config=snap)
        if not self.wait_ready(new):
            logging.getLogger("qmx.serve").error("new generation failed to start; keeping the old one")
            self.term(new)
            self.retiring += new
            return
        old, self.current = self.current, new
        self.active = snap
        self.term(old)  # drain
        self.retiring += old

    def snapshot_initial(self) -> None:
        """The first generation runs a byte copy of the config too: a worker that imports
        slowly must not read the live file while an editor (or a test) rewrites it for the
        next reload — it would load a truncated file.  The copy is raw, so an unreadable or
        invalid initial config keeps load_config's reference fallback."""
        import shutil

        try:
            snap = os.path.join(self.tmp, "config.gen0" + (os.path.splitext(self.config)[1] or ".yaml"))
            shutil.copyfile(self.config, snap)
            self.active = snap
        except OSError:
            pass  # missing file: the workers' load_config falls back to the default config

    def run(self) -> int:
        self.snapshot_initial()
        self.current = self.spawn()

        def on_hup(*_):
            self.reload_requested = True

        def on_stop(*_):
            self.stop_requested = True

        signal.signal(signal.SIGHUP, on_hup)
        signal.signal(signal.SIGTERM, on_stop)
        signal.signal(signal.SIGINT, on_stop)
        while True:
            if self.stop_requested:
                self.term(self.current + self.retiring)
                t0 = time.time()
                while any(p.poll() is None for p in self.current + self.retiring) and time.time() - t0 < 60:
                    time.sleep(0.05)
                return 0
            if self.poll_config():
                logging.getLogger("qmx.serve").warning("config %s changed: rolling reload", self.config)
                self.reload_requested = True
            if self.reload_requested:
                self.reload_requested = False
                self.reload()
            self.retiring = [p for p in self.retiring if p.poll() is None]
            dead = [p for p in self.current if p.poll() is not None]
            if dead:
                self.current = [p for p in self.current if p.poll() is None]
                time.sleep(self.backoff)
                self.backoff = min(self.backoff * 2, 30.0)
                self.restarts += len(dead)
                logging.getLogger("qmx.serve").warning("restarting %d worker(s) (exit %s)", len(dead),
                                                       [p.returncode for p in dead])
                self.current += self.spawn(len(dead) if self.args.impl == "python" else 1)
            else:
                self.backoff = max(0.5, self.backoff * 0.9)
            time.sleep(0.05)


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
    ap.add_argument("--gpus", type=int, default=1, help="rank processes on this node (one per GPU)")
    ap.add_argument("--watch-config", action="store_true",
                    help="roll a new worker generation in whenever the config file's content changes")
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
    if args.gpus > 1 and "QMX_RANK" not in os.environ:
        return launch_ranks(argv, args)
    return Supervisor(args, config).run()


def launch_ranks(argv, args) -> int:
    from .parallel.launcher import launch_ranks as _launch

    return _launch(argv if argv is not None else sys.argv[1:], args.gpus, args.device is None, args.port)


if __name__ == "__main__":
    sys.exit(main())
