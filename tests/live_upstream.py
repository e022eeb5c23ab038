"""Real-socket fake upstream backends + an in-process native server runner (for tests).

A behaviour is one of
    ("json", status, payload)          JSON response (content-length)
    ("text", status, text)             raw body
    ("stream", status, [chunks...])    chunked transfer, one HTTP chunk per item
    ("refuse",)                        nothing listening on the port
"""
from __future__ import annotations

import contextlib
import json
import socket
import threading
import time
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from typing import Any, Dict, List, Optional


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def free_port_block(n: int) -> int:
    """Base of n consecutive bindable ports, below the ephemeral range (the exchange mesh
    listens on base + rank; an ephemeral base would collide with sockets the kernel hands
    out next, e.g. to tests running in parallel)."""
    import random

    rng = random.Random()
    for _ in range(200):
        base = rng.randrange(20000, 30000 - n)
        socks = []
        try:
            for k in range(n):
                s = socket.socket()
                s.bind(("127.0.0.1", base + k))
                socks.append(s)
            return base
        except OSError:
            continue
        finally:
            for s in socks:
                s.close()
    raise RuntimeError("no free port block")


class _Handler(BaseHTTPRequestHandler):
    protocol_version = "HTTP/1.1"

    def log_message(self, *a):  # quiet
        pass

    def do_POST(self):
        n = int(self.headers.get("content-length", "0"))
        raw = self.rfile.read(n)
        try:
            body = json.loads(raw)
        except Exception:  # noqa: BLE001
            body = None
        srv = self.server
        srv.owner.calls.append({"host": srv.name, "path": self.path, "headers": {k.lower(): v for k, v in self.headers.items()},
                                "raw": raw, "body": body})
        beh = srv.owner.behaviours.get(srv.name)
        if callable(beh):
            beh = beh(body)
        kind = beh[0]
        if kind == "json":
            data = json.dumps(beh[2]).encode()
            self.send_response(beh[1])
            self.send_header("content-type", "application/json")
            self.send_header("content-length", str(len(data)))
            self.end_headers()
            self.wfile.write(data)
        elif kind == "text":
            data = beh[2].encode() if isinstance(beh[2], str) else beh[2]
            self.send_response(beh[1])
            self.send_header("content-type", "text/plain")
            self.send_header("content-length", str(len(data)))
            self.end_headers()
            self.wfile.write(data)
        elif kind == "stream":
            self.send_response(beh[1])
            self.send_header("content-type", "text/event-stream")
            self.send_header("transfer-encoding", "chunked")
            self.end_headers()
            for c in beh[2]:
                if isinstance(c, (int, float)):  # pause between chunks (slow upstream)
                    time.sleep(c)
                    continue
                self.wfile.write(b"%x\r\n%s\r\n" % (len(c), c))
                self.wfile.flush()
            self.wfile.write(b"0\r\n\r\n")
        self.wfile.flush()


class LiveUpstream:
    def __init__(self):
        self.behaviours: Dict[str, Any] = {}
        self.calls: List[Dict[str, Any]] = []
        self.ports: Dict[str, int] = {}
        self._servers = []

    def serve(self, name: str, behaviour, tls=None) -> int:
        """tls=(certfile, keyfile): serve HTTPS with that certificate."""
        self.behaviours[name] = behaviour
        if behaviour is not None and not callable(behaviour) and behaviour[0] == "refuse":
            self.ports[name] = free_port()
            return self.ports[name]
        srv = ThreadingHTTPServer(("127.0.0.1", 0), _Handler)
        if tls:
            import ssl

            ctx = ssl.SSLContext(ssl.PROTOCOL_TLS_SERVER)
            ctx.load_cert_chain(*tls)
            srv.socket = ctx.wrap_socket(srv.socket, server_side=True)
        srv.daemon_threads = True
        srv.owner = self
        srv.name = name
        t = threading.Thread(target=srv.serve_forever, daemon=True)
        t.start()
        self._servers.append(srv)
        self.ports[name] = srv.server_address[1]
        return self.ports[name]

    def close(self):
        for s in self._servers:
            s.shutdown()
            s.server_close()


@contextlib.contextmanager
def native_server(cfg: Dict[str, Any], engine: str = "cpu", threads: int = 1, env_key: str = "",
                  verify: bool = False, shared: Optional[bool] = None, lanes: Optional[int] = None,
                  key_from_env: bool = False, tick_mode: Optional[str] = None):
    """Run the C++ data plane in-process (background thread) for one config.

    verify: run the shadow CPU-oracle engine (server_counters()['verify_mismatches']).
    shared: one engine per process shared by all io loops (None = the config's default).
    lanes: tick lanes of the shared engine (None = the config's default).
    tick_mode: "loops" runs the io loops' asynchronous tick path (with the cpu engine: each
    loop's jobs on an engine worker thread, polled by the loop as a GPU grid's doors are)."""
    import http.client
    import os

    from quorum_amd.ops import native
    from quorum_amd.runtime.native_server import native_config

    ext = native.require()
    port = free_port()
    d = native_config(cfg, "127.0.0.1", port, engine, 0, threads)
    d["install_signals"] = False
    d["env_api_key"] = env_key
    d["api_key_from_env"] = key_from_env  # default: the test's key, not the shared process env
    d["verify"] = verify
    if shared is not None:
        d["shared_engine"] = int(shared)
    if lanes is not None:
        d["tick_lanes"] = int(lanes)
    if tick_mode is not None:
        d["tick_mode"] = tick_mode
    th = threading.Thread(target=ext.run_server, args=(d,), daemon=True)
    th.start()
    t0 = time.time()
    while time.time() - t0 < 20:
        try:
            c = http.client.HTTPConnection("127.0.0.1", port, timeout=1)
            c.request("GET", "/health")
            if c.getresponse().status == 200:
                break
        except OSError:
            time.sleep(0.02)
    try:
        yield port
    finally:
        ext.stop_server()
        th.join(timeout=10)
