"""The io loops' wait for in-flight ticks (QMX_LOOP_SPIN_US, default 4 us): a loop sleeps on a
timer until the spin window before a tick's due time and only then looks without a timer.
With no tick in flight it must block in epoll — the window may never turn an idle server into
a busy one (qmx_server.cpp, the run loop's wait; MI355X numbers in profiles/r6/spin)."""
import os
import time

import httpx
import pytest

from quorum_amd.ops import native

from conftest import cfg_parallel, sse_chunk
from live_upstream import LiveUpstream, native_server

pytestmark = pytest.mark.skipif(not native.available(), reason="native extension not built")

AUTH = {"Authorization": "Bearer test-key"}
MSG = [{"role": "user", "content": "hi"}]


def _body(words):
    return [b"".join([sse_chunk({"role": "assistant"})] + [sse_chunk({"content": w}) for w in words]
                     + [sse_chunk({}, finish="stop"), b"data: [DONE]\n\n"])]


@pytest.mark.parametrize("engine", ["cpu", pytest.param("hip", marks=pytest.mark.gpu)])
@pytest.mark.parametrize("spin_us", ["4", "1000"])
def test_idle_loops_block_with_the_spin_window(monkeypatch, spin_us, engine):
    """After traffic through the loops' asynchronous tick path, an idle server uses almost no
    CPU — even with a 1 ms window, which would spin through any tick still counted in flight.
    cpu: each loop's jobs on an engine worker, polled as grid doors are; hip: the loop-tick
    grid on the GPU (which the host stops after 50 ms without a post)."""
    monkeypatch.setenv("QMX_LOOP_SPIN_US", spin_us)
    live = LiveUpstream()
    p1 = live.serve("b1", ("stream", 200, _body([f"a{i} " for i in range(8)])))
    p2 = live.serve("b2", ("stream", 200, _body([f"b{i} " for i in range(8)])))
    try:
        cfg = cfg_parallel(2, block={"skip_final_aggregation": True, "hide_intermediate_think": True,
                                     "thinking_tags": ["think"]})
        cfg["primary_backends"][0]["url"] = f"http://127.0.0.1:{p1}/v1"
        cfg["primary_backends"][1]["url"] = f"http://127.0.0.1:{p2}/v1"
        with native_server(cfg, engine=engine, threads=2, tick_mode="loops") as port:
            base = f"http://127.0.0.1:{port}"
            with httpx.Client(timeout=30) as c:
                for _ in range(20):
                    r = c.post(base + "/chat/completions", json={"messages": MSG, "stream": True}, headers=AUTH)
                    assert r.status_code == 200 and r.text.rstrip().endswith("data: [DONE]")
                    assert "a7 " in r.text and "b7 " in r.text
            time.sleep(0.3)  # pooled connections parked, every tick applied
            c0, w0 = time.process_time(), time.monotonic()
            time.sleep(1.0)
            cpu, wall = time.process_time() - c0, time.monotonic() - w0
    finally:
        live.close()
    # two io loops spinning would be ~2 s of CPU per second; blocked loops, a few ms
    assert cpu < 0.15 * wall, (spin_us, cpu, wall)


def test_light_host_sessions_config(monkeypatch):
    """runtime.light_host_sessions reaches the native server's config (unset: -1, which
    leaves the choice to QMX_LIGHT_HOST — `serve` sets 2 for its workers, bench.py 0)."""
    from quorum_amd.runtime.native_server import native_config
    from quorum_amd.utils.config import RuntimeConfig

    monkeypatch.delenv("QMX_LIGHT_HOST", raising=False)
    cfg = cfg_parallel(2, block={"skip_final_aggregation": True})
    assert RuntimeConfig.from_config(cfg).light_host_sessions is None
    assert native_config(cfg, "127.0.0.1", 8001, "cpu", 0, 1)["light_host"] == -1
    cfg["runtime"] = {"light_host_sessions": 3}
    assert RuntimeConfig.from_config(cfg).light_host_sessions == 3
    assert native_config(cfg, "127.0.0.1", 8001, "cpu", 0, 1)["light_host"] == 3


def test_serve_and_bench_latency_mode_defaults(monkeypatch):
    """`serve` gives its native workers the latency mode (QMX_LIGHT_HOST=2) unless the caller
    set it; bench.py sets 0 first, so the headline measures the GPU path."""
    import subprocess

    from quorum_amd import serve

    seen = {}

    class P:
        def __init__(self, cmd, env=None, **kw):
            seen["env"] = env

    monkeypatch.setattr(subprocess, "Popen", P)
    monkeypatch.delenv("QMX_LIGHT_HOST", raising=False)
    serve.spawn_workers("c.yaml", "127.0.0.1", 1, 1, "hip", 0, impl="native")
    assert seen["env"]["QMX_LIGHT_HOST"] == "2"
    monkeypatch.setenv("QMX_LIGHT_HOST", "0")
    serve.spawn_workers("c.yaml", "127.0.0.1", 1, 1, "hip", 0, impl="native")
    assert seen["env"]["QMX_LIGHT_HOST"] == "0"
    with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "bench.py")) as f:
        src = f.read()
    assert 'os.environ.setdefault("QMX_LIGHT_HOST", "0")' in src
