"""Robustness of the data plane (VERDICT r1 / ADVICE r1 findings):

* slot generations — a stream result of a session that ended while its tick was in flight
  must never reach the session that re-opened the slot;
* client-abort churn through the shared engine (GPU-hub topology, CPU engine) with every
  completed response validated byte-exactly by the load generator;
* the Python ticker survives an engine exception;
* a native fault leaves a backtrace on stderr and the exit status names the signal.
"""
from __future__ import annotations

import asyncio
import json
import os
import signal
import subprocess
import sys
import time

import pytest

from quorum_amd.ops import build as qbuild
from quorum_amd.ops import native

from live_upstream import free_port, native_server

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
native_only = pytest.mark.skipif(not native.available(), reason="native extension not built")
TAGS = ["think", "reason"]
EV = (b'data: {"choices": [{"delta": {"content": "hello"}}]}\n\n')


@native_only
def test_slot_generation_survives_reuse():
    """Release a slot while its tick is unsettled, settle, let the next tick free it and
    re-open it: the in-flight result carries the OLD generation, the new open a new one."""
    e = native.require().CpuEngine(TAGS)
    s0, g0 = e.open_gen(0, True, True)
    e.feed(s0, EV)
    res, _, taken = e.tick_unsettled_gen(1, 0)
    assert taken == [s0] and res and res[0][0] == s0 and res[0][3] == g0
    e.release(s0)  # the session ended while the tick was in flight
    e.settle(taken)
    e.tick_unsettled_gen(1, 0)  # frees the slot
    s1, g1 = e.open_gen(1, True, True)
    assert s1 == s0 and g1 != g0  # same slot, new generation: stale results are detectable
    e.feed(s1, EV)
    res, _, taken = e.tick_unsettled_gen(1, 0)
    assert [(r[0], r[3]) for r in res] == [(s1, g1)]
    e.settle(taken)


def _mock(bin_dir, port, delay_us):
    return subprocess.Popen([os.path.join(bin_dir, "qmx_mock"), "--port", str(port), "--threads", "1", "--tokens",
                             "20", "--think", "1", "--delay-us", str(delay_us)],
                            stderr=subprocess.DEVNULL, start_new_session=True)


def _spec(path, exp, n):
    lines = ["role 1", "done 1"] + [f"stream chatcmpl-parallel-{i} exact {exp['stream_text'].encode().hex()}"
                                    for i in range(n)] + ["final absent", "error absent"]
    with open(path, "w") as f:
        f.write("\n".join(lines) + "\n")


@native_only
@pytest.mark.parametrize("threads,lanes,pipe", [(1, 2, "0"), (3, 3, "0"), (3, 2, "1")])
def test_abort_churn_shared_engine(tmp_path, monkeypatch, threads, lanes, pipe):
    """30% of clients hang up mid-stream while new requests keep landing on the same io
    loops (slot reuse under in-flight ticks): every completed response must still be
    exactly its own two backends' streams — also with pipelined lanes (QMX_PIPELINE=1: the
    next tick taken and prepared while the current one runs)."""
    import yaml  # noqa: F401

    monkeypatch.setenv("QMX_PIPELINE", pipe)

    sys.path.insert(0, ROOT)
    import bench

    bin_dir = os.path.dirname(str(qbuild.build_tools()[0]))
    ports = [free_port(), free_port()]
    mocks = [_mock(bin_dir, p, 300) for p in ports]
    try:
        cfg = {"primary_backends": [{"name": f"LLM{i + 1}", "url": f"http://127.0.0.1:{p}/v1", "model": f"m{i}"}
                                    for i, p in enumerate(ports)],
               "iterations": {"aggregation": {"strategy": "concatenate"}},
               "strategy": {"concatenate": {"separator": "\n-------------\n", "hide_intermediate_think": True,
                                            "skip_final_aggregation": True,
                                            "thinking_tags": ["think", "reason", "reasoning", "thought"]}},
               "settings": {"timeout": 30}}
        spec = str(tmp_path / "spec.txt")
        _spec(spec, bench.mock_expected(bin_dir), 2)
        lg = os.path.join(bin_dir, "qmx_loadgen")
        with native_server(cfg, threads=threads, shared=True, lanes=lanes) as port:
            out = subprocess.run([lg, "--port", str(port), "--conns", "48", "--requests", "1500", "--threads", "2",
                                  "--timeout", "120", "--expect", spec, "--abort-rate", "0.3"],
                                 capture_output=True, text=True, timeout=200)
        r = json.loads(out.stdout.strip().splitlines()[-1])
        assert r["aborted"] > 100, r
        assert r["invalid"] == 0 and r["errors"] == 0 and r["non200"] == 0, (r, out.stderr[-2000:])
        assert r["completed"] + r["aborted"] >= 1500
    finally:
        for m in mocks:
            os.killpg(m.pid, signal.SIGKILL)
            m.wait()


def test_ticker_survives_engine_exception():
    """An engine tick that raises fails the sessions in flight (their streams end) and the
    ticker keeps serving later sessions (reference: a failed backend never takes the
    proxy down, oai_proxy.py:252-259)."""
    from quorum_amd.ops.engine import PyEngine
    from quorum_amd.server.ticker import Ticker

    class Flaky(PyEngine):
        boom = 1

        def tick(self, created):
            if self.boom:
                self.boom -= 1
                raise RuntimeError("device lost")
            return super().tick(created)

    async def main():
        loop = asyncio.get_running_loop()
        t = Ticker(Flaky(TAGS), loop)
        s1 = t.open_session(1, True, True)
        t.feed(s1.slots[0], EV)
        assert await asyncio.wait_for(s1.queue.get(), 5) is None  # failed, not hung
        assert t.failures == 1 and s1.slots[0] in s1.failed
        t.release(s1)
        s2 = t.open_session(1, True, True)
        t.feed(s2.slots[0], EV)
        t.finish(s2.slots[0])
        got = []
        while True:
            x = await asyncio.wait_for(s2.queue.get(), 5)
            if x is None:
                break
            got.append(x)
        assert b"hello" in b"".join(got) and not t._task.done()
        t._task.cancel()

    asyncio.run(main())


@native_only
def test_native_fatal_signal_leaves_backtrace(tmp_path):
    """The silent-exit case of r1 (profiles/r1n_check2_bench_failed_run.json): a native
    worker that dies of a signal must say so on stderr, with a native backtrace."""
    import yaml

    cfg = {"primary_backends": [{"name": "LLM1", "url": f"http://127.0.0.1:{free_port()}/v1", "model": "m"}],
           "settings": {"timeout": 5}}
    p = tmp_path / "config.yaml"
    p.write_text(yaml.safe_dump(cfg))
    port = free_port()
    env = dict(os.environ, PYTHONPATH=ROOT)
    proc = subprocess.Popen([sys.executable, "-m", "quorum_amd.serve", "--native-worker", "--config", str(p),
                             "--port", str(port), "--engine", "cpu", "--threads", "1"],
                            env=env, stderr=subprocess.PIPE, stdout=subprocess.DEVNULL, start_new_session=True)
    try:
        from quorum_amd.serve import wait_healthy

        assert wait_healthy("127.0.0.1", port, 60)
        os.kill(proc.pid, signal.SIGSEGV)
        _, err = proc.communicate(timeout=30)
    finally:
        if proc.poll() is None:
            os.killpg(proc.pid, signal.SIGKILL)
    err = err.decode(errors="replace")
    assert proc.returncode == -signal.SIGSEGV, (proc.returncode, err[-2000:])
    assert "qmx fatal: signal 11" in err and "#0 " in err, err[-2000:]


def test_native_threads_never_read_environ_while_it_changes():
    """Regression (the round-2 'spread delta loss'): a native thread called getenv while a
    library thread wrote the environment, and the process died in getenv.  Native code now
    reads a snapshot (qmx_env.h).  Here the environment is rewritten in a tight loop (a
    putenv/unsetenv pair reallocates ``environ``) while a native server answers requests
    whose auth comes from OPENAI_API_KEY (read per request) — the server must survive and
    answer every one."""
    import threading

    import httpx

    from quorum_amd.ops import native as _native
    from conftest import cfg_parallel, sse_stream
    from live_upstream import LiveUpstream, native_server

    if not _native.available():
        pytest.skip("native extension not built")
    live = LiveUpstream()
    p1 = live.serve("a", ("stream", 200, sse_stream(["x"])))
    cfg = cfg_parallel(2, block={"separator": "\n", "hide_intermediate_think": True, "hide_final_think": False,
                                 "thinking_tags": ["think"], "skip_final_aggregation": False})
    for b in cfg["primary_backends"]:
        b["url"] = f"http://127.0.0.1:{p1}/v1"
    stop = threading.Event()

    def churn():
        i = 0
        while not stop.is_set():
            os.environ[f"QMX_CHURN_{i % 64}"] = "x" * (i % 200)
            os.environ.pop(f"QMX_CHURN_{(i + 32) % 64}", None)
            i += 1

    os.environ["OPENAI_API_KEY"] = "churn-key"
    th = threading.Thread(target=churn, daemon=True)
    try:
        with native_server(cfg, key_from_env=True) as port:
            th.start()
            with httpx.Client() as c:
                for _ in range(80):
                    r = c.post(f"http://127.0.0.1:{port}/chat/completions",
                               json={"messages": [{"role": "user", "content": "q"}], "stream": True}, timeout=20)
                    assert r.status_code == 200 and "[DONE]" in r.text
    finally:
        stop.set()
        if th.is_alive():
            th.join()
        for i in range(64):
            os.environ.pop(f"QMX_CHURN_{i}", None)
        os.environ.pop("OPENAI_API_KEY", None)
        live.close()
