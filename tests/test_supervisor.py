"""Process lifecycle: graceful drain (SIGTERM), rolling config reload (SIGHUP), crash restart.

The supervisor (``python -m quorum_amd.serve``) runs worker generations on one
SO_REUSEPORT port.  A reload starts the new generation, waits until it is listening,
then drains the old one, so a client hammering the port never sees a failed request;
a killed worker is restarted; an invalid config is rejected without disturbing service.
"""
import os
import signal
import subprocess
import sys
import threading
import time

import httpx
import pytest
import yaml

from quorum_amd.ops import native

from conftest import cfg_parallel, sse_stream
from live_upstream import LiveUpstream, free_port, free_port_block

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
AUTH = {"Authorization": "Bearer k"}
MSG = [{"role": "user", "content": "hi"}]
BLOCK = {"separator": "\n--\n", "hide_intermediate_think": True, "hide_final_think": False,
         "thinking_tags": ["think"], "skip_final_aggregation": False}


def _write(path, urls, drain=5.0):
    cfg = cfg_parallel(len(urls), block=BLOCK)
    for b, u in zip(cfg["primary_backends"], urls):
        b["url"] = u
    cfg["runtime"] = {"drain_timeout": drain}
    with open(path, "w") as f:
        yaml.safe_dump(cfg, f)


def _final(text):
    for seg in text.split("\n\n"):
        if '"chatcmpl-parallel-final"' in seg:
            import json
            return json.loads(seg[6:])["choices"][0]["delta"]["content"]
    return None


def _post(port):
    return httpx.post(f"http://127.0.0.1:{port}/chat/completions", json={"messages": MSG, "stream": True},
                      headers=AUTH, timeout=20)


def _wait(port, pred, timeout=60):
    t0 = time.time()
    while time.time() - t0 < timeout:
        try:
            r = _post(port)
            if pred(r):
                return r
        except httpx.HTTPError:
            pass
        time.sleep(0.05)
    raise AssertionError("condition not reached")


@pytest.mark.parametrize("impl", ["native", "python"])
def test_reload_drain_restart(tmp_path, impl):
    if impl == "native" and not native.available():
        pytest.skip("native extension not built")
    live = LiveUpstream()
    pa = live.serve("a", ("stream", 200, sse_stream(["AAA"])))
    pb = live.serve("b", ("stream", 200, sse_stream(["BBB"])))
    cfg = str(tmp_path / "config.yaml")
    _write(cfg, [f"http://127.0.0.1:{pa}/v1", f"http://127.0.0.1:{pa}/v1"])
    port = free_port()
    env = dict(os.environ, PYTHONPATH=ROOT, QMX_ENGINE="cpu" if impl == "native" else "python")
    sup = subprocess.Popen([sys.executable, "-m", "quorum_amd.serve", "--impl", impl, "--engine",
                            "cpu" if impl == "native" else "python", "--config", cfg, "--port", str(port),
                            "--workers", "2", "--threads", "2"], cwd=ROOT, env=env, start_new_session=True)
    errors, stop = [], threading.Event()

    def hammer():
        while not stop.is_set():
            try:
                r = _post(port)
                if r.status_code != 200 or _final(r.text) is None:
                    errors.append(r.status_code)
            except httpx.HTTPError as e:
                errors.append(repr(e))

    try:
        assert _final(_wait(port, lambda r: r.status_code == 200).text) == "AAA\n\n--\nAAA"
        th = threading.Thread(target=hammer)
        th.start()
        # 1. rolling reload to backend b: no failed request while generations swap
        _write(cfg, [f"http://127.0.0.1:{pb}/v1", f"http://127.0.0.1:{pb}/v1"])
        os.kill(sup.pid, signal.SIGHUP)
        _wait(port, lambda r: _final(r.text) == "BBB\n\n--\nBBB")
        time.sleep(0.5)
        # 2. an invalid config is rejected; the current generation keeps serving
        with open(cfg, "w") as f:
            f.write("primary_backends: [unclosed\n")
        os.kill(sup.pid, signal.SIGHUP)
        time.sleep(1.0)
        assert _final(_post(port).text) == "BBB\n\n--\nBBB"
        stop.set()
        th.join()
        assert errors == [], errors[:5]
        # 3. crash restart: kill every worker process of the supervisor
        out = subprocess.run(["pgrep", "-P", str(sup.pid)], capture_output=True, text=True).stdout.split()
        assert out
        for pid in out:
            os.kill(int(pid), signal.SIGKILL)
        _wait(port, lambda r: _final(r.text) == "BBB\n\n--\nBBB")
    finally:
        stop.set()
        # 4. graceful stop
        os.kill(sup.pid, signal.SIGTERM)
        try:
            rc = sup.wait(timeout=30)
        except subprocess.TimeoutExpired:
            os.killpg(sup.pid, signal.SIGKILL)
            rc = None
        live.close()
    assert rc == 0


def test_config_watch_rolls_new_generation(tmp_path):
    """``runtime.watch_config``: editing the YAML (no signal) rolls a new worker generation in
    while a client hammers the port — no request fails, the new backend answers, an edit that
    does not validate is ignored (the current generation keeps serving), and rewriting the
    same bytes is not a change (reference: uvicorn --reload --reload-include "*.yaml",
    Makefile:4, which restarts and drops in-flight requests)."""
    if not native.available():
        pytest.skip("native extension not built")
    live = LiveUpstream()
    pa = live.serve("a", ("stream", 200, sse_stream(["AAA"])))
    pb = live.serve("b", ("stream", 200, sse_stream(["BBB"])))
    cfg = str(tmp_path / "config.yaml")

    def write(url):
        _write(cfg, [url, url])
        with open(cfg) as f:
            c = yaml.safe_load(f)
        c["runtime"].update(watch_config=True, watch_interval=0.1)
        with open(cfg, "w") as f:
            yaml.safe_dump(c, f)

    write(f"http://127.0.0.1:{pa}/v1")
    port = free_port()
    env = dict(os.environ, PYTHONPATH=ROOT, QMX_ENGINE="cpu")
    sup = subprocess.Popen([sys.executable, "-m", "quorum_amd.serve", "--impl", "native", "--engine", "cpu",
                            "--config", cfg, "--port", str(port), "--threads", "2"], cwd=ROOT, env=env,
                           start_new_session=True)
    errors, stop = [], threading.Event()

    def hammer():
        while not stop.is_set():
            try:
                r = _post(port)
                if r.status_code != 200 or _final(r.text) is None:
                    errors.append(r.status_code)
            except httpx.HTTPError as e:
                errors.append(repr(e))

    th = threading.Thread(target=hammer)
    try:
        assert _final(_wait(port, lambda r: r.status_code == 200).text) == "AAA\n\n--\nAAA"
        th.start()
        write(f"http://127.0.0.1:{pb}/v1")  # an edit, no SIGHUP
        _wait(port, lambda r: _final(r.text) == "BBB\n\n--\nBBB", timeout=30)
        time.sleep(0.5)
        with open(cfg, "w") as f:  # an edit that does not validate: ignored
            f.write("primary_backends: [unclosed\n")
        time.sleep(1.0)
        assert _final(_post(port).text) == "BBB\n\n--\nBBB"
        stop.set()
        th.join()
        assert errors == [], errors[:5]
    finally:
        stop.set()
        if th.is_alive():
            th.join()
        os.kill(sup.pid, signal.SIGTERM)
        try:
            sup.wait(timeout=30)
        except subprocess.TimeoutExpired:
            os.killpg(sup.pid, signal.SIGKILL)
        live.close()


def test_watch_poll_ignores_identical_rewrite(tmp_path):
    """Supervisor.poll_config: a touch or an identical rewrite is not a change; new bytes are."""
    from types import SimpleNamespace

    from quorum_amd.serve import Supervisor

    cfg = tmp_path / "c.yaml"
    cfg.write_text("settings: {timeout: 5}\nruntime: {watch_config: true, watch_interval: 0.05}\n")
    sup = Supervisor(SimpleNamespace(watch_config=False), str(cfg))
    assert sup.watch and sup.watch_interval == 0.05
    time.sleep(0.06)
    assert not sup.poll_config()
    os.utime(cfg, None)
    cfg.write_text(cfg.read_text())  # same bytes, new mtime
    time.sleep(0.06)
    assert not sup.poll_config()
    cfg.write_text("settings: {timeout: 6}\nruntime: {watch_config: true, watch_interval: 0.05}\n")
    time.sleep(0.06)
    assert sup.poll_config()
    time.sleep(0.06)
    assert not sup.poll_config()


def test_native_drain_finishes_inflight(tmp_path):
    """SIGTERM to a native worker: the listener closes at once, an in-flight slow stream
    still completes, then the process exits 0."""
    if not native.available():
        pytest.skip("native extension not built")
    import json as _j

    slow = []
    for i in range(6):  # numbers = pauses (seconds) between upstream chunks
        slow += [b"data: " + _j.dumps({"choices": [{"delta": {"content": f"t{i} "}}]}).encode() + b"\n\n", 0.2]
    slow += [b"data: [DONE]\n\n"]
    live = LiveUpstream()
    pa = live.serve("a", ("stream", 200, slow))
    cfg = str(tmp_path / "config.yaml")
    _write(cfg, [f"http://127.0.0.1:{pa}/v1"] * 2)
    port = free_port()
    env = dict(os.environ, PYTHONPATH=ROOT)
    w = subprocess.Popen([sys.executable, "-m", "quorum_amd.serve", "--native-worker", "--engine", "cpu", "--config",
                          cfg, "--port", str(port), "--threads", "1"], cwd=ROOT, env=env, start_new_session=True)
    try:
        _wait(port, lambda r: r.status_code == 200)
        res = {}

        def client():
            with httpx.Client() as c:
                with c.stream("POST", f"http://127.0.0.1:{port}/chat/completions",
                              json={"messages": MSG, "stream": True}, headers=AUTH, timeout=20) as r:
                    res["status"] = r.status_code
                    res["body"] = b"".join(r.iter_bytes())
        th = threading.Thread(target=client)
        th.start()
        # SIGTERM once the stream is in flight (its head arrived), not after a fixed sleep: on
        # a loaded machine the client may not have connected yet and would meet a closed port
        t_end = time.time() + 10
        while "status" not in res and time.time() < t_end:
            time.sleep(0.01)
        os.kill(w.pid, signal.SIGTERM)
        th.join(timeout=20)
        assert res.get("status") == 200
        assert res["body"].rstrip().endswith(b"data: [DONE]")
        assert w.wait(timeout=20) == 0
        with pytest.raises(httpx.HTTPError):
            _post(port)
    finally:
        if w.poll() is None:
            os.killpg(w.pid, signal.SIGKILL)
        live.close()


def test_launcher_two_ranks_spread(tmp_path):
    """`serve --gpus 2`: two rank supervisors on one port; with placement: spread each
    session's second backend stream runs on the other rank (TCP exchange on CPU)."""
    if not native.available():
        pytest.skip("native extension not built")
    live = LiveUpstream()
    pa = live.serve("a", ("stream", 200, sse_stream(["AAA"])))
    pb = live.serve("b", ("stream", 200, sse_stream(["BBB"])))
    cfg = str(tmp_path / "config.yaml")
    _write(cfg, [f"http://127.0.0.1:{pa}/v1", f"http://127.0.0.1:{pb}/v1"])
    with open(cfg) as f:
        c = yaml.safe_load(f)
    c["runtime"]["placement"] = "spread"
    with open(cfg, "w") as f:
        yaml.safe_dump(c, f)
    port = free_port()
    env = dict(os.environ, PYTHONPATH=ROOT, QMX_XCHG_PORT=str(free_port_block(2)))
    env.pop("QMX_RANK", None)
    sup = subprocess.Popen([sys.executable, "-m", "quorum_amd.serve", "--impl", "native", "--engine", "cpu",
                            "--gpus", "2", "--config", cfg, "--port", str(port), "--threads", "1"], cwd=ROOT,
                           env=env, start_new_session=True)
    try:
        _wait(port, lambda r: r.status_code == 200)
        remote = 0.0
        for _ in range(40):
            r = _post(port)
            assert _final(r.text) == "AAA\n\n--\nBBB"
            m = httpx.get(f"http://127.0.0.1:{port}/metrics").text
            remote = max(remote, float([ln for ln in m.splitlines()
                                        if ln.startswith("qmx_remote_streams_total")][0].split()[1]))
        assert remote >= 1
    finally:
        os.kill(sup.pid, signal.SIGTERM)
        try:
            rc = sup.wait(timeout=40)
        except subprocess.TimeoutExpired:
            os.killpg(sup.pid, signal.SIGKILL)
            rc = None
        live.close()
    assert rc == 0


def test_rank_death_survivors_keep_serving(tmp_path):
    """kill one rank's worker mid-traffic (spread placement, TCP exchange).
    The exchange round fails, every rank falls back to local placement, and no client
    request fails at the HTTP level; full answers resume immediately."""
    if not native.available():
        pytest.skip("native extension not built")
    live = LiveUpstream()
    pa = live.serve("a", ("stream", 200, sse_stream(["AAA"])))
    pb = live.serve("b", ("stream", 200, sse_stream(["BBB"])))
    cfg = str(tmp_path / "config.yaml")
    _write(cfg, [f"http://127.0.0.1:{pa}/v1", f"http://127.0.0.1:{pb}/v1"])
    with open(cfg) as f:
        c = yaml.safe_load(f)
    c["runtime"]["placement"] = "spread"
    with open(cfg, "w") as f:
        yaml.safe_dump(c, f)
    port = free_port()
    env = dict(os.environ, PYTHONPATH=ROOT, QMX_XCHG_PORT=str(free_port_block(2)))
    env.pop("QMX_RANK", None)
    sup = subprocess.Popen([sys.executable, "-m", "quorum_amd.serve", "--impl", "native", "--engine", "cpu",
                            "--gpus", "2", "--config", cfg, "--port", str(port), "--threads", "1"], cwd=ROOT,
                           env=env, start_new_session=True)
    errors, finals, stop = [], [], threading.Event()

    def hammer():
        while not stop.is_set():
            try:
                r = _post(port)
                if r.status_code != 200 or not r.text.rstrip().endswith("data: [DONE]"):
                    errors.append(r.status_code)
                finals.append(_final(r.text))
            except httpx.HTTPError as e:
                errors.append(repr(e))
    try:
        _wait(port, lambda r: _final(r.text) == "AAA\n\n--\nBBB")
        th = threading.Thread(target=hammer)
        th.start()
        time.sleep(1.0)
        ranks = subprocess.run(["pgrep", "-P", str(sup.pid)], capture_output=True, text=True).stdout.split()
        assert len(ranks) == 2
        victims = subprocess.run(["pgrep", "-P", ranks[1]], capture_output=True, text=True).stdout.split()
        assert victims
        for v in victims:  # rank 1's native worker dies abruptly
            os.kill(int(v), signal.SIGKILL)
        time.sleep(3.0)
        n_before = len(finals)
        time.sleep(1.5)
        stop.set()
        th.join(timeout=30)
        # connections that were open on the killed process may reset; nothing else may fail
        assert len([e for e in errors if "RemoteProtocolError" not in str(e) and "ReadError" not in str(e)
                    and "ConnectError" not in str(e)]) == 0, errors[:5]
        assert all(f == "AAA\n\n--\nBBB" for f in finals[n_before:]), finals[n_before:][:5]
        assert len(finals) - n_before > 5
    finally:
        stop.set()
        os.kill(sup.pid, signal.SIGTERM)
        try:
            sup.wait(timeout=40)
        except subprocess.TimeoutExpired:
            os.killpg(sup.pid, signal.SIGKILL)
        live.close()


def test_rank_restart_exchange_reforms(tmp_path):
    """SURVEY §5.3 re-join: rank 1's worker is killed, its supervisor restarts it, the new
    process dials the mesh again (the higher rank redials) and spread placement resumes —
    streams run on rank 1 again, rank 0 counts the re-join, and every answer is complete."""
    if not native.available():
        pytest.skip("native extension not built")
    live = LiveUpstream()
    pa = live.serve("a", ("stream", 200, sse_stream(["AAA"])))
    pb = live.serve("b", ("stream", 200, sse_stream(["BBB"])))
    cfg = str(tmp_path / "config.yaml")
    _write(cfg, [f"http://127.0.0.1:{pa}/v1", f"http://127.0.0.1:{pb}/v1"])
    with open(cfg) as f:
        c = yaml.safe_load(f)
    c["runtime"]["placement"] = "spread"
    with open(cfg, "w") as f:
        yaml.safe_dump(c, f)
    port = free_port()
    env = dict(os.environ, PYTHONPATH=ROOT, QMX_XCHG_PORT=str(free_port_block(2)))
    env.pop("QMX_RANK", None)
    sup = subprocess.Popen([sys.executable, "-m", "quorum_amd.serve", "--impl", "native", "--engine", "cpu",
                            "--gpus", "2", "--config", cfg, "--port", str(port), "--threads", "1"], cwd=ROOT,
                           env=env, start_new_session=True)

    def metric(text, name):
        for ln in text.splitlines():
            if ln.startswith(name + " "):
                return float(ln.split()[1])
        return 0.0

    def scrape_all(n=12):  # the shared port answers from either rank
        out = []
        for _ in range(n):
            with httpx.Client() as cl:  # a fresh connection: another SO_REUSEPORT pick
                out.append(cl.get(f"http://127.0.0.1:{port}/metrics").text)
        return out

    try:
        _wait(port, lambda r: _final(r.text) == "AAA\n\n--\nBBB")
        t0 = time.time()  # both ranks up and meshed before the kill
        while not all(metric(m, "qmx_exchange_peers_up") == 2 for m in scrape_all(6)):
            assert time.time() - t0 < 30, "mesh never formed"
            time.sleep(0.2)
        ranks = subprocess.run(["pgrep", "-P", str(sup.pid)], capture_output=True, text=True).stdout.split()
        assert len(ranks) == 2
        victims = subprocess.run(["pgrep", "-P", ranks[1]], capture_output=True, text=True).stdout.split()
        assert victims
        for v in victims:
            os.kill(int(v), signal.SIGKILL)
        # the restarted worker re-joins: both ranks see 2 peers up, rank 0 counted a re-join
        t0 = time.time()
        while time.time() - t0 < 30:
            ms = scrape_all(6)
            if all(metric(m, "qmx_exchange_peers_up") == 2 for m in ms) and \
                    max(metric(m, "qmx_exchange_rejoins_total") for m in ms) >= 1:
                break
            time.sleep(0.3)
        else:
            raise AssertionError("exchange did not re-form")
        for _ in range(40):
            r = _post(port)
            assert r.status_code == 200 and _final(r.text) == "AAA\n\n--\nBBB"
        # streams are spread onto the new rank-1 process again (its own counter starts at 0)
        ms = scrape_all()
        assert all(metric(m, "qmx_remote_streams_total") >= 1 for m in ms), [metric(m, "qmx_remote_streams_total")
                                                                             for m in ms]
    finally:
        os.kill(sup.pid, signal.SIGTERM)
        try:
            sup.wait(timeout=40)
        except subprocess.TimeoutExpired:
            os.killpg(sup.pid, signal.SIGKILL)
        live.close()
