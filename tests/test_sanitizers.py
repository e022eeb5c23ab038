"""ASan + UBSan builds of the host runtime (GPU sanitizers are not used).

* qmx_fuzz_asan: streaming-invariance / JSON round-trip fuzzer over the C++ engine + DOM.
* qmx_server_asan: the standalone C++ data plane under traffic that exercises every
  connection-lifetime path — parallel streams, aborts (content:null), upstream 5xx,
  refused connections, mid-stream disconnects, client disconnects mid-response,
  keep-alive reuse, aggregator calls — then a clean SIGINT shutdown.  Any ASan/UBSan
  report fails the test.
"""
import json
import os
import signal
import socket
import subprocess
import time

import httpx
import pytest

from quorum_amd.ops import native

from conftest import cfg_parallel, completion, sse_chunk, sse_stream
from live_upstream import LiveUpstream, free_port

pytestmark = pytest.mark.skipif(not native.available(), reason="native toolchain/extension not built")
ASAN_ENV = {"ASAN_OPTIONS": "detect_leaks=0:abort_on_error=0:halt_on_error=1",
            "UBSAN_OPTIONS": "halt_on_error=1:print_stacktrace=1"}


@pytest.fixture(scope="module")
def san_bins():
    from quorum_amd.ops import build

    return {p.name: p for p in build.build_sanitized()}


def test_fuzz_host_asan(san_bins):
    for seed in ("1", "20260101"):
        r = subprocess.run([str(san_bins["qmx_fuzz_asan"]), "1500", seed], capture_output=True, text=True,
                           timeout=300, env=dict(os.environ, **ASAN_ENV))
        assert r.returncode == 0, r.stderr[-3000:]
        assert json.loads(r.stdout.strip().splitlines()[-1])["failures"] == 0
        assert "ERROR: AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr


def test_server_asan_traffic(san_bins, tmp_path):
    from quorum_amd.runtime.native_server import native_config

    live = LiveUpstream()
    stream = sse_stream(["Hel", "lo <think>x</think> wor", "ld"])
    ports = {
        "ok": live.serve("ok", ("stream", 200, stream)),
        "null": live.serve("null", ("stream", 200, [sse_chunk({"content": "a"}), sse_chunk({"content": None}),
                                                      sse_chunk({"content": "b"}), b"data: [DONE]\n\n"])),
        "e500": live.serve("e500", ("json", 500, {"error": {"message": "boom"}})),
        "refused": live.serve("refused", ("refuse",)),
        "agg": live.serve("agg", lambda body: (("stream", 200, stream) if body.get("stream")
                                               else ("json", 200, completion("SYNTH")))),
    }
    # a backend that drops the connection mid-stream
    drop_srv = socket.socket()
    drop_srv.bind(("127.0.0.1", 0))
    drop_srv.listen(64)
    drop_port = drop_srv.getsockname()[1]
    import threading

    def dropper():
        while True:
            try:
                c, _ = drop_srv.accept()
            except OSError:
                return
            c.recv(65536)
            c.sendall(b"HTTP/1.1 200 OK\r\ncontent-type: text/event-stream\r\ntransfer-encoding: chunked\r\n\r\n"
                      b"20\r\ndata: {\"choices\": [{\"delta\": {\"con")
            c.close()
    threading.Thread(target=dropper, daemon=True).start()

    urls = [f"http://127.0.0.1:{ports[k]}/v1" for k in ("ok", "null", "e500", "refused", "agg")]
    urls.append(f"http://127.0.0.1:{drop_port}/v1")
    block = {"separator": "\n--\n", "hide_intermediate_think": True, "hide_final_think": True,
             "thinking_tags": ["think"], "skip_final_aggregation": False}
    cfgs = {
        "concat": cfg_parallel(6, block=block),
        "aggregate": cfg_parallel(6, strategy="aggregate",
                                  block={"aggregator_backend": "LLM5", "prompt_template": "P {responses}"}),
    }
    for cfg in cfgs.values():
        for b, u in zip(cfg["primary_backends"], urls):
            b["url"] = u
    errs = []
    try:
        for name, cfg in cfgs.items():
            port = free_port()
            d = native_config(cfg, "127.0.0.1", port, "cpu", 0, 2)
            d["env_api_key"] = ""
            d["api_key_from_env"] = False
            path = tmp_path / f"{name}.json"
            path.write_text(json.dumps(d))
            srv = subprocess.Popen([str(san_bins["qmx_server_asan"]), str(path)], stderr=subprocess.PIPE,
                                   env=dict(os.environ, **ASAN_ENV))
            try:
                t0 = time.time()
                while time.time() - t0 < 30:
                    try:
                        if httpx.get(f"http://127.0.0.1:{port}/health", timeout=1).status_code == 200:
                            break
                    except httpx.HTTPError:
                        time.sleep(0.05)
                req = {"messages": [{"role": "user", "content": "q"}], "stream": True}
                hdr = {"Authorization": "Bearer k"}
                with httpx.Client(base_url=f"http://127.0.0.1:{port}") as c:
                    for i in range(20):
                        r = c.post("/chat/completions", json=req, headers=hdr, timeout=30)
                        assert r.status_code == 200 and r.text.rstrip().endswith("data: [DONE]")
                        r = c.post("/v1/chat/completions", json={"messages": req["messages"]}, headers=hdr,
                                   timeout=30)
                        assert r.status_code in (200, 500)
                # clients that vanish mid-response
                for i in range(10):
                    s = socket.create_connection(("127.0.0.1", port))
                    body = json.dumps(req).encode()
                    s.sendall(b"POST /chat/completions HTTP/1.1\r\nhost: x\r\nauthorization: Bearer k\r\n"
                              b"content-type: application/json\r\ncontent-length: %d\r\n\r\n%s" % (len(body), body))
                    if i % 2:
                        s.recv(64)
                    s.close()
                # garbage requests
                for junk in (b"GARBAGE\r\n\r\n", b"POST /chat/completions HTTP/1.1\r\ncontent-length: 5\r\n\r\n{bad}"):
                    s = socket.create_connection(("127.0.0.1", port))
                    s.sendall(junk)
                    s.settimeout(5)
                    try:
                        s.recv(4096)
                    except OSError:
                        pass
                    s.close()
                assert httpx.get(f"http://127.0.0.1:{port}/metrics").status_code == 200
            finally:
                srv.send_signal(signal.SIGINT)
                try:
                    _, err = srv.communicate(timeout=30)
                except subprocess.TimeoutExpired:
                    srv.kill()
                    _, err = srv.communicate()
                err = err.decode(errors="replace")
                if srv.returncode != 0 or "AddressSanitizer" in err or "runtime error" in err:
                    errs.append((name, srv.returncode, err[-4000:]))
    finally:
        drop_srv.close()
        live.close()
    assert not errs, errs


@pytest.mark.parametrize("mode", ["lanes", "loops"])
def test_server_tsan_shared_engine_lanes(tmp_path, mode):
    """ThreadSanitizer build of the data plane under concurrent clients with aborting and
    failing backends, plus the verify shadow.  lanes: 4 io loops share one engine with 3 tick
    lanes (the GPU-hub topology, CPU engine).  loops: the loop-tick protocol — every io loop
    posts its jobs to its own engine's worker thread and polls them, two in flight (the grid
    doors' pattern, AsyncCpuEngine).  Any data race report fails the test."""
    import concurrent.futures as cf

    from quorum_amd.ops import build
    from quorum_amd.runtime.native_server import native_config

    tsan = build.build_tsan()
    live = LiveUpstream()
    stream = sse_stream(["Hel", "lo <think>x</think> wor", "ld"])
    null_stream = [sse_chunk({"content": "a"}), sse_chunk({"content": None}), b"data: [DONE]\n\n"]
    ports = [live.serve("ok", ("stream", 200, stream)), live.serve("null", ("stream", 200, null_stream)),
             live.serve("e500", ("json", 500, {"error": {"message": "boom"}}))]
    urls = [f"http://127.0.0.1:{p}/v1" for p in ports]
    block = {"separator": "\n--\n", "hide_intermediate_think": True, "hide_final_think": True,
             "thinking_tags": ["think"], "skip_final_aggregation": False}
    cfg = cfg_parallel(3, block=block)
    for b, u in zip(cfg["primary_backends"], urls):
        b["url"] = u
    port = free_port()
    d = native_config(cfg, "127.0.0.1", port, "cpu", 0, 4)
    d.update(env_api_key="", api_key_from_env=False, verify=True)
    if mode == "lanes":
        d.update(shared_engine=1, tick_lanes=3)
    else:
        d.update(tick_mode="loops")
    path = tmp_path / "tsan.json"
    path.write_text(json.dumps(d))
    # pipelined lanes on (QMX_PIPELINE=1): the next tick is taken while the current one runs;
    # lazy wakes (QMX_LAZY_WAKE=1): lanes skip the eventfd of an io loop that is not waiting
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=0:second_deadlock_stack=1:report_signal_unsafe=0",
               QMX_PIPELINE="1", QMX_LAZY_WAKE="1")
    srv = subprocess.Popen([str(tsan), str(path)], stderr=subprocess.PIPE, env=env)
    try:
        t0 = time.time()
        while time.time() - t0 < 60:
            try:
                if httpx.get(f"http://127.0.0.1:{port}/health", timeout=1).status_code == 200:
                    break
            except httpx.HTTPError:
                time.sleep(0.1)
        req = {"messages": [{"role": "user", "content": "q"}], "stream": True}

        def client(i):
            with httpx.Client(base_url=f"http://127.0.0.1:{port}") as c:
                for k in range(12):
                    body = req if (i + k) % 3 else {"messages": req["messages"]}
                    r = c.post("/chat/completions", json=body, headers={"Authorization": "Bearer k"}, timeout=60)
                    assert r.status_code in (200, 500)
                    if body.get("stream"):
                        assert r.text.rstrip().endswith("data: [DONE]")
            return True

        with cf.ThreadPoolExecutor(8) as ex:
            assert all(ex.map(client, range(8)))
        assert httpx.get(f"http://127.0.0.1:{port}/metrics").status_code == 200
    finally:
        srv.send_signal(signal.SIGINT)
        try:
            _, err = srv.communicate(timeout=60)
        except subprocess.TimeoutExpired:
            srv.kill()
            _, err = srv.communicate()
        live.close()
    err = err.decode(errors="replace")
    assert "ThreadSanitizer" not in err, err[-6000:]
    assert srv.returncode == 0, err[-3000:]


def test_server_asan_abort_churn_shared_engine(san_bins, tmp_path):
    """ASan/UBSan data plane, shared engine with 3 tick lanes over 3 io loops (the GPU-hub
    topology, CPU engine), driven by the validating load generator with 30% of clients
    hanging up mid-stream (session teardown while ticks are in flight, slot reuse): no
    sanitizer report, no invalid response, clean shutdown."""
    import sys

    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    from quorum_amd.ops import build
    from quorum_amd.runtime.native_server import native_config

    bin_dir = os.path.dirname(str(build.build_tools()[0]))
    mports = [free_port(), free_port()]
    mocks = [subprocess.Popen([os.path.join(bin_dir, "qmx_mock"), "--port", str(p), "--threads", "1",
                               "--delay-us", "200"], stderr=subprocess.DEVNULL) for p in mports]
    cfg = cfg_parallel(2, block={"separator": "\n--\n", "hide_intermediate_think": True,
                                 "thinking_tags": ["think", "reason", "reasoning", "thought"],
                                 "skip_final_aggregation": True})
    for b, p in zip(cfg["primary_backends"], mports):
        b["url"] = f"http://127.0.0.1:{p}/v1"
    port = free_port()
    d = native_config(cfg, "127.0.0.1", port, "cpu", 0, 3)
    d.update(env_api_key="", api_key_from_env=False, shared_engine=1, tick_lanes=3)
    path = tmp_path / "churn.json"
    path.write_text(json.dumps(d))
    spec = tmp_path / "spec.txt"
    text = bench.mock_expected(bin_dir)["stream_text"].encode().hex()
    spec.write_text(f"role 1\ndone 1\nstream chatcmpl-parallel-0 exact {text}\n"
                    f"stream chatcmpl-parallel-1 exact {text}\nfinal absent\nerror absent\n")
    srv = subprocess.Popen([str(san_bins["qmx_server_asan"]), str(path)], stderr=subprocess.PIPE,
                           env=dict(os.environ, **ASAN_ENV))
    try:
        t0 = time.time()
        while time.time() - t0 < 30:
            try:
                if httpx.get(f"http://127.0.0.1:{port}/health", timeout=1).status_code == 200:
                    break
            except httpx.HTTPError:
                time.sleep(0.05)
        out = subprocess.run([os.path.join(bin_dir, "qmx_loadgen"), "--port", str(port), "--conns", "32",
                              "--requests", "2000", "--threads", "2", "--timeout", "120", "--expect", str(spec),
                              "--abort-rate", "0.3"], capture_output=True, text=True, timeout=200)
        r = json.loads(out.stdout.strip().splitlines()[-1])
    finally:
        srv.send_signal(signal.SIGINT)
        try:
            _, err = srv.communicate(timeout=30)
        except subprocess.TimeoutExpired:
            srv.kill()
            _, err = srv.communicate()
        for m in mocks:
            m.kill()
            m.wait()
    err = err.decode(errors="replace")
    assert srv.returncode == 0 and "AddressSanitizer" not in err and "runtime error" not in err, err[-4000:]
    assert r["aborted"] > 200 and r["invalid"] == 0 and r["errors"] == 0, (r, out.stderr[-2000:])


def test_server_tsan_self_spread_rounds(tmp_path):
    """ThreadSanitizer data plane with the exchange live: QMX_SPREAD_SELF at one rank sends the
    odd backends through the rank's own exchange (mesh thread, tcpbulk round executor on the
    bulk thread, four io loops), every final text through a round (eager 0), round 2 stalled
    to its timeout (QMX_XCHG_FAULT_STALL_ROUND) while clients leave mid-response — the deferred
    shadow-slot releases (forget_bulk -> X_RELEASE) and the mesh fallback run concurrently
    with the loops.  Any data race report fails the test."""
    import concurrent.futures as cf

    from live_upstream import free_port_block
    from quorum_amd.ops import build
    from quorum_amd.runtime.native_server import native_config

    tsan = build.build_tsan()
    live = LiveUpstream()
    stream = sse_stream(["Hel", "lo <think>x</think> wor", "ld"])
    ports = [live.serve("a", ("stream", 200, stream)), live.serve("b", ("stream", 200, sse_stream(["x", "y"])))]
    block = {"separator": "\n--\n", "hide_intermediate_think": True, "hide_final_think": True,
             "thinking_tags": ["think"], "skip_final_aggregation": False}
    cfg = cfg_parallel(2, block=block)
    for b, p in zip(cfg["primary_backends"], ports):
        b["url"] = f"http://127.0.0.1:{p}/v1"
    cfg.setdefault("runtime", {})["placement"] = "spread"
    port = free_port()
    xenv = {"QMX_XCHG": "tcpbulk", "QMX_XCHG_PORT": str(free_port_block(2)), "QMX_XCHG_EAGER_BYTES": "0",
            "QMX_XCHG_TIMEOUT": "2", "QMX_XCHG_ROUND_US": "100"}
    old = {k: os.environ.get(k) for k in xenv}
    os.environ.update(xenv)
    try:
        d = native_config(cfg, "127.0.0.1", port, "cpu", 0, 4)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    d.update(env_api_key="", api_key_from_env=False, tick_mode="loops")
    path = tmp_path / "tsan_spread.json"
    path.write_text(json.dumps(d))
    env = dict(os.environ, **xenv, QMX_SPREAD_SELF="1", QMX_XCHG_FAULT_STALL_ROUND="2",
               TSAN_OPTIONS="halt_on_error=0:second_deadlock_stack=1:report_signal_unsafe=0")
    srv = subprocess.Popen([str(tsan), str(path)], stderr=subprocess.PIPE, env=env)
    try:
        t0 = time.time()
        while time.time() - t0 < 60:
            try:
                m = httpx.get(f"http://127.0.0.1:{port}/metrics", timeout=1).text
                if "qmx_exchange_rccl_active 1.000000" in m:
                    break
            except httpx.HTTPError:
                pass
            time.sleep(0.1)
        req = {"messages": [{"role": "user", "content": "q"}], "stream": True}

        def client(i):
            if i % 3 == 0:  # a client that leaves mid-response (its final may be in a round)
                s = socket.create_connection(("127.0.0.1", port))
                body = json.dumps(req).encode()
                s.sendall(b"POST /chat/completions HTTP/1.1\r\nhost: x\r\nauthorization: Bearer k\r\n"
                          b"content-type: application/json\r\ncontent-length: %d\r\n\r\n%s" % (len(body), body))
                s.recv(256)
                s.close()
                return True
            with httpx.Client(base_url=f"http://127.0.0.1:{port}") as c:
                for _ in range(6):
                    r = c.post("/chat/completions", json=req, headers={"Authorization": "Bearer k"}, timeout=90)
                    assert r.status_code == 200 and r.text.rstrip().endswith("data: [DONE]")
            return True

        with cf.ThreadPoolExecutor(6) as ex:
            assert all(ex.map(client, range(12)))
        m = httpx.get(f"http://127.0.0.1:{port}/metrics").text

        def metric(k):
            return float([ln for ln in m.splitlines() if ln.startswith(k + " ")][0].split()[1])
        assert metric("qmx_remote_streams_total") > 0
        assert metric("qmx_exchange_rounds_total") > 0           # finals moved in rounds ...
        assert metric("qmx_exchange_mesh_finals_total") > 0      # ... and the stalled round's by the mesh
    finally:
        srv.send_signal(signal.SIGINT)
        try:
            _, err = srv.communicate(timeout=60)
        except subprocess.TimeoutExpired:
            srv.kill()
            _, err = srv.communicate()
        live.close()
    err = err.decode(errors="replace")
    assert "ThreadSanitizer" not in err, err[-6000:]
    assert srv.returncode == 0, err[-3000:]
