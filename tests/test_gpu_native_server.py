"""GPU: the native data plane with the CDNA4 HIP engine vs the FastAPI conformance app."""
import pytest

import test_native_server as T

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("tick_mode", ["loops", "lanes"])
@pytest.mark.parametrize("name", sorted(T.SCENARIOS))
def test_native_hip_matches_python(name, tick_mode, monkeypatch):
    """HIP engine + verify mode: every stream and final is also checked against the
    shadow C++ CPU oracle inside the server (byte-identical or counted as mismatch).
    loops: io loops post into the multi-door grid (the default); lanes: the shared engine."""
    from quorum_amd.ops import native

    ext = native.require()
    before = ext.server_counters()["verify_mismatches"]
    monkeypatch.setattr(T, "ENGINE", "hip")
    monkeypatch.setattr(T, "VERIFY", True)
    T.test_native_matches_python(name, tick_mode)
    assert ext.server_counters()["verify_mismatches"] == before


@pytest.mark.parametrize("name", sorted(T.DOC_SCENARIOS))
def test_native_hip_documented_semantics(name, monkeypatch):
    """``semantics: documented`` on the HIP engine (the strip before the aggregator runs in
    the fused finalize's texts kind; the slot's content size names its source), verify mode
    on: python app == native server, and the expected prompt and answer."""
    from quorum_amd.ops import native

    ext = native.require()
    before = ext.server_counters()["verify_mismatches"]
    monkeypatch.setattr(T, "ENGINE", "hip")
    monkeypatch.setattr(T, "VERIFY", True)
    T.test_native_matches_python_documented(name)
    T.test_documented_semantics_expectations(name)
    assert ext.server_counters()["verify_mismatches"] == before


def test_native_hip_keepalive(monkeypatch):
    import live_upstream as L
    orig = L.native_server

    def hip_server(cfg, engine="cpu", threads=1, env_key=""):
        return orig(cfg, engine="hip", threads=threads, env_key=env_key)

    monkeypatch.setattr(T, "native_server", hip_server)
    T.test_native_keepalive_many_requests()


@pytest.mark.parametrize("seed", range(40))
def test_native_hip_random_sessions(seed, monkeypatch):
    """Random sessions (test_native_random_differential) through the HIP engine + verify."""
    from quorum_amd.ops import native

    import test_native_random_differential as R

    ext = native.require()
    before = ext.server_counters()["verify_mismatches"]
    monkeypatch.setattr(T, "ENGINE", "hip")
    monkeypatch.setattr(T, "VERIFY", True)
    R.run_random_session(seed, "loops" if seed % 2 else "lanes")
    assert ext.server_counters()["verify_mismatches"] == before


@pytest.mark.parametrize("name", sorted(T.SCENARIOS))
def test_native_hip_light_host_matches_python(name, monkeypatch):
    """Latency mode (QMX_LIGHT_HOST=4): the scenarios' sessions come one at a time, so their
    streams open on the HIP engine's host path — the C++ engine inline in the loop's tick —
    and must still equal the FastAPI app byte for byte (verify mode on)."""
    from quorum_amd.ops import native

    ext = native.require()
    before = ext.server_counters()["verify_mismatches"]
    monkeypatch.setenv("QMX_LIGHT_HOST", "4")
    monkeypatch.setattr(T, "ENGINE", "hip")
    monkeypatch.setattr(T, "VERIFY", True)
    T.test_native_matches_python(name, "loops")
    assert ext.server_counters()["verify_mismatches"] == before


@pytest.mark.parametrize("conns,light,port", [(2, "0", 23560), (2, "4", 23570), (64, "4", 23580)])
def test_gpu_bench_light_host(tmp_path, conns, light, port):
    """The latency mode under the bench's validation: at 2 connections with QMX_LIGHT_HOST=4
    most streams open on the host path (none without it); at the headline's 64, host-path and
    GPU streams mix on the same loops (a session opened between two ticks goes to the host) —
    every response still valid.  The mode is opt-in: it costs the headline ~5% (r6 lowload)."""
    import json
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, QMX_BENCH_ENGINE="hip", QMX_LIGHT_HOST=light)
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--steps", "3", "--warmup", "1",
                        "--batch", "4096", "--conns", str(conns), "--port", str(port), "--ceiling", "0"],
                       cwd=str(tmp_path), env=env, capture_output=True, text=True, timeout=180)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert lines, r.stderr[-3000:]
    res = json.loads(lines[-1])
    assert r.returncode == 0 and res["valid"] and res["invalid"] == 0, (res.get("invalid"), r.stderr[-2000:])
    bd = res["breakdown_one_rank"]
    streams = 2 * (3 + 1) * 4096  # two backends per request, warmup included
    if light == "0":
        assert bd["light_host_opens"] == 0 and bd["kernel_launches"] > 0, bd
    elif conns == 2:
        # (the engines' counters are snapshots up to 100 ms old — a fifth of this short run —
        # and a finished session can outlive its response by its upstreams' last bytes)
        # (r6: 72-86% of the streams at 1-8 connections on full-length runs)
        assert bd["light_host_opens"] >= streams * 0.25, (bd["light_host_opens"], streams)
    else:  # loops with ticks in flight: host-path and GPU streams mixed on the same loops, all valid
        assert bd["kernel_launches"] > 0, bd


@pytest.mark.parametrize("knob,port", [("", 23400), ("QMX_EAGER_POST=1", 23500)])
def test_gpu_bench_headline_valid(tmp_path, knob, port):
    """The headline bench on the HIP engine (shared engine, pipelined tick lanes, persistent
    grids, result views) under full closed-loop load: every response is validated byte for
    byte by the load generator, so a lane that reuses an output arena too early, or any other
    cross-tick corruption, fails here.  QMX_EAGER_POST=1: an io loop posts upstream bytes to a
    free door in the middle of its event batch (an A/B knob, off by default) — same bytes."""
    import json
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, QMX_BENCH_ENGINE="hip")
    if knob:
        k, v = knob.split("=")
        env[k] = v
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--steps", "4", "--warmup", "1",
                        "--batch", "8192", "--port", str(port)],
                       cwd=str(tmp_path), env=env, capture_output=True, text=True, timeout=180)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert lines, r.stderr[-3000:]
    res = json.loads(lines[-1])
    assert r.returncode == 0 and res["valid"] and res["invalid"] == 0, (res.get("invalid"), r.stderr[-2000:])
    assert res["validated"] == 4 * 8192 and res["breakdown_one_rank"]["kernel_launches"] > 0


def test_gpu_self_spread_rccl_rounds_under_load(tmp_path):
    """The world > 1 data path on one GPU, under headline load (round-5 verdict, next #1).
    The full native server — 8 io loops on the loop-tick grid, GPU_MAX_HW_QUEUES=4 as on the
    box — with QMX_SPREAD_SELF: backend 2 of every session runs through the rank's own
    exchange (mesh frames to itself, a worker session, its deltas back), and every final text
    goes HBM → HBM in an RCCL round to itself (exchange_eager_bytes 0), is copied out by the
    exchange's bulk thread (QMX_REMOTE_HBM=0: the world > 1 default, where a peer GPU wrote the
    bytes) and finalized in the owner's fused GPU items.  Every response is validated by the
    load generator; every final went through a round (no mesh fallback); no io loop copied a
    text itself or stalled for more than 5 ms; the grid's queue is its own."""
    import json
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, QMX_BENCH_ENGINE="hip", QMX_SPREAD_SELF="1", QMX_REMOTE_HBM="0", GPU_MAX_HW_QUEUES="4",
               QMX_LOOP_STALL_LOG="1")  # a pass over 5 ms prints its phase split (in the failure message)
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--steps", "4", "--warmup", "1",
                        "--batch", "8192", "--port", "23600", "--threads", "8", "--placement", "spread",
                        "--eager-bytes", "0", "--skip-final", "0", "--ceiling", "0"],
                       cwd=str(tmp_path), env=env, capture_output=True, text=True, timeout=240)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert lines, r.stderr[-3000:]
    res = json.loads(lines[-1])
    (tmp_path / "self_spread.json").write_text(lines[-1])
    assert r.returncode == 0 and res["valid"] and res["invalid"] == 0, (res.get("invalid"), r.stderr[-2000:])
    bd = res["breakdown_one_rank"]
    x = bd["exchange"]
    assert x and x["remote_streams"] >= 4 * 8192, json.dumps(x)
    assert x["bulk_rounds"] > 0 and x["mesh_finals"] == 0 and x["eager_finals"] == 0, json.dumps(x)
    assert x["delta_mismatch"] == 0 and x["worker_nodata"] == 0, json.dumps(x)
    assert x["host_copied_by_exchange"] > 0 and x["copied_inline"] == 0, json.dumps(x)
    # every RCCL text reached its engine as a host copy, none read from HBM directly (the
    # engines' counters are snapshots up to 100 ms old — a third of this short run — so only
    # their sign is compared with the exchange's live count)
    assert x["remote_texts_hbm"] == 0 and x["remote_texts_copied"] > 0, json.dumps(x)
    assert bd["finalize_host"] == 0 and bd["escalations"] == 0, bd
    # no io loop blocked: a synchronous device copy or lock on a loop stalls it again and again
    # (3-8 passes over 5 ms per run before the round-6 fixes).  One isolated long pass is
    # allowed: a runnable loop thread can be preempted for a few ms on the CCD it shares with
    # the mocks and the load generator (r6: one 19.5 ms pass in ~10 runs, 0 in the others)
    stalls = [ln for ln in r.stderr.splitlines() if "stalled pass" in ln or "ms pass (" in ln]
    assert bd["loop_passes_over_5ms"] <= 1 and bd["loop_pass_max_ms"] < 50, (
        bd["loop_passes_over_5ms"], bd["loop_pass_max_ms"], stalls[:6])
    q = bd["hip_streams"]
    assert q and q["grid_queue_exclusive"] and q["grid_queue_ok"] and q["hw_queues_per_priority"] == 4, q


def _metric(text, name):
    for ln in text.splitlines():
        if ln.startswith(name + " "):
            return float(ln.split()[1])
    return None


@pytest.mark.parametrize("sharers,want_grid", [("1", True), ("16", True), ("64", False)])
def test_native_hip_grid_sizing(sharers, want_grid, monkeypatch):
    """The loop-tick grid fits within half the CUs split between the processes sharing the
    GPU (QMX_GPU_SHARERS, set by rank rehearsals): 16 sharers shrink it to 2 workgroups per
    door; 64 leave no room and the server falls back to tick lanes — it serves either way."""
    import time

    import httpx

    from quorum_amd.ops import native

    ext = native.require()
    monkeypatch.setenv("QMX_GPU_SHARERS", sharers)
    live = T.LiveUpstream()
    p1 = live.serve("b1", ("stream", 200, T.THINK))
    p2 = live.serve("b2", ("stream", 200, T.sse_stream(["Wor", "ld <think>x</think>", " é😀"])))
    cfg = T.cfg_parallel(2, block=dict(T.CONCAT))
    cfg["primary_backends"][0]["url"] = f"http://127.0.0.1:{p1}/v1"
    cfg["primary_backends"][1]["url"] = f"http://127.0.0.1:{p2}/v1"
    before = ext.server_counters()["verify_mismatches"]
    try:
        with T.native_server(cfg, engine="hip", threads=2, verify=True) as port:
            for _ in range(20):
                r = httpx.post(f"http://127.0.0.1:{port}/chat/completions", json={"messages": T.MSG, "stream": True},
                               headers=T.AUTH, timeout=30)
                assert r.status_code == 200 and r.text.rstrip().endswith("data: [DONE]")
            time.sleep(0.3)  # an io-loop sweep snapshots the engines' counters
            m = httpx.get(f"http://127.0.0.1:{port}/metrics").text
    finally:
        live.close()
    assert ext.server_counters()["verify_mismatches"] == before
    doors, wpd = _metric(m, "qmx_kernel_grid_doors"), _metric(m, "qmx_kernel_grid_wg_per_door")
    if want_grid:
        assert doors == 4 and wpd == (2 if sharers == "16" else 8), (doors, wpd)
    else:
        assert doors is None and (_metric(m, "qmx_kernel_launches") or 0) > 0


@pytest.mark.parametrize("xchg,eager", [("tcp", None), ("tcpbulk", 0)])
@pytest.mark.parametrize("name", ["concat_think", "concat_null_abort", "aggregate_4", "concat_4_one_fails"])
def test_hip_spread_cluster_matches_local(name, xchg, eager, monkeypatch):
    """Spread placement on the HIP engine: 2 in-process ranks sharing GPU 0 (loop ticks, a
    grid each), session messages on per-loop links, remote finals eager over the link or
    through tcpbulk rounds.  Every response equals the single-rank HIP server's, and every
    rank finalized its merged sessions on the GPU: fin_host stays 0 while remote texts were
    staged into finalize items."""
    import httpx

    import test_native_spread as S
    from live_upstream import native_server

    monkeypatch.setenv("QMX_GPU_SHARERS", "2")  # two grids on one GPU (set before any server starts)
    n, block, strategy, behs = S.SPREAD_CASES[name]
    live, ports = S._live({f"b{i + 1}": b for i, b in enumerate(behs)})
    try:
        cfg = S._cfg(n, block, strategy, [f"http://127.0.0.1:{ports[f'b{i + 1}']}/v1" for i in range(n)])
        req = {"messages": S.MSG, "stream": True}
        with native_server(cfg, engine="hip") as p:
            ref = httpx.post(f"http://127.0.0.1:{p}/chat/completions", json=req, headers=S.AUTH, timeout=30)
        with S.native_cluster(cfg, 2, xchg=xchg, eager=eager, engine="hip") as cports:
            m0 = [httpx.get(f"http://127.0.0.1:{p}/metrics").text for p in cports]
            for owner in range(2):
                for _ in range(3):
                    r = httpx.post(f"http://127.0.0.1:{cports[owner]}/chat/completions", json=req, headers=S.AUTH,
                                   timeout=30)
                    assert r.status_code == ref.status_code
                    assert S._split(S._events(r.text)) == S._split(S._events(ref.text)), (name, owner)
            ms = [httpx.get(f"http://127.0.0.1:{p}/metrics").text for p in cports]

        def delta(k):
            return sum((_metric(ms[r], k) or 0.0) - (_metric(m0[r], k) or 0.0) for r in range(2))

        assert delta("qmx_kernel_fin_host") == 0
        assert delta("qmx_spread_delta_mismatch_total") == 0
        if name in ("concat_think", "aggregate_4"):  # finals with text from the remote rank
            assert (delta("qmx_kernel_remote_texts_staged") + delta("qmx_kernel_remote_texts_hbm")
                    + delta("qmx_kernel_remote_texts_copied")) > 0
            assert delta("qmx_kernel_fin_items") > 0
    finally:
        live.close()


@pytest.mark.parametrize("light", ["", "0"])
def test_gpu_serve_latency_mode(tmp_path, light):
    """`serve --impl native --engine hip` — the production launcher, with its default latency
    mode (QMX_LIGHT_HOST=2 for its workers) or with it off: one client's sessions, one at a
    time, give the same finals either way (the host path is the byte-identical C++ engine),
    and /metrics says which path took them."""
    import os
    import signal
    import subprocess
    import sys
    import time

    import json

    import httpx
    import yaml

    from conftest import cfg_parallel, sse_stream
    from live_upstream import LiveUpstream, free_port

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    live = LiveUpstream()
    pa = live.serve("a", ("stream", 200, sse_stream(["<think>x</think>", "AAA ", "aaa"])))
    pb = live.serve("b", ("stream", 200, sse_stream(["BBB ", "<think>y</think>", "bbb"])))
    cfg = cfg_parallel(2, block={"separator": "\n--\n", "hide_intermediate_think": True, "hide_final_think": False,
                                 "thinking_tags": ["think"], "skip_final_aggregation": False})
    cfg["primary_backends"][0]["url"] = f"http://127.0.0.1:{pa}/v1"
    cfg["primary_backends"][1]["url"] = f"http://127.0.0.1:{pb}/v1"
    path = str(tmp_path / "config.yaml")
    with open(path, "w") as f:
        yaml.safe_dump(cfg, f)
    port = free_port()
    env = dict(os.environ, PYTHONPATH=root)
    env.pop("QMX_LIGHT_HOST", None)
    if light:
        env["QMX_LIGHT_HOST"] = light
    sup = subprocess.Popen([sys.executable, "-m", "quorum_amd.serve", "--impl", "native", "--engine", "hip",
                            "--config", path, "--port", str(port), "--threads", "2"], cwd=root, env=env,
                           start_new_session=True)
    try:
        base = f"http://127.0.0.1:{port}"
        t0 = time.time()
        while True:
            try:
                if httpx.get(base + "/health", timeout=2).status_code == 200:
                    break
            except httpx.HTTPError:
                pass
            assert time.time() - t0 < 120 and sup.poll() is None, "serve did not come up"
            time.sleep(0.2)
        finals = set()
        with httpx.Client(timeout=30) as c:
            for _ in range(12):
                r = c.post(base + "/chat/completions", json={"messages": [{"role": "user", "content": "hi"}],
                                                             "stream": True}, headers={"Authorization": "Bearer k"})
                assert r.status_code == 200 and r.text.rstrip().endswith("data: [DONE]")
                for seg in r.text.split("\n\n"):
                    if '"chatcmpl-parallel-final"' in seg:
                        finals.add(json.loads(seg[6:])["choices"][0]["delta"]["content"])
        # the C++ CPU engine's final for the same streams (the reference semantics' oracle)
        from live_upstream import native_server as cpu_server
        with cpu_server(cfg, engine="cpu") as cport:
            rt = httpx.post(f"http://127.0.0.1:{cport}/chat/completions", headers={"Authorization": "Bearer k"},
                            json={"messages": [{"role": "user", "content": "hi"}], "stream": True}, timeout=30).text
        want = {json.loads(seg[6:])["choices"][0]["delta"]["content"] for seg in rt.split("\n\n")
                if '"chatcmpl-parallel-final"' in seg}
        assert len(want) == 1 and "AAA aaa" in next(iter(want)) and "think" not in next(iter(want)), want
        assert finals == want, (finals, want)
        time.sleep(0.3)  # the engines' counters are snapshots up to 100 ms old
        m = httpx.get(base + "/metrics", timeout=5).text
        opens = sum(float(ln.split()[-1]) for ln in m.splitlines() if ln.startswith("qmx_kernel_light_host_opens"))
        if light == "0":
            assert opens == 0, opens
        else:
            assert opens > 0, opens
    finally:
        os.killpg(sup.pid, signal.SIGTERM)
        try:
            sup.wait(timeout=20)
        except subprocess.TimeoutExpired:
            os.killpg(sup.pid, signal.SIGKILL)
        live.close()
