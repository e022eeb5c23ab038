"""Spread (EP-style) backend placement across ranks, CPU rehearsal with the TCP exchange.

Two (or three) native server "ranks" run in this process, each with its own port, engine
and keep-alive pools; with ``placement: spread`` backend i of a session owned by rank r
runs on rank (r + i) % world and its SSE deltas + final text come back through the
lock-step all-gather exchange (qmx_exchange.cpp).  Results must match the single-rank
(local placement) server exactly — per-backend event streams, final event, aggregator
prompt — whichever rank owns the session.  On MI355X the same code path uses RCCL
(``exchange: rccl``) instead of the TCP hub.
"""
import contextlib
import copy
import json
import os
import threading
import time

import httpx
import pytest

from quorum_amd.ops import native

from conftest import cfg_parallel, completion, sse_chunk, sse_stream
from live_upstream import LiveUpstream, free_port, free_port_block, native_server

pytestmark = pytest.mark.skipif(not native.available(), reason="native extension not built")

AUTH = {"Authorization": "Bearer test-key"}
MSG = [{"role": "user", "content": "What is 2+2?"}]
CONCAT = {"separator": "\n-------------\n", "hide_intermediate_think": True, "hide_final_think": True,
          "thinking_tags": ["think", "reason", "reasoning", "thought"], "skip_final_aggregation": False}
AGG = {"aggregator_backend": "LLM4", "intermediate_separator": "\n\n---\n\n", "include_source_names": True,
       "source_label_format": "Response from {backend_name}:\n", "prompt_template": "R:\n{responses}\nEnd.",
       "include_original_query": True}
THINK = [sse_chunk({"role": "assistant"}), sse_chunk({"content": "<think>"}), sse_chunk({"content": "hmm"}),
         sse_chunk({"content": "</think>"}), sse_chunk({"content": "The answer "}), sse_chunk({"content": "is 4."}),
         sse_chunk({}, finish="stop"), b"data: [DONE]\n\n"]


@contextlib.contextmanager
def native_cluster(cfg, world: int, placement: str = "spread", xchg: str = "tcp", eager=None, tick_mode=None,
                   links=None, engine: str = "cpu", run_env=None):
    """`world` native ranks in-process (threads), TCP exchange on a free port block.
    ``xchg="tcpbulk"``: final texts move in rank-0-numbered bulk rounds (the RCCL round
    protocol with a socket executor) instead of riding the mesh.  ``eager``: the largest final
    text that rides the mesh behind its deltas instead (None: the default; 0: none).
    ``tick_mode="loops"``: every rank's io loops drive their own engine asynchronously (the
    loop-tick protocol, AsyncCpuEngine on the CPU) while remote streams come and go.
    ``run_env``: environment set while the servers start (they snapshot it then) and restored
    after they stopped."""
    from quorum_amd.runtime.native_server import native_config

    ext = native.require()
    cfg = copy.deepcopy(cfg)
    cfg.setdefault("runtime", {})["placement"] = placement
    ports = [free_port() for _ in range(world)]
    xport = free_port_block(2 * world)  # the mesh: rank r listens on xport + r (tcpbulk: + world + r)
    threads = []
    # every rank's config first, then the servers: the environment is only changed while no
    # server thread runs (a running server reads it — getenv racing setenv can crash)
    cfgs = []
    for r in range(world):
        env = {"QMX_RANK": str(r), "QMX_WORLD": str(world), "QMX_XCHG": xchg, "QMX_XCHG_PORT": str(xport),
               "QMX_XCHG_ROUND_US": "100"}
        if eager is not None:
            env["QMX_XCHG_EAGER_BYTES"] = str(eager)
        env.update(run_env or {})
        old = {k: os.environ.get(k) for k in env}
        os.environ.update(env)
        try:
            d = native_config(cfg, "127.0.0.1", ports[r], engine, 0, 1)
        finally:
            for k, v in old.items():
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v
        d["install_signals"] = False
        if links is not None:  # per-loop links on / off (off: every message through the mesh thread)
            d["xchg_links"] = 1 if links else 0
        if tick_mode is not None:
            d["tick_mode"] = tick_mode
        cfgs.append(d)
    saved = {k: os.environ.get(k) for k in (run_env or {})}
    os.environ.update(run_env or {})
    for d in cfgs:
        th = threading.Thread(target=ext.run_server, args=(d,), daemon=True)
        th.start()
        threads.append(th)
    for p in ports:
        t0 = time.time()
        while time.time() - t0 < 20:
            try:
                if httpx.get(f"http://127.0.0.1:{p}/health", timeout=1).status_code == 200:
                    break
            except httpx.HTTPError:
                time.sleep(0.02)
    if placement == "spread":  # sessions spread only once every rank's mesh is complete
        for p in ports:
            t0 = time.time()
            while time.time() - t0 < 20:
                m = httpx.get(f"http://127.0.0.1:{p}/metrics").text
                if (f"qmx_exchange_peers_up {float(world):f}" in m and "qmx_exchange_healthy 1.000000" in m
                        and (xchg == "tcp" or "qmx_exchange_rccl_active 1.000000" in m)):
                    break
                time.sleep(0.02)
    try:
        yield ports
    finally:
        ext.stop_server()
        for th in threads:
            th.join(timeout=15)
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def _metric(text, name):
    return float([ln for ln in text.splitlines() if ln.startswith(name + " ")][0].split()[1])


def _events(text):
    out = []
    for seg in text.split("\n\n"):
        if not seg.strip():
            continue
        p = seg[6:]
        if p == "[DONE]":
            out.append(p)
            continue
        ev = json.loads(p)
        ev["created"] = 0
        out.append(ev)
    return out


def _split(evs):
    per, rest = {}, []
    for e in evs:
        if e != "[DONE]" and e["id"].startswith("chatcmpl-parallel-") and e["id"][-1].isdigit():
            per.setdefault(e["id"], []).append(e)
        else:
            rest.append(e)
    return per, rest


def _live(ups):
    live = LiveUpstream()
    return live, {h: live.serve(h, b) for h, b in ups.items()}


def _cfg(n, block, strategy="concatenate", urls=None):
    cfg = cfg_parallel(n, strategy=strategy, block=block)
    for i, b in enumerate(cfg["primary_backends"]):
        b["url"] = urls[i]
    return cfg


SPREAD_CASES = {
    "concat_think": (2, CONCAT, "concatenate",
                     [("stream", 200, THINK), ("stream", 200, sse_stream(["Wor", "ld <think>x</think>"]))]),
    "concat_4_one_fails": (4, CONCAT, "concatenate",
                           [("stream", 200, sse_stream(["a"])), ("json", 503, {"error": {"message": "down"}}),
                            ("stream", 200, THINK), ("refuse",)]),
    "concat_all_fail": (2, CONCAT, "concatenate", [("json", 500, {"error": {"message": "x"}}), ("refuse",)]),
    "concat_null_abort": (3, CONCAT, "concatenate",
                          [("stream", 200, [sse_chunk({"content": "alpha "}), sse_chunk({"content": None}),
                                            sse_chunk({"content": "beta"}), b"data: [DONE]\n\n"]),
                           ("stream", 200, sse_stream(["B"])), ("stream", 200, sse_stream(["C é😀"]))]),
    "skip_final": (3, dict(CONCAT, skip_final_aggregation=True), "concatenate",
                   [("stream", 200, sse_stream(["x"])), ("stream", 200, sse_stream(["y"])),
                    ("stream", 200, sse_stream(["z"]))]),
    "aggregate_4": (4, AGG, "aggregate",
                    [("stream", 200, sse_stream(["one"])), ("stream", 200, THINK),
                     ("stream", 200, sse_stream(["three"])),
                     lambda body: (("stream", 200, sse_stream(["four"])) if body.get("stream")
                                   else ("json", 200, completion("SYNTH")))]),
}


@pytest.mark.parametrize("world,xchg,eager,links", [(2, "tcp", None, True), (3, "tcp", 0, True),
                                                     (2, "tcpbulk", 0, True), (4, "tcpbulk", 0, True),
                                                     (3, "tcpbulk", None, True), (2, "tcp", None, False),
                                                     (3, "tcpbulk", 0, False)])
@pytest.mark.parametrize("name", sorted(SPREAD_CASES))
def test_spread_matches_local(name, world, xchg, eager, links):
    """Spread responses equal single-rank ones, with every final-text path: eager (short texts
    ride the mesh behind their deltas: the default), mesh bulk (tcp, eager off) and bulk
    rounds (tcpbulk, eager off) — session messages over the io loops' own links (default) or
    through the mesh thread (links off)."""
    n, block, strategy, behs = SPREAD_CASES[name]
    live, ports = _live({f"b{i + 1}": b for i, b in enumerate(behs)})
    try:
        cfg = _cfg(n, block, strategy, [f"http://127.0.0.1:{ports[f'b{i + 1}']}/v1" for i in range(n)])
        req = {"messages": MSG, "stream": True}
        with native_server(cfg) as p:
            ref = httpx.post(f"http://127.0.0.1:{p}/chat/completions", json=req, headers=AUTH, timeout=30)
        ref_calls = sorted(json.dumps(c["body"], sort_keys=True) for c in live.calls)
        live.calls.clear()
        with native_cluster(cfg, world, xchg=xchg, eager=eager, links=links) as cports:
            # (in-process ranks share one process's counters, across tests too: deltas)
            m0 = [httpx.get(f"http://127.0.0.1:{p}/metrics").text for p in cports]
            for owner in range(world):  # every rank as session owner
                r = httpx.post(f"http://127.0.0.1:{cports[owner]}/chat/completions", json=req, headers=AUTH,
                               timeout=30)
                assert r.status_code == ref.status_code
                assert _split(_events(r.text)) == _split(_events(ref.text)), (name, owner)
            ms = [httpx.get(f"http://127.0.0.1:{p}/metrics").text for p in cports]
            m = ms[0]
        # each owner's run sent exactly the single-rank upstream requests
        calls = sorted(json.dumps(c["body"], sort_keys=True) for c in live.calls)
        assert calls == sorted(ref_calls * world)
        assert "qmx_exchange_rounds_total" in m
        remote = float([ln for ln in m.splitlines() if ln.startswith("qmx_remote_streams_total")][0].split()[1])
        assert remote >= 1, m
        assert _metric(m, "qmx_spread_delta_mismatch_total") == 0
        link_msgs = _metric(ms[0], "qmx_exchange_link_messages_total") - _metric(m0[0], "qmx_exchange_link_messages_total")
        assert (link_msgs > 0) == links, link_msgs

        def total(k):
            # exchange counters are per rank (summed); server counters are per process, which
            # the in-process ranks share (rank 0's delta)
            ranks = range(world) if k.startswith("qmx_exchange_") else [0]
            return sum(_metric(ms[r], k) - _metric(m0[r], k) for r in ranks)
        texts = total("qmx_spread_remote_ends_total{how=\"text\"}")
        if eager is None:  # short texts: every one eager, nothing through a round or mesh bulk
            assert total("qmx_spread_eager_finals_total") == texts
            assert total("qmx_exchange_mesh_finals_total") == 0 and total("qmx_exchange_rounds_total") == 0
        else:
            assert total("qmx_spread_eager_finals_total") == 0
            if xchg == "tcpbulk":  # final texts moved by bulk rounds, none over the mesh
                assert total("qmx_exchange_mesh_finals_total") == 0, m
                assert (total("qmx_exchange_rounds_total") > 0) == (texts > 0)
            else:
                assert total("qmx_exchange_mesh_finals_total") == texts
    finally:
        live.close()


@pytest.mark.parametrize("xchg,eager", [("tcp", None), ("tcp", 0), ("tcpbulk", 0)])
@pytest.mark.parametrize("name", ["concat_think", "aggregate_4", "concat_null_abort"])
def test_self_spread_matches_local(name, xchg, eager):
    """QMX_SPREAD_SELF at world 1: every odd backend runs through the rank's own exchange (mesh
    frames to itself, a worker session on the same loop, final texts eager / over the mesh /
    in bulk rounds to itself) — the multi-rank path on one rank, as the GPU test runs it with
    RCCL.  Responses equal the local server's, and the odd streams really went remote."""
    n, block, strategy, behs = SPREAD_CASES[name]
    live, ports = _live({f"b{i + 1}": b for i, b in enumerate(behs)})
    try:
        cfg = _cfg(n, block, strategy, [f"http://127.0.0.1:{ports[f'b{i + 1}']}/v1" for i in range(n)])
        req = {"messages": MSG, "stream": True}
        with native_server(cfg) as p:
            ref = httpx.post(f"http://127.0.0.1:{p}/chat/completions", json=req, headers=AUTH, timeout=30)
        with native_cluster(cfg, 1, xchg=xchg, eager=eager, run_env={"QMX_SPREAD_SELF": "1"}) as cports:
            m0 = httpx.get(f"http://127.0.0.1:{cports[0]}/metrics").text
            for _ in range(3):
                r = httpx.post(f"http://127.0.0.1:{cports[0]}/chat/completions", json=req, headers=AUTH, timeout=30)
                assert r.status_code == ref.status_code
                assert _split(_events(r.text)) == _split(_events(ref.text)), name
            m = httpx.get(f"http://127.0.0.1:{cports[0]}/metrics").text

        def d(k):
            return _metric(m, k) - _metric(m0, k)
        assert d("qmx_remote_streams_total") == 3 * (n // 2), m
        assert _metric(m, "qmx_spread_delta_mismatch_total") == 0
        texts = d("qmx_spread_remote_ends_total{how=\"text\"}")
        if xchg == "tcpbulk":
            assert d("qmx_exchange_rounds_total") > 0 or texts == 0
            assert d("qmx_exchange_mesh_finals_total") == 0
    finally:
        live.close()


def test_session_end_during_stalled_round_does_not_block_its_loop():
    """Advisor finding (round 5): forget_bulk() made the io loop wait, up to twice the round
    timeout, for a round still receiving into a leaving session's shadow slot — every other
    connection on that loop froze meanwhile.  Now the release is deferred: the slot stays
    pinned, the loop goes on, and the exchange hands the slot back (X_RELEASE) when the round
    is over.  One io loop, self spread (backend 2 of every session through the rank's own
    exchange), bulk round 1 stalled for its 3 s timeout (QMX_XCHG_FAULT_STALL_ROUND=1): client
    A leaves while its final text is in that round; client B, on the same loop, must get its
    first delta at once, and every slot must come back."""
    import socket

    behs = [("stream", 200, THINK), ("stream", 200, sse_stream(["x", "y", "z"]))]
    live, ports = _live({"b1": behs[0], "b2": behs[1]})
    try:
        cfg = _cfg(2, dict(CONCAT, skip_final_aggregation=False), "concatenate",
                   [f"http://127.0.0.1:{ports['b1']}/v1", f"http://127.0.0.1:{ports['b2']}/v1"])
        env = {"QMX_SPREAD_SELF": "1", "QMX_XCHG_FAULT_STALL_ROUND": "1", "QMX_XCHG_TIMEOUT": "3"}
        with native_cluster(cfg, 1, xchg="tcpbulk", eager=0, run_env=env) as cports:
            base = f"http://127.0.0.1:{cports[0]}"
            m0 = httpx.get(base + "/metrics").text
            body = json.dumps({"messages": MSG, "stream": True}).encode()
            a = socket.create_connection(("127.0.0.1", cports[0]))
            a.sendall(b"POST /chat/completions HTTP/1.1\r\nHost: x\r\nAuthorization: Bearer test-key\r\n"
                      b"Content-Type: application/json\r\nContent-Length: " + str(len(body)).encode() +
                      b"\r\n\r\n" + body)
            got = b""
            t0 = time.time()
            while b'"content": "x"' not in got and time.time() - t0 < 5:  # backend 2's deltas came back
                got += a.recv(65536)
            time.sleep(0.3)  # its final text is announced and sits in the stalled round 1
            a.close()
            time.sleep(0.2)
            t1 = time.time()
            assert httpx.get(base + "/health", timeout=2).status_code == 200
            first = None
            with httpx.Client(base_url=base) as c:
                with c.stream("POST", "/chat/completions", json={"messages": MSG, "stream": True}, headers=AUTH,
                              timeout=30) as r:
                    for chunk in r.iter_text():
                        if first is None and '"content"' in chunk:
                            first = time.time() - t1
            assert first is not None and first < 1.0, first  # the loop was not held by A's round
            t2 = time.time()
            while time.time() - t2 < 10:
                m = httpx.get(base + "/metrics").text
                if _metric(m, "qmx_engine_free") >= _metric(m0, "qmx_engine_free"):
                    break
                time.sleep(0.1)
        assert _metric(m, "qmx_spread_release_deferred_total") - _metric(m0, "qmx_spread_release_deferred_total") >= 1, m
        assert _metric(m, "qmx_exchange_deferred_releases_total") >= 1
        assert _metric(m, "qmx_engine_free") >= _metric(m0, "qmx_engine_free"), "a shadow slot was never released"
    finally:
        live.close()


@pytest.mark.parametrize("tick_mode", [None, "loops"])
def test_spread_many_concurrent_sessions(tick_mode):
    """Concurrent sessions on both ranks; every response complete and correct (also with
    every rank's io loops on the loop-tick protocol)."""
    behs = [("stream", 200, THINK), ("stream", 200, sse_stream(["x", "y", "z"]))]
    live, ports = _live({"b1": behs[0], "b2": behs[1]})
    try:
        cfg = _cfg(2, dict(CONCAT, skip_final_aggregation=False), "concatenate",
                   [f"http://127.0.0.1:{ports['b1']}/v1", f"http://127.0.0.1:{ports['b2']}/v1"])
        req = {"messages": MSG, "stream": True}
        with native_server(cfg) as p:
            ref = _split(_events(httpx.post(f"http://127.0.0.1:{p}/chat/completions", json=req, headers=AUTH,
                                            timeout=30).text))
        with native_cluster(cfg, 2, tick_mode=tick_mode) as cports:
            import concurrent.futures as cf

            def one(i):
                with httpx.Client(base_url=f"http://127.0.0.1:{cports[i % 2]}") as c:
                    return [_split(_events(c.post("/chat/completions", json=req, headers=AUTH, timeout=30).text))
                            for _ in range(5)]
            with cf.ThreadPoolExecutor(8) as ex:
                for res in ex.map(one, range(8)):
                    for r in res:
                        assert r == ref
    finally:
        live.close()


def _selftest(world, transport, rounds, env=None, **opts):
    ext = native.require()
    port = free_port_block(2 * world)
    res = {}
    old = {k: os.environ.get(k) for k in (env or {})}
    os.environ.update(env or {})

    def run(r):
        res[r] = ext.exchange_selftest(dict({"rank": r, "world": world, "transport": transport, "port": port,
                                             "timeout": 20.0}, **opts), rounds)
    try:
        ts = [threading.Thread(target=run, args=(r,)) for r in range(world)]
        for t in ts:
            t.start()
        for t in ts:
            t.join(timeout=90)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    assert len(res) == world, res
    return res


def test_exchange_transport_selftest_tcp():
    """Raw transport: 3 ranks, 60 rounds of deltas and final texts over the mesh; every rank
    must receive every rank's exact bytes and flags."""
    res = _selftest(3, "tcp", 60)
    assert all(v["ok"] for v in res.values()), res


@pytest.mark.parametrize("world", [2, 4, 8])
def test_exchange_bulk_rounds_tcpbulk(world):
    """The RCCL round protocol with the socket executor: every rank sends every other rank
    40 final texts (1 B .. 20 KB) in rank-0-numbered rounds; each pair's transfers run in
    manifest order (each carries its round/skey/bi/len, so a desynchronised round would
    fail loudly), every byte is checked, and no text falls back to the mesh."""
    res = _selftest(world, "tcpbulk", 40)
    assert all(v["ok"] for v in res.values()), res
    for v in res.values():
        assert v["bad"] == 0 and v["bulk"] == 40 * (world - 1)
        assert v["rccl_rounds"] > 0 and v["mesh_finals"] == 0 and v["epochs"] >= 1


@pytest.mark.parametrize("world", [3, 4])
def test_exchange_bulk_round_stall_falls_back_and_reforms(world):
    """Fault injection: every rank of global round 3 hangs in it (QMX_XCHG_FAULT_STALL_ROUND;
    the sends are paced 3 ms apart so there are many rounds): the round times out, the
    communicator is dropped everywhere, the texts its receivers missed are resent over the
    mesh on their receivers' reports, and rank 0 re-forms a new epoch.  Every text must
    arrive exactly once and byte-exact — including texts whose SENDER finished the round
    while their receiver failed it on a third rank (the round-3 loss: before receiver reports
    the sender released those as sent and they vanished).  A second wave sent after the
    re-formed epoch must travel in its rounds again, with no mesh fallback."""
    res = _selftest(world, "tcpbulk", 24, env={"QMX_XCHG_FAULT_STALL_ROUND": "3"}, round_timeout=0.5,
                    min_epochs=2, pace_ms=3.0, wave2=12)
    assert all(v["ok"] for v in res.values()), res
    for v in res.values():
        assert v["bad"] == 0 and v["dups"] == 0
        assert v["bulk"] == v["sent"] == 36 * (world - 1)
        assert v["mesh_finals"] > 0          # the stalled round's texts took the mesh
        assert v["epochs"] >= 2              # a new communicator formed after the failure
        assert v["wave2_rounds"] > 0 and v["wave2_mesh_finals"] == 0, v  # ... and carries traffic


@pytest.mark.parametrize("control", [False, True])
def test_exchange_early_missed_report_is_kept(control):
    """A receiver on another epoch reports "missed" as soon as it reads a round's manifest,
    while its sender is still in its previous round: the report arrives before the send moves
    into `await` (round-4 advisor finding: it was dropped, and the send waited forever).
    QMX_XCHG_FAULT_EARLY_MISSED=1:3 — in the first global round >= 3 in which rank 1 receives,
    it acts as such a receiver (its own sends take the mesh) and every other rank carries its
    sends 100 ms late.  Every text
    must arrive exactly once, each missed one resent at its round's end from the kept report,
    never by the stale-await sweep (sweeps == 0).  control: the early reports dropped
    (QMX_XCHG_DEBUG_DROP_EARLY, the round-4 behaviour) — only the sweep recovers them."""
    env = {"QMX_XCHG_FAULT_EARLY_MISSED": "1:3"}
    if control:
        env["QMX_XCHG_DEBUG_DROP_EARLY"] = "1"
    res = _selftest(3, "tcpbulk", 24, env=env, round_timeout=0.5, min_epochs=2, pace_ms=3.0)
    assert sum(v["early_reports"] for v in res.values()) > 0, res  # the fault hit the path
    sweeps = sum(v["sweeps"] for v in res.values())
    if control:  # dropped reports: those texts wait for the sweep (3 round timeouts), or the test's end
        assert sweeps > 0 or any(v["bulk"] < 24 * 2 for v in res.values()), res
        return
    assert all(v["ok"] for v in res.values()), res
    for v in res.values():
        assert v["bad"] == 0 and v["dups"] == 0 and v["bulk"] == v["sent"] == 24 * 2, v
    assert sweeps == 0, res


def test_idle_cluster_exchanges_nothing():
    """Event-driven exchange: once the traffic stops, a 3-rank cluster sends no mesh message
    and runs no bulk round (the r1 design paced all-gather rounds forever)."""
    behs = [("stream", 200, sse_stream(["x"])), ("stream", 200, sse_stream(["y"])), ("stream", 200, sse_stream(["z"]))]
    live, ports = _live({f"b{i + 1}": b for i, b in enumerate(behs)})
    try:
        cfg = _cfg(3, CONCAT, "concatenate", [f"http://127.0.0.1:{ports[f'b{i + 1}']}/v1" for i in range(3)])
        req = {"messages": MSG, "stream": True}

        def snap(cports):
            tot = {}
            for p in cports:
                for ln in httpx.get(f"http://127.0.0.1:{p}/metrics").text.splitlines():
                    if ln.startswith("qmx_exchange_"):
                        k, v = ln.split()
                        tot[k] = tot.get(k, 0.0) + float(v)
            return tot

        with native_cluster(cfg, 3) as cports:
            for p in cports:
                assert httpx.post(f"http://127.0.0.1:{p}/chat/completions", json=req, headers=AUTH,
                                  timeout=30).status_code == 200
            time.sleep(0.3)
            a = snap(cports)
            time.sleep(1.0)
            b = snap(cports)
        # the traffic did cross ranks: over the io loops' own links (the default) and the mesh
        # (control: epochs, links' set-up); idle, neither moves
        assert a["qmx_exchange_link_messages_total"] > 0 and a["qmx_exchange_links_total"] > 0
        assert b["qmx_exchange_messages_total"] == a["qmx_exchange_messages_total"], (a, b)
        assert b["qmx_exchange_link_messages_total"] == a["qmx_exchange_link_messages_total"], (a, b)
        assert b["qmx_exchange_rounds_total"] == a["qmx_exchange_rounds_total"] == 0  # tcp: no RCCL rounds
        assert b["qmx_exchange_peers_up"] == 9  # 3 ranks x 3
    finally:
        live.close()


def test_spread_remote_deltas_coalesce_client_sends():
    """Spread placement: a session's remote streams deliver their deltas from other ranks, each
    in an io-loop pass of its own.  After the session's first content, a remote stream's last
    deltas (XF_LAST) wait corked while the rest of the session is to come — another stream
    still running (QMX_SESSION_HOLD) or the aggregator's answer (QMX_FINAL_HOLD), both default
    on — so the last arrival sends them all: the same bytes, fewer client sends than off
    (the 4-rank aggregate4 rehearsal on the MI355X box: 4.4 -> 2.8 client sends per request,
    74-77k -> 91-93k req/s, profiles/r6/spread_hold)."""
    n, block, strategy, behs = SPREAD_CASES["aggregate_4"]
    live, ports = _live({f"b{i + 1}": b for i, b in enumerate(behs)})
    try:
        cfg = _cfg(n, block, strategy, [f"http://127.0.0.1:{ports[f'b{i + 1}']}/v1" for i in range(n)])
        req = {"messages": MSG, "stream": True}
        runs = {}
        for hold in ("1", "0"):
            with native_cluster(cfg, 4, run_env={"QMX_SESSION_HOLD": hold, "QMX_FINAL_HOLD": hold}) as cports:
                m0 = [httpx.get(f"http://127.0.0.1:{p}/metrics").text for p in cports]
                bodies = [httpx.post(f"http://127.0.0.1:{cports[0]}/chat/completions", json=req, headers=AUTH,
                                     timeout=30).text for _ in range(24)]
                m1 = [httpx.get(f"http://127.0.0.1:{p}/metrics").text for p in cports]

            def d(k, m0=m0, m1=m1):  # rank 0: the owner of every session (its clients)
                return _metric(m1[0], k) - _metric(m0[0], k)
            runs[hold] = (bodies, d("qmx_output_coalesced_total"), d('qmx_syscalls_total{op="client_send"}'),
                          d("qmx_remote_streams_total"))
        on, off = runs["1"], runs["0"]
        print("spread hold on/off (coalesced, client sends):", on[1:3], off[1:3])
        assert [_split(_events(b)) for b in on[0]] == [_split(_events(b)) for b in off[0]]
        assert on[3] == off[3] == 3 * 24  # backends 1..3 of every session ran on other ranks
        assert on[1] > off[1]  # remote deltas were held ...
        assert on[2] < off[2]  # ... and left in fewer client sends
    finally:
        live.close()
