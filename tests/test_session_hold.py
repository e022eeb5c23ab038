"""Session-level output holds (qmx_server.cpp ``session_hold``): a stream's LAST output may wait
for the rest of its session (another stream still running; an aggregator answer to come), so
fast sessions leave in fewer client sends.  A trickling stream's earlier deltas must never wait
for other streams: per-token latency of a realistic (per-event) upstream is unchanged even
with a long coalescing deadline."""
import threading
import time

import httpx
import pytest

from quorum_amd.ops import native

from conftest import cfg_parallel, sse_chunk
from live_upstream import LiveUpstream, native_server

pytestmark = pytest.mark.skipif(not native.available(), reason="native extension not built")

AUTH = {"Authorization": "Bearer test-key"}
MSG = [{"role": "user", "content": "hi"}]
GAP = 0.05


def _trickle(words):
    out = [sse_chunk({"role": "assistant"})]
    for w in words:
        out += [sse_chunk({"content": w}), GAP]
    return out + [sse_chunk({}, finish="stop"), b"data: [DONE]\n\n"]


def test_trickling_tokens_do_not_wait_for_a_slow_sibling(monkeypatch):
    # a 300 ms coalescing deadline: a token wrongly held for the slow stream (or the deadline)
    # would reach the client hundreds of ms late, after the slow stream's answer
    monkeypatch.setenv("QMX_COALESCE_US", "300000")
    monkeypatch.setenv("QMX_READ_PACE_US", "0")
    live = LiveUpstream()
    words = [f"tok{i} " for i in range(6)]
    p1 = live.serve("b1", ("stream", 200, _trickle(words)))
    p2 = live.serve("b2", ("stream", 200, [1.2, sse_chunk({"role": "assistant"}), sse_chunk({"content": "late"}),
                                           sse_chunk({}, finish="stop"), b"data: [DONE]\n\n"]))
    try:
        cfg = cfg_parallel(2, block={"separator": "\n--\n", "hide_intermediate_think": True,
                                     "hide_final_think": False, "thinking_tags": ["think"],
                                     "skip_final_aggregation": False})
        cfg["primary_backends"][0]["url"] = f"http://127.0.0.1:{p1}/v1"
        cfg["primary_backends"][1]["url"] = f"http://127.0.0.1:{p2}/v1"
        with native_server(cfg, threads=1) as port:
            seen = {}
            t0 = time.time()
            buf = b""
            with httpx.stream("POST", f"http://127.0.0.1:{port}/chat/completions",
                              json={"messages": MSG, "stream": True}, headers=AUTH, timeout=30) as r:
                for chunk in r.iter_bytes():
                    buf += chunk
                    now = time.time() - t0
                    for w in words + ["late"]:
                        if w.encode() in buf and w not in seen:
                            seen[w] = now
        assert set(seen) == set(words + ["late"]), seen
        # the fast stream's tokens arrive at its own pace (one every GAP), long before the slow
        # stream answers (1.2 s) — not held from tok1 on for it or the 300 ms coalescing deadline
        print("arrivals (s):", {w.strip(): round(t, 3) for w, t in seen.items()})
        for i, w in enumerate(words[:5]):
            assert seen[w] - seen[words[0]] < i * GAP + 0.08, (w, seen)
        assert seen["late"] >= 1.1
    finally:
        live.close()
