"""Read pacing (runtime.read_pace_us): an io-loop pass that read trickling upstreams — short
reads of responses still in progress, one SSE event per write — is stretched to the pace so
the events that arrive meanwhile share receives, waits and client sends.  Pacing only moves
time: responses must be byte-identical with it on and off, it must engage on per-event
upstreams and never on whole-response ones (the headline's shape)."""
import concurrent.futures as cf
import copy

import httpx
import pytest

from quorum_amd.ops import native

from conftest import cfg_parallel, sse_chunk
from live_upstream import LiveUpstream, native_server

pytestmark = pytest.mark.skipif(not native.available(), reason="native extension not built")

AUTH = {"Authorization": "Bearer test-key"}
MSG = [{"role": "user", "content": "hi"}]
BLOCK = {"separator": "\n--\n", "hide_intermediate_think": True, "hide_final_think": False,
         "thinking_tags": ["think"], "skip_final_aggregation": False}


def _trickle(words, gap=0.0005):
    """One HTTP chunk per SSE event, with a short gap between writes (a token-by-token LLM)."""
    out = [sse_chunk({"role": "assistant"}), gap, sse_chunk({"content": "<think>"}), gap,
           sse_chunk({"content": "plan"}), gap, sse_chunk({"content": "</think>"})]
    for w in words:
        out += [gap, sse_chunk({"content": w})]
    return out + [gap, sse_chunk({}, finish="stop"), b"data: [DONE]\n\n"]


def _whole(words):
    """The whole response in one chunk (one write)."""
    body = b"".join([sse_chunk({"role": "assistant"})] + [sse_chunk({"content": w}) for w in words]
                    + [sse_chunk({}, finish="stop"), b"data: [DONE]\n\n"])
    return [body]


def _metric(text, name):
    return float([ln for ln in text.splitlines() if ln.startswith(name + " ")][0].split()[1])


def _run(cfg, pace_us, n=12):
    cfg = copy.deepcopy(cfg)
    cfg.setdefault("runtime", {})["read_pace_us"] = pace_us
    with native_server(cfg, threads=1) as port:
        base = f"http://127.0.0.1:{port}"
        m0 = httpx.get(base + "/metrics").text

        def one(_):
            return httpx.post(base + "/chat/completions", json={"messages": MSG, "stream": True}, headers=AUTH,
                              timeout=30).text
        with cf.ThreadPoolExecutor(4) as ex:
            bodies = list(ex.map(one, range(n)))
        m1 = httpx.get(base + "/metrics").text
    return bodies, _metric(m1, "qmx_loop_paced_total") - _metric(m0, "qmx_loop_paced_total")


def _strip_ids(text):
    """Per-stream event lists (the two backends' deltas interleave by timing) + the rest."""
    import json
    per, rest = {}, []
    for seg in text.split("\n\n"):
        if not seg.startswith("data: "):
            continue
        p = seg[6:]
        if p == "[DONE]":
            rest.append(p)
            continue
        ev = json.loads(p)
        ev["created"] = 0
        per.setdefault(ev.get("id", ""), []).append(json.dumps(ev, sort_keys=True))
    return json.dumps([sorted(per.items()), rest])


@pytest.mark.parametrize("shape", ["trickle", "whole"])
def test_read_pacing_changes_timing_not_bytes(shape):
    words = [f"w{i} " for i in range(24)]
    live = LiveUpstream()
    make = _trickle if shape == "trickle" else _whole
    p1 = live.serve("b1", ("stream", 200, make(words)))
    p2 = live.serve("b2", ("stream", 200, make(words[::-1])))
    try:
        cfg = cfg_parallel(2, block=dict(BLOCK))
        cfg["primary_backends"][0]["url"] = f"http://127.0.0.1:{p1}/v1"
        cfg["primary_backends"][1]["url"] = f"http://127.0.0.1:{p2}/v1"
        on, paced = _run(cfg, 200)
        off, unpaced = _run(cfg, 0)
    finally:
        live.close()
    assert unpaced == 0
    # same bytes per request (ids and timestamps aside), every one complete
    assert sorted(map(_strip_ids, on)) == sorted(map(_strip_ids, off))
    assert all(b.rstrip().endswith("data: [DONE]") for b in on)
    if shape == "trickle":
        assert paced > 0  # per-event upstreams engaged it
    else:
        assert paced == 0  # whole-response reads never do
