"""Streaming conformance (quorum tests/test_streaming.py + SURVEY §2.6 event shapes)."""
import json

import httpx

from conftest import CFG_BLANK, cfg_parallel, make_client, sse_chunk, sse_events, sse_lines, sse_stream

AUTH = {"Authorization": "Bearer test-key"}
MSG = [{"role": "user", "content": "Hello!"}]
CONCAT = {"separator": "\n-------------\n", "hide_intermediate_think": True,
          "hide_final_think": False, "thinking_tags": ["think", "reason", "reasoning", "thought", "Thought"],
          "skip_final_aggregation": False}


def test_single_backend_stream_four_lines(upstream):
    upstream.stream("b1.test", sse_stream(["Hello"]))
    c = make_client(CFG_BLANK, upstream)
    r = c.post("/chat/completions", json={"model": "gpt-4", "messages": MSG, "stream": True}, headers=AUTH)
    assert r.status_code == 200
    assert r.headers["content-type"].split(";")[0] == "text/event-stream"
    assert upstream.calls[0]["body"]["stream"] is True
    lines = sse_lines(r)
    assert len(lines) == 4
    role = json.loads(lines[0][6:])
    assert set(role) == {"id", "object", "created", "model", "choices"}
    assert role["object"] == "chat.completion.chunk" and role["id"] == "chatcmpl-role"
    assert role["model"] == "gpt-4"
    assert role["choices"][0]["delta"] == {"role": "assistant"}
    assert "Hello" in json.loads(lines[1][6:])["choices"][0]["delta"]["content"]
    assert json.loads(lines[2][6:])["choices"][0]["finish_reason"] == "stop"
    assert lines[3] == "data: [DONE]"


def test_single_backend_stream_appends_done(upstream):
    upstream.stream("b1.test", sse_stream(["x"], done=False))
    c = make_client(CFG_BLANK, upstream)
    r = c.post("/chat/completions", json={"model": "gpt-4", "messages": MSG, "stream": True}, headers=AUTH)
    assert sse_lines(r)[-1] == "data: [DONE]"


def test_single_backend_stream_failure(upstream):
    upstream.json("b1.test", {"error": {"message": "boom", "type": "x"}}, status=502)
    c = make_client(CFG_BLANK, upstream)
    r = c.post("/chat/completions", json={"model": "gpt-4", "messages": MSG, "stream": True}, headers=AUTH)
    assert r.status_code == 502
    assert r.json()["error"] == {"message": "Backend failed: boom", "type": "proxy_error"}


def test_parallel_stream_shapes(upstream):
    upstream.stream("b1.test", sse_stream(["Hel", "lo"]))
    upstream.stream("b2.test", sse_stream(["Wor", "ld"]))
    c = make_client(cfg_parallel(2, block=CONCAT), upstream)
    r = c.post("/chat/completions", json={"messages": MSG, "stream": True}, headers=AUTH)
    assert r.status_code == 200
    assert r.headers["content-type"].split(";")[0] == "text/event-stream"
    evs = sse_events(r)
    assert evs[-1] == "[DONE]"
    role, final = evs[0], evs[-2]
    assert role["id"] == "chatcmpl-parallel" and role["model"] == "parallel-proxy"
    assert role["choices"][0] == {"index": 0, "delta": {"role": "assistant"}, "finish_reason": None}
    assert final["id"] == "chatcmpl-parallel-final" and final["choices"][0]["finish_reason"] == "stop"
    assert final["choices"][0]["delta"]["content"] == "Hello\n\n-------------\nWorld"
    per = {0: "", 1: ""}
    for e in evs[1:-2]:
        idx = int(e["id"].rsplit("-", 1)[1])
        assert e["choices"][0]["finish_reason"] is None and e["model"] == "parallel-proxy"
        per[idx] += e["choices"][0]["delta"]["content"]
    assert per == {0: "Hello", 1: "World"}


def test_parallel_stream_exact_bytes(upstream):
    """Exact wire format: json.dumps separators, ensure_ascii escaping."""
    upstream.stream("b1.test", sse_stream(['é"\\\n😀']))
    upstream.stream("b2.test", sse_stream(["z"]))
    c = make_client(cfg_parallel(2, block=dict(CONCAT, skip_final_aggregation=True)), upstream)
    r = c.post("/chat/completions", json={"messages": MSG, "stream": True}, headers=AUTH)
    raw = r.content
    ev0 = [seg for seg in raw.split(b"\n\n") if b"chatcmpl-parallel-0" in seg][0]
    created = json.loads(ev0[6:])["created"]
    expect = ('data: {"id": "chatcmpl-parallel-0", "object": "chat.completion.chunk", "created": %d, '
              '"model": "parallel-proxy", "choices": [{"index": 0, "delta": {"content": '
              '"\\u00e9\\"\\\\\\n\\ud83d\\ude00"}, "finish_reason": null}]}' % created).encode()
    assert ev0 == expect


def test_parallel_all_fail_error_event(upstream):
    upstream.route("b1.test", lambda req, b: httpx.Response(500, json={"error": {"message": "e"}}))
    upstream.route("b2.test", lambda req, b: httpx.Response(500, json={"error": {"message": "e"}}))
    c = make_client(cfg_parallel(2, block=CONCAT), upstream)
    r = c.post("/chat/completions", json={"messages": MSG, "stream": True}, headers=AUTH)
    evs = sse_events(r)
    assert evs[-1] == "[DONE]"
    err = evs[-2]
    assert err["id"] == "error" and err["choices"][0]["finish_reason"] == "error"
    assert err["choices"][0]["delta"]["content"] == "Error: All backends failed to provide content"


def test_parallel_all_fail_skip_final_no_error(upstream):
    upstream.route("b1.test", lambda req, b: httpx.Response(500, json={}))
    upstream.route("b2.test", lambda req, b: httpx.Response(500, json={}))
    c = make_client(cfg_parallel(2, block=dict(CONCAT, skip_final_aggregation=True)), upstream)
    r = c.post("/chat/completions", json={"messages": MSG, "stream": True}, headers=AUTH)
    evs = sse_events(r)
    assert len(evs) == 2 and evs[0]["id"] == "chatcmpl-parallel" and evs[1] == "[DONE]"


def test_parallel_suppress_individual(upstream):
    upstream.stream("b1.test", sse_stream(["a"]))
    upstream.stream("b2.test", sse_stream(["b"]))
    c = make_client(cfg_parallel(2, block=CONCAT), upstream)
    r = c.post("/chat/completions", json={"messages": MSG, "stream": True,
                                          "suppress_individual_responses": True}, headers=AUTH)
    evs = sse_events(r)
    assert [e if e == "[DONE]" else e["id"] for e in evs] == \
        ["chatcmpl-parallel", "chatcmpl-parallel-final", "[DONE]"]
    # the flag is forwarded upstream (body passed as-is, quorum :1072-1075)
    assert upstream.calls[0]["body"]["suppress_individual_responses"] is True


def test_parallel_think_filtering(upstream):
    def thinking(tag):
        return [sse_chunk({"role": "assistant"}), sse_chunk({"content": f"<{tag}>"}),
                sse_chunk({"content": "Let me think about this..."}), sse_chunk({"content": f"</{tag}>"}),
                sse_chunk({"content": "The answer "}), sse_chunk({"content": "is "}),
                sse_chunk({"content": "4"}), sse_chunk({"content": "."}),
                sse_chunk({}, finish="stop"), b"data: [DONE]\n\n"]
    upstream.stream("b1.test", thinking("think"))
    upstream.stream("b2.test", thinking("reason"))
    c = make_client(cfg_parallel(2, block=dict(CONCAT, hide_final_think=True,
                                               thinking_tags=["think", "reason", "reasoning", "thought"])),
                    upstream)
    r = c.post("/chat/completions", json={"messages": MSG, "stream": True}, headers=AUTH)
    evs = sse_events(r)
    body = "".join(e["choices"][0]["delta"].get("content", "") for e in evs[1:-2])
    final = evs[-2]["choices"][0]["delta"]["content"]
    assert "<think>" not in body and "Let me think" not in body
    assert final == "The answer is 4.\n\n-------------\nThe answer is 4."


def test_parallel_split_events_and_bytes(upstream):
    """Events split at arbitrary byte boundaries (incl. inside UTF-8) reassemble exactly."""
    stream = b"".join(sse_stream(["héllo ", "<thi", "nk>x</th", "ink>wörld"]))
    chunks = [stream[i:i + 7] for i in range(0, len(stream), 7)]
    upstream.stream("b1.test", chunks)
    upstream.stream("b2.test", sse_stream(["b"]))
    c = make_client(cfg_parallel(2, block=CONCAT), upstream)
    r = c.post("/chat/completions", json={"messages": MSG, "stream": True}, headers=AUTH)
    evs = sse_events(r)
    got = "".join(e["choices"][0]["delta"]["content"] for e in evs[1:-2] if e["id"] == "chatcmpl-parallel-0")
    assert got == "héllo wörld"


def test_parallel_null_content_aborts_backend(upstream):
    """quorum: content:null raises in the filter → rest of that backend dropped and it is
    excluded from the final (SURVEY §2.7-C probe)."""
    upstream.stream("b1.test", [sse_chunk({"content": "alpha "}), sse_chunk({"content": None}),
                                sse_chunk({"content": "beta"}), b"data: [DONE]\n\n"])
    upstream.stream("b2.test", sse_stream(["B"]))
    c = make_client(cfg_parallel(2, block=CONCAT), upstream)
    r = c.post("/chat/completions", json={"messages": MSG, "stream": True}, headers=AUTH)
    evs = sse_events(r)
    b0 = [e["choices"][0]["delta"]["content"] for e in evs if e != "[DONE]" and e["id"] == "chatcmpl-parallel-0"]
    assert b0 == ["alpha "]
    assert evs[-2]["choices"][0]["delta"]["content"] == "B"


def test_parallel_empty_after_strip_still_joined(upstream):
    """`if text` filters BEFORE the strip (quorum :760-764): an all-think backend joins as ''."""
    upstream.stream("b1.test", sse_stream(["<think>only</think>"]))
    upstream.stream("b2.test", sse_stream(["B"]))
    c = make_client(cfg_parallel(2, block=dict(CONCAT, hide_intermediate_think=False, hide_final_think=True)),
                    upstream)
    r = c.post("/chat/completions", json={"messages": MSG, "stream": True}, headers=AUTH)
    evs = sse_events(r)
    assert evs[-2]["choices"][0]["delta"]["content"] == "\n\n-------------\nB"


def test_parallel_malformed_events_skipped(upstream):
    upstream.stream("b1.test", [b"data: {bad json}\n\n", b"event: x\n\n", b"data:{\"a\":1}\n\n",
                                sse_chunk({"content": "ok"}), b"data: [DONE]\n\n"])
    upstream.stream("b2.test", sse_stream(["B"]))
    c = make_client(cfg_parallel(2, block=CONCAT), upstream)
    r = c.post("/chat/completions", json={"messages": MSG, "stream": True}, headers=AUTH)
    evs = sse_events(r)
    assert evs[-2]["choices"][0]["delta"]["content"] == "ok\n\n-------------\nB"


def test_parallel_one_backend_refused(upstream):
    upstream.route("b1.test", lambda req, b: httpx.ConnectError("refused"))
    upstream.stream("b2.test", sse_stream(["B"]))
    c = make_client(cfg_parallel(2, block=CONCAT), upstream)
    r = c.post("/chat/completions", json={"messages": MSG, "stream": True}, headers=AUTH)
    evs = sse_events(r)
    assert evs[-2]["choices"][0]["delta"]["content"] == "B"
