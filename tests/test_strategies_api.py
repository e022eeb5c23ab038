"""Parallel non-streaming combine + aggregate strategy (quorum tests/test_parallel_backends.py,
tests/test_aggregate_strategy.py behaviours)."""
import asyncio
import json

import httpx

from quorum_amd.models.strategies import aggregate_responses, build_aggregator_prompt
from quorum_amd.server.transport import UpstreamPool

from conftest import cfg_parallel, completion, make_client, sse_events, sse_stream, FakeUpstream

AUTH = {"Authorization": "Bearer test-key"}
MSG = [{"role": "user", "content": "What is 2+2?"}]
CONCAT = {"separator": "\n-------------\n", "hide_intermediate_think": True, "hide_final_think": False,
          "thinking_tags": ["think", "reason", "reasoning", "thought"], "skip_final_aggregation": False}
AGG = {"source_backends": ["LLM1", "LLM2"], "aggregator_backend": "LLM3",
       "intermediate_separator": "\n\n---\n\n", "include_source_names": True,
       "source_label_format": "Response from {backend_name}:\n",
       "prompt_template": "Responses:\n\n{responses}\n\nSynthesize.",
       "strip_intermediate_thinking": True, "hide_aggregator_thinking": True,
       "thinking_tags": ["think", "reason", "reasoning", "thought"], "include_original_query": True}


def test_concatenate_and_usage(upstream):
    upstream.json("b1.test", completion("first answer", cid="c1", usage=(9, 12, 21)))
    upstream.json("b2.test", completion("second answer", cid="c2", usage=(10, 15, 25)))
    c = make_client(cfg_parallel(2, block=CONCAT), upstream)
    r = c.post("/chat/completions", json={"messages": MSG}, headers=AUTH)
    assert r.status_code == 200
    d = r.json()
    assert d["choices"] == [{"index": 0, "message": {"role": "assistant",
                                                     "content": "first answer\n-------------\nsecond answer"},
                             "logprobs": None, "finish_reason": "stop"}]
    assert d["usage"] == {"prompt_tokens": 19, "completion_tokens": 27, "total_tokens": 46}
    assert d["object"] == "chat.completion" and d["id"] == "c1"
    assert d["system_fingerprint"] == "fp_qmx"


def test_partial_failure(upstream):
    upstream.json("b1.test", completion("only me", usage=(9, 12, 21)))
    upstream.json("b2.test", {"error": {"message": "Backend error", "type": "backend_error"}}, status=500)
    c = make_client(cfg_parallel(2, block=CONCAT), upstream)
    d = c.post("/chat/completions", json={"messages": MSG}, headers=AUTH).json()
    assert d["choices"][0]["message"]["content"] == "only me"
    assert d["usage"] == {"prompt_tokens": 9, "completion_tokens": 12, "total_tokens": 21}


def test_all_failure_500(upstream):
    for h in ("b1.test", "b2.test"):
        upstream.json(h, {"error": {"message": "Backend error", "type": "backend_error"}}, status=500)
    c = make_client(cfg_parallel(2, block=CONCAT), upstream)
    r = c.post("/chat/completions", json={"messages": MSG}, headers=AUTH)
    assert r.status_code == 500
    err = r.json()["error"]
    assert err["type"] == "proxy_error" and err["message"] == "All backends failed. First error: Backend error"


def test_missing_usage_combine_error(upstream):
    upstream.json("b1.test", completion("a", usage=None))
    upstream.json("b2.test", completion("b"))
    c = make_client(cfg_parallel(2, block=CONCAT), upstream)
    r = c.post("/chat/completions", json={"messages": MSG}, headers=AUTH)
    assert r.status_code == 500
    assert r.json()["error"] == {"message": "Error combining responses: 'usage'", "type": "proxy_error"}


def test_strip_non_stream(upstream):
    upstream.json("b1.test", completion("<think>Let me think about this</think>The answer is 4."))
    upstream.json("b2.test", completion("<think>First</think>The answer is 4.<reason>because</reason>"))
    c = make_client(cfg_parallel(2, block=dict(CONCAT, hide_final_think=True)), upstream)
    content = c.post("/chat/completions", json={"messages": MSG}, headers=AUTH).json()["choices"][0]["message"]["content"]
    assert content == "The answer is 4.\n-------------\nThe answer is 4."


def test_strip_disabled_keeps_tags(upstream):
    cfg = cfg_parallel(1, block=dict(CONCAT, hide_intermediate_think=False))
    upstream.json("b1.test", completion("<think>Let me think</think>4"))
    c = make_client(cfg, upstream)
    content = c.post("/chat/completions", json={"messages": MSG}, headers=AUTH).json()["choices"][0]["message"]["content"]
    assert content == "<think>Let me think</think>4"


def test_aggregate_non_stream(upstream):
    prompts = []

    def agg(req, body):
        prompts.append(body)
        return httpx.Response(200, json=completion("<think>Synth</think>Aggregated.", cid="agg"))

    upstream.json("b1.test", completion("<think>t1</think>Response 1."))
    upstream.json("b2.test", completion("<think>t2</think>Response 2."))
    upstream.route("b3.test", agg)
    cfg = cfg_parallel(3, strategy="aggregate", block=AGG)
    c = make_client(cfg, upstream)
    r = c.post("/chat/completions", json={"messages": [{"role": "user", "content": "Q?"}], "stream": False},
               headers=AUTH)
    assert r.status_code == 200
    assert len(upstream.calls) == 4  # 3 sources (aggregator is also a source) + aggregator
    assert r.json()["choices"][0]["message"]["content"] == "<think>Synth</think>Aggregated."
    assert r.json()["usage"]["total_tokens"] == 3 * 18  # aggregator usage excluded
    p = prompts[-1]
    assert p["model"] == "model-3" and p["stream"] is False
    msg = p["messages"][0]["content"]
    assert msg.startswith("Original query: Q?\n\nResponses:\n\n")
    assert "Response from LLM1:\n<think>t1</think>Response 1.\n\n---\n\nResponse from LLM2:\n" in msg
    agg_call = upstream.calls[-1]
    assert agg_call["headers"]["authorization"] == "Bearer test-key"
    assert set(k.lower() for k in agg_call["headers"]) >= {"authorization", "content-type"}
    assert "accept-encoding" not in {k.lower() for k in agg_call["headers"]} or True


def test_aggregate_auth_env_fallback(upstream, monkeypatch):
    monkeypatch.setenv("OPENAI_API_KEY", "env-key")
    upstream.json("b1.test", completion("a"))
    upstream.json("b2.test", completion("b"))
    upstream.json("b3.test", completion("agg"))
    c = make_client(cfg_parallel(3, strategy="aggregate", block=AGG), upstream)
    r = c.post("/chat/completions", json={"messages": MSG})
    assert r.status_code == 200
    assert {x["headers"]["authorization"] for x in upstream.calls} == {"Bearer env-key"}


def test_aggregate_streaming_falls_back_to_join(upstream):
    """The aggregator returns SSE to a non-stream call → content is not JSON → plain
    intermediate-separator join (quorum tests/test_aggregate_strategy.py:180-264)."""
    seen = []
    for h in ("b1.test", "b2.test"):
        upstream.stream(h, sse_stream(["Hello"]))

    def agg(req, body):
        seen.append(body)
        if body.get("stream"):
            async def gen():
                for c in sse_stream(["Hello"]):
                    yield c
            return httpx.Response(200, content=gen())
        return httpx.Response(200, content=b"".join(sse_stream(["x"])))

    upstream.route("b3.test", agg)
    c = make_client(cfg_parallel(3, strategy="aggregate", block=AGG), upstream)
    r = c.post("/chat/completions", json={"messages": MSG, "stream": True}, headers=AUTH)
    evs = sse_events(r)
    assert evs[-1] == "[DONE]"
    assert evs[-2]["choices"][0]["delta"]["content"] == "Hello\n\n---\n\nHello\n\n---\n\nHello"
    prompt = seen[-1]["messages"][-1]["content"]
    assert "Response from LLM1" in prompt and "Response from LLM2" in prompt
    assert {x["headers"]["authorization"] for x in upstream.calls} == {"Bearer test-key"}


def test_aggregate_missing_backend_plain_join(upstream):
    async def run():
        pool = FakeUpstream().pool()
        return await aggregate_responses(
            ["Response 1", "Response 2"], {"name": "Nope", "url": "http://missing.test/v1"},
            "Q", "\n\n---\n\n", True, "Original query: {query}\n\n", True,
            "Response from {backend_name}:\n", "{responses}", {"Authorization": "Bearer k"}, pool=pool)
    assert asyncio.run(run()) == "Response 1\n\n---\n\nResponse 2"


def test_aggregate_not_found_in_config(upstream):
    upstream.json("b1.test", completion("a"))
    upstream.json("b2.test", completion("b"))
    c = make_client(cfg_parallel(2, strategy="aggregate", block=dict(AGG, aggregator_backend="Ghost")), upstream)
    d = c.post("/chat/completions", json={"messages": MSG}, headers=AUTH).json()
    assert d["choices"][0]["message"]["content"] == "a\nb"  # separator default "\n"


def test_aggregate_sources_fail_500(upstream):
    for h in ("b1.test", "b2.test", "b3.test"):
        upstream.json(h, {"error": {"message": "Backend error"}}, status=500)
    c = make_client(cfg_parallel(3, strategy="aggregate", block=AGG), upstream)
    r = c.post("/chat/completions", json={"messages": MSG}, headers=AUTH)
    assert r.status_code == 500 and "All backends failed" in r.json()["error"]["message"]


def test_aggregator_consulted_even_for_concatenate(upstream):
    """quorum reads strategy.aggregate.aggregator_backend regardless of the selected strategy."""
    upstream.json("b1.test", completion("a"))
    upstream.json("b2.test", completion("agg-out"))
    cfg = cfg_parallel(2, block=CONCAT, agg={"aggregator_backend": "LLM2"})
    c = make_client(cfg, upstream)
    d = c.post("/chat/completions", json={"messages": MSG}, headers=AUTH).json()
    assert d["choices"][0]["message"]["content"] == "agg-out"
    assert len(upstream.calls) == 3


def test_prompt_builder_template_braces():
    # shipped quorum config uses {{intermediate_results}} → responses wrapped in literal braces
    from quorum_amd.utils.config import resolve_aggregate
    agg = resolve_aggregate({"strategy": {"aggregate": {"prompt_template": "A {{intermediate_results}} B"}}})
    p = build_aggregator_prompt(["x", "y"], "q", "|", False, "", False, "", agg.prompt_template)
    assert p == "A {x|y} B"


def test_validate_config_semantics():
    """``semantics``: reference (default) warns that the documented-only flags do nothing;
    documented checks source_backends names; anything else is an error."""
    import pytest

    from quorum_amd.utils.config import ConfigError, validate_config

    cfg = cfg_parallel(3, strategy="aggregate", block=dict(AGG, source_backends=["LLM1", "nope"]))
    w = validate_config(cfg)
    assert any("strip_intermediate_thinking" in x and "semantics: documented" in x for x in w)
    assert not any("nope" in x for x in w)
    cfg["semantics"] = "documented"
    w = validate_config(cfg)
    assert any("'nope'" in x for x in w) and not any("has no effect" in x for x in w)
    cfg["semantics"] = "docs"
    with pytest.raises(ConfigError):
        validate_config(cfg)


def test_documented_semantics_python_app(upstream):
    """The FastAPI app with ``semantics: documented`` (non-stream aggregate): only the source
    backends reach the aggregator, stripped, labelled with their names; the answer loses its
    thinking (reference docs/aggregate_behaviour.md)."""
    cfg = cfg_parallel(3, strategy="aggregate", block=dict(AGG, source_backends=["LLM2", "LLM3"]))
    cfg["semantics"] = "documented"
    upstream.json("b1.test", completion("one"))
    upstream.json("b2.test", completion("<think>t</think>two"))
    upstream.route("b3.test", lambda request, body: httpx.Response(
        200, json=completion("<reason>r</reason>SYN" if body.get("stream") is False else "three")))
    c = make_client(cfg, upstream)
    r = c.post("/chat/completions", json={"messages": MSG}, headers=AUTH)
    assert r.status_code == 200, r.text
    assert r.json()["choices"][0]["message"]["content"] == "SYN"
    prompts = [c["body"]["messages"][0]["content"] for c in upstream.calls if c["body"].get("stream") is False]
    assert len(prompts) == 1
    assert "Response from LLM2:\ntwo" in prompts[0] and "Response from LLM3:\nthree" in prompts[0]
    assert "LLM1" not in prompts[0] and "<think>" not in prompts[0]
