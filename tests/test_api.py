"""HTTP conformance: health, auth, config, single-backend and multi-backend non-streaming.

Re-expresses quorum's tests/test_health.py, test_auth.py, test_config.py and
test_chat_completions.py behaviours against a transport-level fake upstream.
"""
import json

import httpx
import yaml

from quorum_amd.utils.config import load_config

from conftest import CFG_BLANK, CFG_MODEL, completion, make_client

AUTH = {"Authorization": "Bearer test-key"}
MSG = [{"role": "user", "content": "Hello!"}]


def test_health(upstream):
    c = make_client(CFG_BLANK, upstream)
    r = c.get("/health")
    assert r.status_code == 200 and r.json() == {"status": "healthy"}


def test_metrics_endpoint(upstream):
    c = make_client(CFG_BLANK, upstream)
    r = c.get("/metrics")
    assert r.status_code == 200 and "qmx_request_seconds" in r.text


def test_no_auth_401(upstream):
    c = make_client(CFG_BLANK, upstream)
    r = c.post("/chat/completions", json={"model": "gpt-4", "messages": MSG})
    assert r.status_code == 401
    assert r.json()["error"] == {
        "message": "Authorization header is required and OPENAI_API_KEY environment variable is not set",
        "type": "auth_error"}


def test_env_key_fallback(upstream, monkeypatch):
    monkeypatch.setenv("OPENAI_API_KEY", "k-from-env")
    upstream.json("b1.test", completion("Hello from the mock!"))
    c = make_client(CFG_BLANK, upstream)
    r = c.post("/chat/completions", json={"model": "gpt-4", "messages": MSG})
    assert r.status_code == 200
    assert r.json()["choices"][0]["message"]["content"] == "Hello from the mock!"
    assert upstream.calls[0]["headers"]["authorization"] == "Bearer k-from-env"


def test_lowercase_authorization_normalised(upstream):
    upstream.json("b1.test", completion("ok"))
    c = make_client(CFG_BLANK, upstream)
    r = c.post("/chat/completions", json={"model": "gpt-4", "messages": MSG},
               headers={"authorization": "Bearer lower"})
    assert r.status_code == 200
    assert upstream.calls[0]["headers"]["authorization"] == "Bearer lower"


def test_no_model_400(upstream):
    c = make_client(CFG_BLANK, upstream)
    r = c.post("/chat/completions", json={"messages": MSG}, headers=AUTH)
    assert r.status_code == 400
    assert r.json()["error"] == {"message": "Model must be specified when config.yaml model is blank",
                                 "type": "invalid_request_error"}


def test_config_model_overrides_request(upstream):
    upstream.json("b1.test", completion("hi"))
    c = make_client(CFG_MODEL, upstream)
    for body in ({"model": "gpt-4", "messages": MSG}, {"messages": MSG}):
        r = c.post("/chat/completions", json=body, headers=AUTH)
        assert r.status_code == 200
        assert r.headers["content-type"] == "application/json"
        data = r.json()
        assert {"id", "object", "created", "model", "choices", "usage"} <= set(data)
        assert data["object"] == "chat.completion"
        sent = upstream.calls[-1]["body"]
        assert sent["model"] == "cfg-model" and sent["messages"] == MSG
        # re-serialised with json.dumps separators (quorum :161-163)
        assert upstream.calls[-1]["raw"] == json.dumps({**body, "model": "cfg-model"}).encode()


def test_request_model_when_config_blank(upstream):
    upstream.json("b1.test", completion("hi"))
    c = make_client(CFG_BLANK, upstream)
    r = c.post("/chat/completions", json={"model": "gpt-4", "messages": MSG}, headers=AUTH)
    assert r.status_code == 200
    assert upstream.calls[0]["body"]["model"] == "gpt-4"
    # non-parallel passthrough returns upstream JSON + "backend" (quorum :212)
    assert r.json()["backend"] == "LLM1"


def test_content_length_matches_body(upstream):
    upstream.json("b1.test", completion("hi"))
    c = make_client(CFG_BLANK, upstream)
    r = c.post("/chat/completions", json={"model": "deepseek-r1:1.5bt", "messages": MSG}, headers=AUTH)
    assert r.status_code == 200
    call = upstream.calls[0]
    assert int(call["headers"]["content-length"]) == len(call["raw"])


def test_multiple_backends_non_stream_calls_all(upstream):
    cfg = {"primary_backends": [{"name": "a", "url": "http://b1.test", "model": ""},
                                {"name": "b", "url": "http://b2.test", "model": ""}],
           "settings": {"timeout": 60}}
    upstream.json("b1.test", completion("one"))
    upstream.json("b2.test", completion("two"))
    c = make_client(cfg, upstream)
    r = c.post("/chat/completions", json={"model": "gpt-4", "messages": MSG}, headers=AUTH)
    assert r.status_code == 200
    assert sorted(x["url"] for x in upstream.calls) == ["http://b1.test/chat/completions",
                                                        "http://b2.test/chat/completions"]
    assert r.json()["choices"][0]["message"]["content"] == "one"  # first success passthrough


def test_invalid_backends_are_skipped(upstream):
    cfg = {"primary_backends": [{"name": "a", "url": "http://b1.test/v1", "model": "m"},
                                {"name": "b", "url": "", "model": "m"}],
           "settings": {"timeout": 30}}
    upstream.json("b1.test", completion("one"))
    c = make_client(cfg, upstream)
    r = c.post("/chat/completions", json={"messages": MSG}, headers=AUTH)
    assert r.status_code == 200 and len(upstream.calls) == 1


def test_no_valid_backend_500(upstream):
    cfg = {"primary_backends": [{"name": "a", "url": "", "model": "m"}], "settings": {"timeout": 3}}
    c = make_client(cfg, upstream)
    r = c.post("/chat/completions", json={"messages": MSG}, headers=AUTH)
    assert r.status_code == 500
    assert r.json()["error"] == {"message": "No valid backends configured", "type": "configuration_error"}


def test_timeout_passed_through(upstream):
    upstream.json("b1.test", completion("hi"))
    c = make_client(CFG_BLANK, upstream)
    c.post("/chat/completions", json={"model": "gpt-4", "messages": MSG}, headers=AUTH)
    t = upstream.calls[0]["timeout"]
    assert t == {"connect": 30.0, "read": 30.0, "write": 30.0, "pool": 30.0}


def test_invalid_json_body_500(upstream):
    c = make_client(CFG_BLANK, upstream)
    r = c.post("/chat/completions", content=b"{not json", headers=AUTH)
    assert r.status_code == 500
    assert r.json()["error"]["type"] == "proxy_error"
    assert r.json()["error"]["message"].startswith("Error processing request: ")


def test_upstream_exception_is_proxy_error(upstream):
    upstream.route("b1.test", lambda req, body: httpx.ConnectError("refused"))
    c = make_client(CFG_BLANK, upstream)
    r = c.post("/chat/completions", json={"model": "gpt-4", "messages": MSG}, headers=AUTH)
    assert r.status_code == 500
    assert r.json()["error"] == {"message": "All backends failed. First error: refused",
                                 "type": "proxy_error"}


def test_upstream_non_json_error(upstream):
    upstream.route("b1.test", lambda req, body: httpx.Response(503, text="overloaded"))
    c = make_client(CFG_BLANK, upstream)
    r = c.post("/chat/completions", json={"model": "gpt-4", "messages": MSG}, headers=AUTH)
    assert r.status_code == 500
    assert r.json()["error"]["message"] == "All backends failed. First error: overloaded"


def test_v1_alias(upstream):
    upstream.json("b1.test", completion("hi"))
    c = make_client(CFG_BLANK, upstream)
    r = c.post("/v1/chat/completions", json={"model": "gpt-4", "messages": MSG}, headers=AUTH)
    assert r.status_code == 200


# --- config -----------------------------------------------------------------

def test_load_config_roundtrip(tmp_path):
    cfg = {"primary_backends": [{"name": "LLM1", "url": "http://t/v1", "model": ""}],
           "settings": {"timeout": 45}}
    p = tmp_path / "c.yaml"
    p.write_text(yaml.dump(cfg))
    loaded = load_config(p)
    assert loaded == cfg and len(loaded) == 2


def test_load_config_default_fallback(tmp_path):
    loaded = load_config(tmp_path / "missing.yaml")
    assert loaded["settings"]["timeout"] == 60
    assert loaded["primary_backends"][0] == {"name": "default", "url": "https://api.openai.com/v1",
                                             "model": ""}


def test_env_config_path(tmp_path, monkeypatch):
    p = tmp_path / "x.yaml"
    p.write_text(yaml.dump({"primary_backends": [], "settings": {"timeout": 5}}))
    monkeypatch.setenv("QMX_CONFIG", str(p))
    assert load_config()["settings"]["timeout"] == 5


def test_openapi_component_schemas(upstream):
    """/openapi.json carries the request, completion, stream-chunk, usage and error schemas
    (the reference's vendored spec: CreateChatCompletionRequest, CreateChatCompletionStreamResponse,
    CompletionUsage — api_reference/chat_completions.yaml:1437, :398, :1968), referenced from
    both chat routes; the committed api_reference/openapi.json is that document."""
    import os

    c = make_client(CFG_BLANK, upstream)
    doc = c.get("/openapi.json").json()
    comps = doc["components"]["schemas"]
    for name in ("CreateChatCompletionRequest", "CreateChatCompletionResponse", "CreateChatCompletionStreamResponse",
                 "CompletionUsage", "ErrorResponse", "ChatMessage"):
        assert name in comps, name
    assert set(comps["CompletionUsage"]["required"]) == {"prompt_tokens", "completion_tokens", "total_tokens"}
    assert comps["CreateChatCompletionRequest"]["required"] == ["messages"]
    for path in ("/chat/completions", "/v1/chat/completions"):
        op = doc["paths"][path]["post"]
        assert op["requestBody"]["content"]["application/json"]["schema"]["$ref"].endswith(
            "/CreateChatCompletionRequest")
        ok = op["responses"]["200"]["content"]
        assert ok["text/event-stream"]["schema"]["$ref"].endswith("/CreateChatCompletionStreamResponse")
        for code in ("400", "401", "500"):
            assert op["responses"][code]["content"]["application/json"]["schema"]["$ref"].endswith("/ErrorResponse")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    committed = json.load(open(os.path.join(root, "api_reference", "openapi.json")))
    assert committed["components"]["schemas"] == comps
