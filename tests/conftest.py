"""Shared fixtures: an in-process fake upstream (httpx.MockTransport) and app builders.

quorum's own suite monkeypatches ``httpx.AsyncClient.post`` (reference
``tests/conftest.py:184-249``); qmx uses a pooled streaming client, so upstreams are faked
at the transport layer instead — every request still goes through the real client,
header handling, body rewriting and incremental stream reading.
"""
from __future__ import annotations

import json
import os
import sys
from typing import Any, Callable, Dict, List, Optional

import httpx
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

from quorum_amd.server.app import create_app  # noqa: E402
from quorum_amd.server.transport import UpstreamPool  # noqa: E402
from quorum_amd.utils.config import RuntimeConfig  # noqa: E402

# engine used by the HTTP conformance tests (CI: python + cpu; GPU box: hip)
ENGINE = os.environ.get("QMX_TEST_ENGINE", "auto")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run via gpurun)")
    config.addinivalue_line("markers", "slow: long-running tests")


def completion(content: Any, cid: str = "cmpl-a", usage=(7, 11, 18), model: str = "mock-model",
               fingerprint: Optional[str] = "fp_qmx") -> Dict[str, Any]:
    out = {
        "id": cid,
        "object": "chat.completion",
        "created": 1700000000,
        "model": model,
        "choices": [{"index": 0, "message": {"role": "assistant", "content": content},
                     "logprobs": None, "finish_reason": "stop"}],
    }
    if fingerprint is not None:
        out["system_fingerprint"] = fingerprint
    if usage is not None:
        out["usage"] = {"prompt_tokens": usage[0], "completion_tokens": usage[1],
                        "total_tokens": usage[2]}
    return out


def sse_chunk(delta: Dict[str, Any], finish=None, cid="chunk-1") -> bytes:
    ev = {"id": cid, "object": "chat.completion.chunk", "created": 1700000000, "model": "m",
          "choices": [{"index": 0, "delta": delta, "finish_reason": finish}]}
    return f"data: {json.dumps(ev)}\n\n".encode()


def sse_stream(pieces: List[str], role: bool = True, done: bool = True) -> List[bytes]:
    out = []
    if role:
        out.append(sse_chunk({"role": "assistant", "content": ""}))
    for p in pieces:
        out.append(sse_chunk({"content": p}))
    out.append(sse_chunk({}, finish="stop"))
    if done:
        out.append(b"data: [DONE]\n\n")
    return out


class FakeUpstream:
    """Routes requests by host to per-backend behaviours; records every call."""

    def __init__(self):
        self.routes: Dict[str, Callable[[httpx.Request, Dict[str, Any]], httpx.Response]] = {}
        self.calls: List[Dict[str, Any]] = []

    def route(self, host: str, fn):
        self.routes[host] = fn

    def json(self, host: str, payload: Any, status: int = 200):
        self.routes[host] = lambda req, body: httpx.Response(status, json=payload)

    def stream(self, host: str, chunks: List[bytes], status: int = 200):
        def _fn(req, body):
            async def gen():
                for c in chunks:
                    yield c
            return httpx.Response(status, headers={"content-type": "text/event-stream"}, content=gen())
        self.routes[host] = _fn

    async def handler(self, request: httpx.Request) -> httpx.Response:
        raw = await request.aread()
        try:
            body = json.loads(raw)
        except Exception:  # noqa: BLE001
            body = None
        self.calls.append({"url": str(request.url), "host": request.url.host,
                           "headers": dict(request.headers), "raw": raw, "body": body,
                           "timeout": request.extensions.get("timeout")})
        fn = self.routes.get(request.url.host)
        if fn is None:
            return httpx.Response(500, json={"error": {"message": "Unknown backend",
                                                       "type": "backend_error"}})
        resp = fn(request, body)
        if isinstance(resp, Exception):
            raise resp
        return resp

    def pool(self) -> UpstreamPool:
        return UpstreamPool(transport_factory=lambda: httpx.MockTransport(self.handler))


def make_client(cfg_holder, upstream: FakeUpstream, engine: str = None):
    from fastapi.testclient import TestClient

    provider = cfg_holder if callable(cfg_holder) else (lambda: cfg_holder)
    app = create_app(provider, pool=upstream.pool(), runtime=RuntimeConfig(engine=engine or ENGINE))
    return TestClient(app)


def sse_lines(resp) -> List[str]:
    return [ln for ln in resp.iter_lines() if ln.strip()]


def sse_events(resp) -> List[Any]:
    out = []
    for ln in sse_lines(resp):
        assert ln.startswith("data: "), ln
        payload = ln[6:]
        out.append(payload if payload == "[DONE]" else json.loads(payload))
    return out


CFG_BLANK = {"primary_backends": [{"name": "LLM1", "url": "http://b1.test/v1", "model": ""}],
             "settings": {"timeout": 30}}
CFG_MODEL = {"primary_backends": [{"name": "LLM1", "url": "http://b1.test/v1", "model": "cfg-model"}],
             "settings": {"timeout": 30}}


def cfg_parallel(n=2, strategy="concatenate", block=None, agg=None, timeout=30):
    cfg = {
        "primary_backends": [{"name": f"LLM{i + 1}", "url": f"http://b{i + 1}.test/v1",
                              "model": f"model-{i + 1}"} for i in range(n)],
        "iterations": {"aggregation": {"strategy": strategy}},
        "strategy": {},
        "settings": {"timeout": timeout},
    }
    if block is not None:
        cfg["strategy"][strategy] = block
    if agg is not None:
        cfg["strategy"]["aggregate"] = agg
    return cfg


@pytest.fixture
def upstream():
    return FakeUpstream()


@pytest.fixture(autouse=True)
def _no_env_key(monkeypatch):
    monkeypatch.delenv("OPENAI_API_KEY", raising=False)
