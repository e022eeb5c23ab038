"""Upstream transport: pooled, incremental HTTP to the LLM backends.

Reference ``call_backend`` (``src/quorum/oai_proxy.py:142-259``) builds a NEW
``httpx.AsyncClient`` per call (≈50 ms of SSL-context CPU each, 58 % of the reference's
wall time — SURVEY §0) and buffers the whole streamed body before returning.  Here one
long-lived pooled client per event loop is reused for every call, and streamed bodies
are returned as an *incremental* async byte iterator.

``call_backend`` keeps the reference's result contract exactly:
``{backend_name, status_code, headers?, content, is_stream}`` and never raises.
"""
from __future__ import annotations

import asyncio
import json
import logging
from typing import Any, AsyncIterator, Callable, Dict, Optional

import httpx

logger = logging.getLogger("quorum_amd.transport")

# headers that must not be forwarded verbatim once the body is re-framed
_HOP_BY_HOP = {"transfer-encoding", "connection", "keep-alive", "upgrade", "te", "trailer"}


class UpstreamStream:
    """Incremental view of a streamed upstream response (async-iterable of bytes)."""

    def __init__(self, response: httpx.Response):
        self.response = response
        self._it: Optional[AsyncIterator[bytes]] = None

    def aiter_bytes(self) -> AsyncIterator[bytes]:
        return self.response.aiter_bytes()

    def __aiter__(self):
        self._it = self.response.aiter_bytes()
        return self

    async def __anext__(self) -> bytes:
        if self._it is None:
            self._it = self.response.aiter_bytes()
        return await self._it.__anext__()

    async def aclose(self) -> None:
        await self.response.aclose()


class UpstreamPool:
    """One pooled AsyncClient per running event loop (TestClient portals use their own)."""

    def __init__(self, transport_factory: Optional[Callable[[], httpx.AsyncBaseTransport]] = None,
                 max_connections: int = 4096):
        self.transport_factory = transport_factory
        self.max_connections = max_connections
        self._clients: Dict[int, httpx.AsyncClient] = {}

    def client(self) -> httpx.AsyncClient:
        loop = asyncio.get_running_loop()
        key = id(loop)
        cl = self._clients.get(key)
        if cl is None or cl.is_closed:
            kwargs: Dict[str, Any] = dict(
                limits=httpx.Limits(max_connections=self.max_connections,
                                    max_keepalive_connections=self.max_connections),
                timeout=None,
            )
            if self.transport_factory is not None:
                kwargs["transport"] = self.transport_factory()
            cl = httpx.AsyncClient(**kwargs)
            self._clients[key] = cl
        return cl

    async def aclose(self) -> None:
        loop = asyncio.get_running_loop()
        cl = self._clients.pop(id(loop), None)
        if cl is not None:
            await cl.aclose()


_DEFAULT_POOL = UpstreamPool()


def default_pool() -> UpstreamPool:
    return _DEFAULT_POOL


def _error(name: str, status: int, message: str, etype: str, headers=None) -> Dict[str, Any]:
    res = {
        "backend_name": name,
        "status_code": status,
        "content": {"error": {"message": message, "type": etype}},
        "is_stream": False,
    }
    if headers is not None:
        res["headers"] = headers
    return res


def prepare_body(backend: Dict[str, Any], body: bytes):
    """Model override + content-length fixup (reference oai_proxy.py:157-180).

    Returns (json_body, body_bytes) or raises (caller maps to proxy_error); returns
    (json_body, None) when no model is available anywhere (synthetic 400)."""
    json_body = json.loads(body)
    if backend["model"]:
        json_body["model"] = backend["model"]
        body = json.dumps(json_body).encode()
    elif "model" not in json_body:
        return json_body, None
    return json_body, body


async def call_backend(backend: Dict[str, Any], body: bytes, headers: Dict[str, str],
                       timeout: float, pool: Optional[UpstreamPool] = None,
                       total_timeout: Optional[float] = None) -> Dict[str, Any]:
    """POST ``{url}/chat/completions``; classify the result; never raise."""
    name = backend.get("name")
    pool = pool or _DEFAULT_POOL
    try:
        json_body, out_body = prepare_body(backend, body)
        if out_body is None:
            return _error(name, 400, "No model specified in config.yaml or request",
                          "invalid_request_error")
        fwd = {k: v for k, v in headers.items() if k.lower() not in _HOP_BY_HOP}
        fwd["content-length"] = str(len(out_body))
        url = f"{backend['url']}/chat/completions"
        client = pool.client()
        req = client.build_request("POST", url, content=out_body, headers=fwd,
                                   timeout=httpx.Timeout(timeout))
        streaming = bool(json_body.get("stream", False))

        async def _send():
            return await client.send(req, stream=True)

        resp = await (asyncio.wait_for(_send(), total_timeout) if total_timeout else _send())
        rheaders = dict(resp.headers)
        if resp.status_code == 200 and streaming:
            return {"backend_name": name, "status_code": 200, "headers": rheaders,
                    "content": UpstreamStream(resp), "is_stream": True}
        try:
            raw = await (asyncio.wait_for(resp.aread(), total_timeout) if total_timeout else resp.aread())
        finally:
            await resp.aclose()
        text = raw.decode()
        if resp.status_code == 200:
            try:
                content = json.loads(text)
                if isinstance(content, dict):
                    content["backend"] = name
                return {"backend_name": name, "status_code": 200, "headers": rheaders,
                        "content": content, "is_stream": False}
            except json.JSONDecodeError:
                return {"backend_name": name, "status_code": 200, "headers": rheaders,
                        "content": text, "is_stream": False}
        try:
            err = json.loads(text)
        except json.JSONDecodeError:
            err = {"error": {"message": text, "type": "backend_error"}}
        return {"backend_name": name, "status_code": resp.status_code, "headers": rheaders,
                "content": err, "is_stream": False}
    except Exception as exc:  # noqa: BLE001 - reference: every failure becomes a 500 dict
        logger.warning("error calling backend %s: %s", name, exc)
        return _error(name, 500, str(exc), "proxy_error")


def error_message(result: Dict[str, Any]) -> str:
    """reference oai_proxy.py:1108-1116 / 1142-1150."""
    content = result.get("content", {})
    if isinstance(content, dict) and "error" in content:
        err = content["error"]
        return err.get("message", "Unknown error") if isinstance(err, dict) else str(err)
    return str(content)
