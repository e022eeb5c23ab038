"""HTTP API: OpenAI-compatible ``/chat/completions`` (+ ``/v1`` alias), ``/health``, ``/metrics``.

Observable contract = quorum's: request validation, auth/header
normalisation, error table, SSE event shapes, non-streaming combine.  Reference:
``proxy_chat_completions`` (``src/quorum/oai_proxy.py:959-1408``), ``stream_with_role``
(``:888-956``), ``progress_streaming_aggregator`` (``:489-885``), ``health_check``
(``:1411-1414``).

Intentional, documented improvements (none is pinned by quorum's tests):
* streaming is incremental: upstream deltas are forwarded as they arrive (quorum buffers
  every upstream body and polls every 100 ms), so backends interleave instead of being
  emitted one whole backend at a time;
* one pooled upstream client instead of one ``AsyncClient`` (+SSL context) per call;
* bearer tokens are never logged; hop-by-hop / entity headers of upstream responses
  (content-length, transfer-encoding, content-encoding) are not copied onto re-framed
  bodies.
"""
from __future__ import annotations

import asyncio
import json
import logging
import os
import time
from typing import Any, Callable, Dict, List, Optional

from fastapi import FastAPI, Request, Response
from fastapi.responses import StreamingResponse

from ..models.strategies import combine_finals
from ..ops import reference as ref
from ..ops.engine import FinalizeRequest, make_engine
from ..utils import metrics
from ..utils.config import (RuntimeConfig, is_parallel, request_timeout, resolve_aggregate,
                            resolve_flags, valid_backends)
from .ticker import ticker_for
from .transport import UpstreamPool, call_backend, default_pool, error_message

logger = logging.getLogger("quorum_amd.server")

_DROP_RESP_HEADERS = {"content-length", "transfer-encoding", "content-encoding", "connection"}


def _json_error(message: str, etype: str, status: int) -> Response:
    return Response(content=json.dumps({"error": {"message": message, "type": etype}}),
                    status_code=status, media_type="application/json")


def normalize_headers(raw_items) -> Optional[Dict[str, str]]:
    """Forward everything but ``host``; auth fallback + normalisation; content-type default.

    Returns None when auth is missing and ``OPENAI_API_KEY`` is unset (→ 401).
    reference oai_proxy.py:972-1008."""
    headers = {k: v for k, v in raw_items if k.lower() != "host"}
    lower = {k.lower(): k for k in headers}
    if "authorization" not in lower:
        key = os.environ.get("OPENAI_API_KEY", "")
        if not key:
            return None
        headers["Authorization"] = f"Bearer {key}"
    elif "Authorization" not in headers:
        orig = lower["authorization"]
        headers["Authorization"] = headers.pop(orig)
    if "content-type" not in lower:
        headers["Content-Type"] = "application/json"
    return headers


class ProxyService:
    """Request handling with an injectable config provider / upstream pool / engine kind."""

    def __init__(self, config_provider: Callable[[], Dict[str, Any]],
                 pool: Optional[UpstreamPool] = None, runtime: Optional[RuntimeConfig] = None):
        self.config_provider = config_provider
        self.pool = pool
        self.runtime = runtime

    def _pool(self) -> UpstreamPool:
        return self.pool or default_pool()

    def _runtime(self, cfg) -> RuntimeConfig:
        return self.runtime or RuntimeConfig.from_config(cfg)

    # ------------------------------------------------------------------
    async def chat_completions(self, request: Request) -> Response:
        t0 = time.perf_counter()
        metrics.inc("qmx_requests_total")
        try:
            body = await request.body()
            json_body = json.loads(body)
            is_streaming = json_body.get("stream", False)
            headers = normalize_headers(request.headers.items())
            if headers is None:
                metrics.inc("qmx_errors_total", kind="auth")
                return _json_error("Authorization header is required and OPENAI_API_KEY "
                                   "environment variable is not set", "auth_error", 401)
            cfg = self.config_provider()
            backends = valid_backends(cfg)
            if not backends:
                return _json_error("No valid backends configured", "configuration_error", 500)
            if "model" not in json_body and not any(b.get("model") for b in backends):
                return _json_error("Model must be specified when config.yaml model is blank",
                                   "invalid_request_error", 400)
            parallel = is_parallel(cfg, len(backends))
            timeout = request_timeout(cfg)
            if is_streaming:
                if parallel:
                    flags = resolve_flags(cfg, json_body)
                    return StreamingResponse(
                        self.parallel_stream(cfg, backends, body, json_body, headers, timeout, flags, t0),
                        media_type="text/event-stream")
                return await self.single_stream(cfg, backends[0], body, json_body, headers, timeout)
            return await self.non_stream(cfg, backends, body, json_body, headers, timeout, parallel)
        except Exception as exc:  # noqa: BLE001 - reference :1395-1408
            logger.error("error in chat_completions: %s", exc)
            return _json_error(f"Error processing request: {exc}", "proxy_error", 500)
        finally:
            metrics.observe("request", time.perf_counter() - t0)

    # ------------------------------------------------------------------
    async def _pump(self, ticker, sess, slot, backend, body, headers, timeout, total_timeout):
        """One upstream stream → engine slot (incremental; no buffering)."""
        t0 = time.perf_counter()
        res = await call_backend(backend, body, headers, timeout, pool=self._pool(),
                                 total_timeout=total_timeout)
        if res.get("status_code") != 200 or not res.get("is_stream"):
            metrics.inc("qmx_upstream_failures_total", backend=str(backend.get("name")))
            sess.fail(slot)
            return
        stream = res["content"]
        try:
            async def _read():
                async for chunk in stream:
                    if chunk:
                        ticker.feed(slot, chunk)

            if total_timeout:
                await asyncio.wait_for(_read(), max(total_timeout - (time.perf_counter() - t0), 0.001))
            else:
                await _read()
            ticker.finish(slot)
        except asyncio.CancelledError:
            raise
        except Exception as exc:  # noqa: BLE001 - mid-stream failure: exclude from the final
            logger.warning("backend %s stream failed: %s", backend.get("name"), exc)
            metrics.inc("qmx_upstream_failures_total", backend=str(backend.get("name")))
            sess.fail(slot)
        finally:
            await stream.aclose()
            metrics.observe("upstream", time.perf_counter() - t0)

    async def parallel_stream(self, cfg, backends, body, json_body, headers, timeout, flags, t0):
        """Parallel SSE merge (reference progress_streaming_aggregator :489-885)."""
        created = int(time.time())
        yield ref.role_event(created)
        rt = self._runtime(cfg)
        engine = make_engine(rt.engine, flags.thinking_tags, device=rt.device)
        ticker = ticker_for(engine)
        sess = ticker.open_session(len(backends), bool(flags.hide_intermediate_think),
                                   not flags.suppress_individual_responses)
        tasks = [asyncio.create_task(self._pump(ticker, sess, slot, b, body, headers, timeout,
                                                rt.total_timeout))
                 for slot, b in zip(sess.slots, backends)]
        first = True
        try:
            while True:
                item = await sess.queue.get()
                if item is None:
                    break
                if first:
                    metrics.observe("ttft", time.perf_counter() - t0)
                    first = False
                yield item
            if not flags.skip_final_aggregation:
                agg = resolve_aggregate(cfg)
                joiner = "\n" + flags.separator
                good = sess.good_slots()
                if agg.aggregator_backend:
                    names, strip_answer = None, None
                    if agg.documented:
                        texts, names, strip_answer = await self._documented_sources(
                            ticker, sess, backends, good, agg, flags, rt)
                    else:
                        texts = await ticker.finalize(FinalizeRequest(good, bool(flags.hide_final_think), "texts"))
                    if texts:
                        combined = await combine_finals(texts, cfg, agg, json_body, headers, joiner,
                                                        pool=self._pool(), source_names=names,
                                                        strip_answer=strip_answer)
                        yield ref.final_event(int(time.time()), combined)
                    else:
                        yield ref.error_event(int(time.time()))
                else:
                    ev = await ticker.finalize(FinalizeRequest(
                        good, bool(flags.hide_final_think), "event", joiner, int(time.time())))
                    yield ev if ev is not None else ref.error_event(int(time.time()))
            yield ref.DONE
        finally:
            for t in tasks:
                if not t.done():
                    t.cancel()
            ticker.release(sess)

    @staticmethod
    async def _documented_sources(ticker, sess, backends, good, agg, flags, rt):
        """``semantics: documented`` aggregator inputs: the texts of the ``source_backends``
        among the good slots, stripped when ``strip_intermediate_thinking`` (or
        hide_final_think) is set, with their backends' names; one finalize per slot keeps each
        kept text paired with its backend (a slot with no content contributes nothing, as in
        the batched finalize)."""
        name_of = {slot: b.get("name") for slot, b in zip(sess.slots, backends)}
        src = agg.sources()
        if src is not None:
            good = [s for s in good if name_of[s] in src]
        strip = bool(flags.hide_final_think or agg.strip_intermediate_thinking)
        texts, names = [], []
        for slot in good:
            t = await ticker.finalize(FinalizeRequest([slot], strip, "texts"))
            if t:
                texts.append(t[0])
                names.append(name_of[slot])
        return texts, names, _answer_stripper(agg, rt, flags)

    # ------------------------------------------------------------------
    async def single_stream(self, cfg, backend, body, json_body, headers, timeout) -> Response:
        """Single-backend passthrough (reference :1094-1128 + stream_with_role :888-956)."""
        rt = self._runtime(cfg)
        res = await call_backend(backend, body, headers, timeout, pool=self._pool(),
                                 total_timeout=rt.total_timeout)
        if res["status_code"] == 200 and res.get("is_stream", False):
            model = json_body.get("model") or backend.get("model", "unknown")
            out_headers = {k: v for k, v in res["headers"].items() if k.lower() not in _DROP_RESP_HEADERS}
            return StreamingResponse(stream_with_role(res["content"], model), status_code=200,
                                     headers=out_headers, media_type="text/event-stream")
        return _json_error(f"Backend failed: {error_message(res)}", "proxy_error", res["status_code"])

    # ------------------------------------------------------------------
    async def non_stream(self, cfg, backends, body, json_body, headers, timeout, parallel) -> Response:
        rt = self._runtime(cfg)
        try:
            responses = await asyncio.gather(*[
                call_backend(b, body, headers, timeout, pool=self._pool(), total_timeout=rt.total_timeout)
                for b in backends])
            ok = [r for r in responses if r["status_code"] == 200]
            if not ok:
                return _json_error(f"All backends failed. First error: {error_message(responses[0])}",
                                   "proxy_error", 500)
            if parallel:
                names = [b.get("name") for b, r in zip(backends, responses) if r["status_code"] == 200]
                return await self._combine_non_stream(cfg, ok, json_body, headers, names)
            first = ok[0]
            ctype = first["headers"].get("content-type", "application/json")
            content = json.dumps(first["content"]) if isinstance(first["content"], (dict, list)) \
                else first["content"]
            resp = Response(content=content, status_code=200, media_type=ctype)
            for k, v in first["headers"].items():
                if k.lower() not in {"content-length", "content-type", "transfer-encoding",
                                     "content-encoding", "connection"}:
                    resp.headers[k] = v
            return resp
        except Exception as exc:  # noqa: BLE001 - reference :1381-1394
            return _json_error(f"Error processing request: {exc}", "proxy_error", 500)

    async def _combine_non_stream(self, cfg, ok, json_body, headers, names) -> Response:
        flags = resolve_flags(cfg, json_body)
        try:
            rt = self._runtime(cfg)
            stripper = _stripper(rt, flags.thinking_tags)
            agg = resolve_aggregate(cfg)
            doc = agg.documented
            strip = flags.hide_final_think or bool(doc and agg.aggregator_backend and agg.strip_intermediate_thinking)
            processed = [stripper(r["content"]["choices"][0]["message"]["content"], strip) for r in ok]
            src = agg.sources() if agg.aggregator_backend else None
            if src is not None:  # documented source_backends
                keep = [i for i, n in enumerate(names) if n in src]
                processed, names = [processed[i] for i in keep], [names[i] for i in keep]
                if not processed:
                    return _json_error("All source backends failed", "proxy_error", 500)
            if doc and flags.suppress_individual_responses and not agg.aggregator_backend:
                combined = processed[0]  # documented: "only the first response"
            else:
                combined = await combine_finals(processed, cfg, agg, json_body, headers, flags.separator,
                                                pool=self._pool(), source_names=names if doc else None,
                                                strip_answer=_answer_stripper(agg, rt, flags))
            usage = {k: sum(r["content"]["usage"][k] for r in ok)
                     for k in ("prompt_tokens", "completion_tokens", "total_tokens")}
            first = ok[0]["content"]
            out = {
                "id": first["id"],
                "object": "chat.completion",
                "created": first["created"],
                "model": first["model"],
                "system_fingerprint": first.get("system_fingerprint", ""),
                "choices": [{"index": 0, "message": {"role": "assistant", "content": combined},
                             "logprobs": None, "finish_reason": "stop"}],
                "usage": usage,
            }
            return Response(content=json.dumps(out), status_code=200, media_type="application/json")
        except Exception as exc:  # noqa: BLE001 - reference :1342-1355
            logger.error("error combining responses: %s", exc)
            return _json_error(f"Error combining responses: {exc}", "proxy_error", 500)


def _answer_stripper(agg, rt: RuntimeConfig, flags):
    """documented ``hide_aggregator_thinking``: the aggregator's answer loses its thinking."""
    if not (agg.documented and agg.hide_aggregator_thinking):
        return None
    strip = _stripper(rt, flags.thinking_tags)
    return lambda text: strip(text, True)


def _stripper(rt: RuntimeConfig, tags: List[str]):
    """Final strip for host-side texts: native when available, else the python oracle."""
    if rt.engine != "python":
        try:
            from ..ops import native
            if native.available():
                return native.strip_fn(tags)
        except Exception:  # noqa: BLE001
            pass
    return lambda text, on: ref.strip_thinking_tags(text, tags, hide_intermediate=on)


async def stream_with_role(upstream, model: str):
    """Own role event, drop a leading bare-role upstream event, forward the rest verbatim,
    append ``[DONE]`` if the upstream never sent it (reference :888-956)."""
    yield ref.role_event(int(time.time()), "chatcmpl-role", model)
    pending = b""
    decided = False
    saw_done = False
    tail = b""
    try:
        async for chunk in upstream:
            if not decided:
                pending += chunk
                j = pending.find(b"\n\n")
                if j < 0:
                    continue
                first, rest = pending[:j + 2], pending[j + 2:]
                decided = True
                if not _is_bare_role(first):
                    rest = first + rest
                chunk = rest
            if not chunk.strip():
                continue
            window = tail + chunk
            if b"data: [DONE]" in window:
                saw_done = True
            tail = window[-16:]
            yield chunk
        if not decided and pending.strip():
            if not _is_bare_role(pending):
                if b"data: [DONE]" in pending:
                    saw_done = True
                yield pending
    finally:
        await upstream.aclose()
    if not saw_done:
        yield ref.DONE


def _is_bare_role(event: bytes) -> bool:
    try:
        s = event.decode()
        if s.startswith("data: "):
            s = s[6:]
        data = json.loads(s)
        delta = data.get("choices", [{}])[0].get("delta", {})
        return bool(delta.get("role")) and delta.get("content", "") == ""
    except Exception:  # noqa: BLE001
        return False


def create_app(config_provider: Callable[[], Dict[str, Any]], pool: Optional[UpstreamPool] = None,
               runtime: Optional[RuntimeConfig] = None, title: str = "OpenAI API Proxy") -> FastAPI:
    app = FastAPI(title=title)
    svc = ProxyService(config_provider, pool=pool, runtime=runtime)
    app.state.service = svc

    @app.post("/chat/completions")
    async def chat_completions(request: Request) -> Response:
        return await svc.chat_completions(request)

    @app.post("/v1/chat/completions")
    async def chat_completions_v1(request: Request) -> Response:
        return await svc.chat_completions(request)

    @app.get("/health")
    async def health_check():
        return {"status": "healthy"}

    @app.get("/metrics")
    async def metrics_endpoint():
        return Response(content=metrics.render(), media_type="text/plain; version=0.0.4")

    from .schemas import install_openapi

    install_openapi(app)  # request / response / error component schemas in /openapi.json
    return app
