"""OpenAPI component schemas of the proxy's surface (documentation only).

The proxy forwards request bodies opaquely and builds its own responses byte for byte
(SURVEY §2.6), so nothing here validates traffic.  These models describe what a client
sends and receives, in the shape of the OpenAI spec subset the reference vendors
(``api_reference/chat_completions.yaml``: ``CreateChatCompletionRequest`` at :1437,
``CreateChatCompletionStreamResponse`` at :398, ``CompletionUsage`` at :1968), narrowed
to the fields quorum reads or writes (``oai_proxy.py:959-1408``), and are published under
``components.schemas`` of the served ``/openapi.json`` (:func:`install_openapi`).
"""
from __future__ import annotations

from typing import Any, Dict, List, Literal, Optional, Union

from pydantic import BaseModel, ConfigDict, Field


class ChatMessage(BaseModel):
    """One message of ``messages``; the first ``user`` message is the aggregator's
    "original query" (``oai_proxy.py:795-799``)."""
    model_config = ConfigDict(extra="allow")
    role: str = Field(..., description="system | user | assistant | tool")
    content: Optional[Union[str, List[Dict[str, Any]]]] = None
    name: Optional[str] = None


class CreateChatCompletionRequest(BaseModel):
    """``POST /chat/completions`` body.  Fields the proxy reads are listed; every other
    field (temperature, max_tokens, tools, ...) is forwarded to each backend untouched."""
    model_config = ConfigDict(extra="allow")
    model: Optional[str] = Field(None, description="Overridden by a backend's configured `model`; required when "
                                                   "every configured model is blank (400 otherwise)")
    messages: List[ChatMessage]
    stream: bool = Field(False, description="true: text/event-stream of chat.completion.chunk events")
    suppress_individual_responses: Optional[bool] = Field(
        None, description="Overrides the strategy's flag (streaming: no per-backend events); also forwarded upstream")


class CompletionUsage(BaseModel):
    """Token counts; the parallel non-streaming response sums them over the successful
    source backends (the aggregator call excluded)."""
    prompt_tokens: int
    completion_tokens: int
    total_tokens: int


class ChatCompletionResponseMessage(BaseModel):
    role: Literal["assistant"] = "assistant"
    content: Optional[str] = None


class ChatCompletionChoice(BaseModel):
    index: int = 0
    message: ChatCompletionResponseMessage
    logprobs: Optional[Any] = None
    finish_reason: Optional[str] = Field(None, description="`stop` for the combined parallel answer")


class CreateChatCompletionResponse(BaseModel):
    """Non-streaming response.  Parallel mode: `id`, `created`, `model`,
    `system_fingerprint` of the first successful backend, the combined content, summed usage.
    Single backend: the upstream JSON passed through plus `"backend": <name>`."""
    model_config = ConfigDict(extra="allow")
    id: str
    object: Literal["chat.completion"] = "chat.completion"
    created: int
    model: str
    system_fingerprint: Optional[str] = None
    choices: List[ChatCompletionChoice]
    usage: Optional[CompletionUsage] = None
    backend: Optional[str] = Field(None, description="single-backend passthrough: the backend's name")


class ChatCompletionStreamDelta(BaseModel):
    role: Optional[Literal["assistant"]] = None
    content: Optional[str] = None


class ChatCompletionStreamChoice(BaseModel):
    index: int = 0
    delta: ChatCompletionStreamDelta
    finish_reason: Optional[str] = Field(None, description="null, `stop` (final event) or `error` (all failed)")


class CreateChatCompletionStreamResponse(BaseModel):
    """One ``data: <json>`` event of a parallel stream (``json.dumps`` spacing,
    ``ensure_ascii``): id `chatcmpl-parallel` (role), `chatcmpl-parallel-{i}` (backend i's
    filtered delta), `chatcmpl-parallel-final` (combined answer, unless
    skip_final_aggregation), `error` (every backend failed); the stream ends with
    ``data: [DONE]``.  Single-backend streams forward the upstream events after a
    `chatcmpl-role` role event."""
    id: str = Field(..., examples=["chatcmpl-parallel-0"])
    object: Literal["chat.completion.chunk"] = "chat.completion.chunk"
    created: int
    model: str = Field(..., examples=["parallel-proxy"])
    choices: List[ChatCompletionStreamChoice]


class ErrorDetail(BaseModel):
    message: str
    type: str = Field(..., description="auth_error | configuration_error | invalid_request_error | proxy_error | "
                                       "backend_error")
    param: Optional[str] = None
    code: Optional[str] = None


class ErrorResponse(BaseModel):
    """Every error the proxy produces itself (SURVEY §2.6 error table: 400 / 401 / 500, and
    upstream status codes passed through)."""
    error: ErrorDetail


class HealthResponse(BaseModel):
    status: Literal["healthy"] = "healthy"


SCHEMAS = (CreateChatCompletionRequest, CreateChatCompletionResponse, CreateChatCompletionStreamResponse,
           CompletionUsage, ErrorResponse, HealthResponse)


def _ref(name: str) -> Dict[str, str]:
    return {"$ref": f"#/components/schemas/{name}"}


def install_openapi(app) -> None:
    """Publish the component schemas and reference them from the chat routes' request and
    responses in ``app.openapi()`` (what both front ends serve at ``/openapi.json``)."""
    from fastapi.openapi.utils import get_openapi

    def openapi():
        if app.openapi_schema:
            return app.openapi_schema
        doc = get_openapi(title=app.title, version=app.version, routes=app.routes)
        comps = doc.setdefault("components", {}).setdefault("schemas", {})
        for model in SCHEMAS:
            js = model.model_json_schema(ref_template="#/components/schemas/{model}")
            for name, d in js.pop("$defs", {}).items():
                comps[name] = d
            comps[model.__name__] = js
        errors = {"content": {"application/json": {"schema": _ref("ErrorResponse")}}}
        for path in ("/chat/completions", "/v1/chat/completions"):
            op = doc.get("paths", {}).get(path, {}).get("post")
            if op is None:
                continue
            op["requestBody"] = {"required": True, "content": {
                "application/json": {"schema": _ref("CreateChatCompletionRequest")}}}
            op["responses"] = {
                "200": {"description": "stream=false: the completion; stream=true: chat.completion.chunk events",
                        "content": {"application/json": {"schema": _ref("CreateChatCompletionResponse")},
                                    "text/event-stream": {"schema": _ref("CreateChatCompletionStreamResponse")}}},
                "400": dict(errors, description="no model in the request or the config"),
                "401": dict(errors, description="no Authorization header and no OPENAI_API_KEY"),
                "500": dict(errors, description="no valid backend, every backend failed, or a proxy error"),
            }
        health = doc.get("paths", {}).get("/health", {}).get("get")
        if health is not None:
            health["responses"]["200"]["content"]["application/json"]["schema"] = _ref("HealthResponse")
        app.openapi_schema = doc
        return doc

    app.openapi = openapi
