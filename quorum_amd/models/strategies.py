"""Merge strategies — the proxy's "model families".

* ``concatenate`` — join the per-backend finals with the separator
  (streaming: ``"\\n" + separator``; non-streaming: ``separator``; reference
  ``src/quorum/oai_proxy.py:834-841`` / ``:1279-1286``).
* ``aggregate``  — send every final to one aggregator backend for synthesis
  (reference ``aggregate_responses``, ``oai_proxy.py:374-486``); any failure falls back
  to ``intermediate_separator.join(sources)``.

Semantics kept from quorum: labels are ``LLM{i+1}`` by position among
the *successful* texts; ``source_backends`` is parsed but all valid backends are sources;
the aggregator is consulted whenever ``strategy.aggregate.aggregator_backend`` is set,
whatever strategy is selected; the aggregator's answer is returned as-is (no strip).
With ``semantics: documented`` (utils/config.py SEMANTICS) the flags of the reference's
docs/aggregate_behaviour.md apply instead: labels carry the backend's name, only
``source_backends`` feed the aggregator (callers filter), their texts are stripped with
``strip_intermediate_thinking`` (callers strip) and the answer with ``hide_aggregator_thinking``.
"""
from __future__ import annotations

import json
import logging
import os
from typing import Any, Callable, Dict, List, Optional

from ..server.transport import UpstreamPool, call_backend
from ..utils.logging_setup import log_content, redact
from ..utils.config import (DEFAULT_PROMPT_TEMPLATE, DEFAULT_QUERY_FORMAT,
                            DEFAULT_SOURCE_LABEL_FORMAT, AggregateSettings)

aggregation_logger = logging.getLogger("aggregation")


def first_user_message(json_body: Dict[str, Any]) -> Any:
    """reference oai_proxy.py:794-799."""
    if "messages" in json_body and json_body["messages"]:
        for msg in json_body["messages"]:
            if msg.get("role") == "user":
                return msg.get("content", "")
    return ""


def build_aggregator_prompt(source_responses: List[str], user_query: Any, separator: str,
                            include_original_query: bool, query_format: str,
                            include_source_names: bool, source_label_format: str,
                            prompt_template: str, source_names: Optional[List[str]] = None) -> str:
    """reference oai_proxy.py:406-423; ``source_names`` (documented mode) replaces the
    positional ``LLM{i+1}`` labels with the backends' names."""
    parts = []
    for i, text in enumerate(source_responses):
        if include_source_names:
            label = source_names[i] if source_names is not None else f"LLM{i + 1}"
            parts.append(source_label_format.format(backend_name=label) + text)
        else:
            parts.append(text)
    prompt = query_format.format(query=user_query) if include_original_query else ""
    return prompt + prompt_template.replace("{responses}", separator.join(parts))


def aggregator_headers(headers: Optional[Dict[str, str]]) -> Optional[Dict[str, str]]:
    """Only Authorization + Content-Type go to the aggregator (oai_proxy.py:436-466).
    Returns None when no credential is available (caller falls back to a plain join)."""
    clean: Dict[str, str] = {}
    if headers:
        if "Authorization" in headers:
            clean["Authorization"] = headers["Authorization"]
        elif "authorization" in headers:
            clean["Authorization"] = headers["authorization"]
        else:
            key = os.environ.get("OPENAI_API_KEY", "")
            if not key:
                return None
            clean["Authorization"] = f"Bearer {key}"
    else:
        key = os.environ.get("OPENAI_API_KEY", "")
        if not key:
            return None
        clean["Authorization"] = f"Bearer {key}"
    clean["Content-Type"] = "application/json"
    return clean


async def aggregate_responses(
    source_responses: List[str],
    aggregator_backend: Dict[str, str],
    user_query: str,
    separator: str,
    include_original_query: bool = True,
    query_format: str = DEFAULT_QUERY_FORMAT,
    include_source_names: bool = False,
    source_label_format: str = DEFAULT_SOURCE_LABEL_FORMAT,
    prompt_template: str = DEFAULT_PROMPT_TEMPLATE,
    headers: Optional[Dict[str, str]] = None,
    pool: Optional[UpstreamPool] = None,
    source_names: Optional[List[str]] = None,
    strip_answer: Optional[Callable[[str], str]] = None,
) -> str:
    """Synthesis call to the aggregator backend; plain join on any failure.

    Unlike quorum this never logs the Authorization header (oai_proxy.py:468 does).
    ``strip_answer`` (documented ``hide_aggregator_thinking``) applies to a string answer."""
    prompt = build_aggregator_prompt(source_responses, user_query, separator,
                                     include_original_query, query_format,
                                     include_source_names, source_label_format, prompt_template,
                                     source_names)
    clean = aggregator_headers(headers)
    if clean is None:
        aggregation_logger.error("no Authorization header or OPENAI_API_KEY for the aggregator")
        return separator.join(source_responses)
    body = {"model": aggregator_backend.get("model", ""),
            "messages": [{"role": "user", "content": prompt}], "stream": False}
    aggregation_logger.info("aggregator call to %s, headers %s", aggregator_backend.get("name"), redact(clean))
    if log_content():
        aggregation_logger.info("aggregator prompt: %s", prompt)
    try:
        res = await call_backend(aggregator_backend, json.dumps(body).encode(), clean, 60.0, pool=pool)
        if res["status_code"] == 200:
            out = res["content"]["choices"][0]["message"]["content"]
            if strip_answer is not None and isinstance(out, str):
                out = strip_answer(out)
            if log_content():
                aggregation_logger.info("aggregator result: %s", out)
            return out
        aggregation_logger.error("aggregator backend failed: status %s", res["status_code"])
    except Exception as exc:  # noqa: BLE001
        aggregation_logger.error("error calling aggregator backend: %s", exc)
    return separator.join(source_responses)


async def combine_finals(texts: List[str], cfg: Dict[str, Any], agg: AggregateSettings,
                         json_body: Dict[str, Any], headers: Dict[str, str], joiner: str,
                         pool: Optional[UpstreamPool] = None, source_names: Optional[List[str]] = None,
                         strip_answer: Optional[Callable[[str], str]] = None) -> str:
    """Final combine shared by stream (joiner = "\\n"+sep) and non-stream (joiner = sep)."""
    from ..utils.config import find_backend

    if agg.aggregator_backend:
        backend = find_backend(cfg, agg.aggregator_backend)
        if backend is None:
            aggregation_logger.error("aggregator backend %s not found", agg.aggregator_backend)
            return joiner.join(texts)
        try:
            return await aggregate_responses(
                texts, backend, first_user_message(json_body), agg.intermediate_separator,
                agg.include_original_query, agg.query_format, agg.include_source_names,
                agg.source_label_format, agg.prompt_template, headers, pool=pool,
                source_names=source_names, strip_answer=strip_answer)
        except Exception as exc:  # noqa: BLE001 - reference :832-834 / :1275-1279
            aggregation_logger.error("error during aggregation: %s", exc)
            return joiner.join(texts)
    return joiner.join(texts)
