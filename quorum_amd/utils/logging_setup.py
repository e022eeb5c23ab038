"""Logging bootstrap (reference ``src/quorum/oai_proxy.py:13-37``).

quorum calls ``basicConfig(INFO)`` and, at import time, attaches a FileHandler for the
``aggregation`` logger at ``<repo>/logs/aggregation.log`` and writes a test line.  Its INFO
logs carry request bodies, prompts, per-backend content and even the aggregator's bearer
token (``oai_proxy.py:468``).  qmx keeps the logger names with three differences:

* nothing is written at import: :func:`enable_aggregation_log` attaches the file handler on
  demand (``QMX_AGGREGATION_LOG=<path>`` does it when a worker starts);
* content (prompts, per-backend finals, the combined answer) is logged only when
  :func:`set_log_content` turned it on, because it is user data;
* credentials are never logged: :func:`redact` masks Authorization-like headers.
"""
from __future__ import annotations

import logging
import os
from pathlib import Path
from typing import Dict, Mapping, Optional

AGGREGATION = "aggregation"
_SECRET_HEADERS = ("authorization", "proxy-authorization", "x-api-key", "api-key", "cookie")
_content_enabled = False


def configure_logging(level: int = logging.WARNING) -> None:
    """Root logging for a worker (quorum: INFO at import; qmx: WARNING unless asked)."""
    logging.basicConfig(level=level, format="%(asctime)s %(name)s %(levelname)s %(message)s")


def default_log_path() -> Path:
    return Path(__file__).resolve().parents[2] / "logs" / "aggregation.log"


def enable_aggregation_log(path: Optional[os.PathLike] = None) -> Path:
    """Attach (once per path) an append-mode FileHandler to the ``aggregation`` logger.
    Default path: ``<repo>/logs/aggregation.log``, as in quorum (``oai_proxy.py:20-29``)."""
    p = (Path(path) if path else default_log_path()).resolve()
    p.parent.mkdir(parents=True, exist_ok=True)
    log = logging.getLogger(AGGREGATION)
    for h in log.handlers:
        if isinstance(h, logging.FileHandler) and Path(h.baseFilename) == p:
            return p
    h = logging.FileHandler(p, mode="a", encoding="utf-8")
    h.setFormatter(logging.Formatter("%(asctime)s - %(name)s - %(levelname)s - %(message)s"))
    log.addHandler(h)
    log.setLevel(logging.INFO)
    return p


def set_log_content(on: bool) -> None:
    global _content_enabled
    _content_enabled = bool(on)


def log_content() -> bool:
    """Whether prompts / responses may be logged."""
    return _content_enabled


def redact(headers: Optional[Mapping[str, str]]) -> Dict[str, str]:
    """A copy of ``headers`` that is safe to log: credential values masked."""
    return {k: ("<redacted>" if k.lower() in _SECRET_HEADERS else v) for k, v in (headers or {}).items()}


def from_env(env: Optional[Mapping[str, str]] = None) -> Optional[Path]:
    """Worker start: ``QMX_AGGREGATION_LOG`` (a path, or ``1`` for the default path) opts
    into the aggregation file log; ``QMX_LOG_CONTENT=1`` allows content in it."""
    e = os.environ if env is None else env
    set_log_content(e.get("QMX_LOG_CONTENT", "") in ("1", "true", "yes"))
    path = e.get("QMX_AGGREGATION_LOG")
    if not path:
        return None
    return enable_aggregation_log(None if path in ("1", "default") else path)
