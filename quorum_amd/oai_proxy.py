"""quorum-compatible module surface (drop-in for ``quorum.oai_proxy``).

Exposes the same names quorum's users and tests import ("Python-level
API"): ``config`` (module global, re-read on every request so monkeypatching works),
``app``, ``load_config``, ``ThinkingTagFilter``, ``strip_thinking_tags``,
``call_backend``, ``aggregate_responses``, ``stream_with_role``, ``health_check``.
Reference: ``src/quorum/oai_proxy.py`` (whole file).

Unlike quorum, importing this module does not write ``logs/aggregation.log``; call
:func:`quorum_amd.utils.logging_setup.enable_aggregation_log` to opt in.
"""
from __future__ import annotations

import logging

from .models.strategies import aggregate_responses  # noqa: F401
from .ops.reference import ThinkingTagFilter, strip_thinking_tags  # noqa: F401
from .server.app import create_app, stream_with_role  # noqa: F401
from .server.transport import call_backend  # noqa: F401
from .utils.config import load_config  # noqa: F401

logger = logging.getLogger(__name__)

config = load_config()


def _current_config():
    return globals()["config"]


app = create_app(_current_config)

TIMEOUT = (config.get("settings") or {}).get("timeout", 60) if isinstance(config, dict) else 60


async def health_check():
    return {"status": "healthy"}


if __name__ == "__main__":  # pragma: no cover
    import uvicorn

    uvicorn.run(app, host="0.0.0.0", port=8006)
