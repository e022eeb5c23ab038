"""qmx — an MI355X-native multi-backend LLM proxy/aggregator (quorum-compatible).

Public API (quorum parity, see ``quorum_amd.oai_proxy``): ``load_config``,
``ThinkingTagFilter``, ``strip_thinking_tags``, ``call_backend``, ``aggregate_responses``,
``create_app``.
"""
__version__ = "0.1.0"

from .ops.reference import ThinkingTagFilter, strip_thinking_tags  # noqa: E402,F401
from .utils.config import load_config  # noqa: E402,F401
