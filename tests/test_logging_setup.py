"""Logging bootstrap: opt-in aggregation file log, no credentials in it."""
import asyncio
import logging

import pytest

from quorum_amd.models import strategies
from quorum_amd.utils import logging_setup as ls


@pytest.fixture
def agg_log(tmp_path):
    log = logging.getLogger(ls.AGGREGATION)
    before = list(log.handlers)
    p = ls.enable_aggregation_log(tmp_path / "logs" / "aggregation.log")
    yield p
    for h in list(log.handlers):
        if h not in before:
            log.removeHandler(h)
            h.close()
    ls.set_log_content(False)


def test_off_by_default():
    # unlike quorum (oai_proxy.py:20-37) no file handler is attached unless asked for
    assert ls.from_env({}) is None and not ls.log_content()
    assert ls.default_log_path().name == "aggregation.log"


def test_enable_is_idempotent(agg_log):
    log = logging.getLogger(ls.AGGREGATION)
    n = len(log.handlers)
    assert ls.enable_aggregation_log(agg_log) == agg_log
    assert len(log.handlers) == n
    assert agg_log.parent.is_dir()


def test_redact_masks_credentials():
    h = ls.redact({"Authorization": "Bearer sk-secret", "Content-Type": "application/json", "x-api-key": "k"})
    assert h == {"Authorization": "<redacted>", "Content-Type": "application/json", "x-api-key": "<redacted>"}


def test_from_env(tmp_path):
    log = logging.getLogger(ls.AGGREGATION)
    before = list(log.handlers)
    try:
        p = ls.from_env({"QMX_AGGREGATION_LOG": str(tmp_path / "a.log"), "QMX_LOG_CONTENT": "1"})
        assert p == (tmp_path / "a.log").resolve() and ls.log_content()
    finally:
        for h in list(log.handlers):
            if h not in before:
                log.removeHandler(h)
                h.close()
        ls.set_log_content(False)


@pytest.mark.parametrize("content", [False, True])
def test_aggregator_call_logged_without_token(agg_log, monkeypatch, content):
    async def fake_call(backend, body, headers, timeout, pool=None):
        return {"status_code": 200, "content": {"choices": [{"message": {"content": "SYNTH"}}]}}

    monkeypatch.setattr(strategies, "call_backend", fake_call)
    ls.set_log_content(content)
    out = asyncio.run(strategies.aggregate_responses(
        ["alpha", "beta"], {"name": "agg", "url": "http://x", "model": "m"}, "Q?", "\n---\n",
        headers={"Authorization": "Bearer sk-secret-token"}))
    assert out == "SYNTH"
    for h in logging.getLogger(ls.AGGREGATION).handlers:
        h.flush()
    text = agg_log.read_text()
    assert "aggregator call to agg" in text
    assert "sk-secret-token" not in text
    assert ("SYNTH" in text) == content and ("alpha" in text) == content
