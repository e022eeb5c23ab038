"""GPU: the FastAPI front-end (server/app.py + ticker) driving the CDNA4 HIP engine.

Re-runs the streaming and strategy API suites (reference re-expressions) with the python
app's engine forced to ``hip``: every stream of these tests goes through the tick kernel
and every final through the finalize kernel.
"""
import pytest

import conftest
from test_streaming_api import *  # noqa: F401,F403  (re-collected here with the gpu mark)
from test_strategies_api import *  # noqa: F401,F403

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _hip_engine(monkeypatch):
    monkeypatch.setattr(conftest, "ENGINE", "hip")
