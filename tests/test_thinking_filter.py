"""Streaming think-tag filter semantics.

Behaviours of quorum's ``tests/test_thinking_tag_filter.py`` (9 cases) plus the survey's
probe rows, run against every filter implementation available: the python oracle and,
when built, the native C++ streaming filter (``_qmx.StreamFilter``).
"""
import pytest

from quorum_amd.ops.reference import ThinkingTagFilter
from quorum_amd.ops import native

DEFAULT = ["think", "reason", "reasoning", "thought"]


def _impls():
    impls = [("python", ThinkingTagFilter)]
    if native.available():
        ext = native.require()

        class NativeFilter:
            def __init__(self, tags):
                self._f = ext.StreamFilter([t.lower() for t in tags])

            def feed(self, text):
                return self._f.feed(text.encode("utf-8", "surrogatepass")).decode("utf-8", "surrogatepass")

            def flush(self):
                return self._f.flush().decode("utf-8", "surrogatepass")

        impls.append(("native", NativeFilter))
    return impls


@pytest.fixture(params=_impls(), ids=lambda p: p[0])
def F(request):
    return request.param[1]


def test_basic(F):
    assert F(DEFAULT).feed("Hello <think>secret</think> World") == "Hello  World"
    assert F(DEFAULT).feed("A <think>b1</think> B <think>b2</think> C") == "A  B  C"


def test_split_tags(F):
    f = F(["think"])
    assert f.feed("Hello <thi") == "Hello "
    assert f.feed("nk>secret</th") == ""
    assert f.feed("ink> World") == " World"


def test_nested(F):
    assert F(["think", "reason"]).feed("A <think>x <think>y</think> z</think> D") == "A  D"
    assert F(["think", "reason"]).feed("X <think>h <reason>i</reason> w</think> Y") == "X  Y"


def test_incomplete(F):
    f = F(["think"])
    assert f.feed("Hello <think>not closed") == "Hello "
    assert f.flush() == ""
    f = F(["think"])
    assert f.feed("Test <think>secret</nope> End") == "Test "
    assert f.flush() == ""


def test_case_insensitive(F):
    assert F(["think"]).feed("Hello <THINK>S</THINK> World") == "Hello  World"
    assert F(["think"]).feed("Hello <ThInK>S</tHiNk> World") == "Hello  World"


def test_flush(F):
    f = F(["think"])
    assert f.feed("No tags here.") == "No tags here."
    assert f.flush() == ""
    f = F(["think"])
    assert f.feed("Partial open <think") == "Partial open "
    assert f.flush() == ""


def test_streaming_simulation(F):
    f = F(["think"])
    assert f.feed("Stream start <thin") == "Stream start "
    assert f.feed("k>secret mess") == ""
    assert f.feed("age</think> and then safe") == " and then safe"


def test_multiple_tag_types(F):
    assert F(["think", "reason"]).feed("Hello <think>s</think> world <reason>i</reason> done") == \
        "Hello  world  done"


def test_newlines(F):
    assert F(["think"]).feed("Line1\n<think>a\nb</think>\nLine2") == "Line1\n\nLine2"
    f = F(["think"])
    assert f.feed("Hello <thin") == "Hello "
    assert f.feed("k>\nsecret\n") == ""
    assert f.feed("content</think>\nWorld") == "\nWorld"


# --- survey probe rows (§2.7-A) ------------------------------------------------

def test_close_at_depth_zero_is_literal(F):
    assert F(DEFAULT).feed("x </think> y") == "x </think> y"


def test_cross_type_close(F):
    assert F(["think", "reason"]).feed("<think>a</reason>b") == "b"
    f = F(["think"])
    assert f.feed("<think>a</reason>b") == ""
    assert f.flush() == ""


def test_lone_trailing_lt_dropped_at_flush(F):
    f = F(DEFAULT)
    assert f.feed(" c <") == " c "
    assert f.flush() == ""


def test_holdback_released_when_not_a_tag(F):
    f = F(["think"])
    assert f.feed("x <t") == "x "
    assert f.feed("able>") == "<table>"


def test_attributes_are_literal(F):
    assert F(["think"]).feed("<think attr='1'>x") == "<think attr='1'>x"


def test_holdback_only_last_lt(F):
    f = F(["think"])
    assert f.feed("a <th <thi") == "a <th "
    assert f.feed("nk>zz</think>q") == "q"


def test_non_ascii_passthrough(F):
    f = F(["think"])
    assert f.feed("héllo <think>ü</think>wörld 😀") == "héllo wörld 😀"
